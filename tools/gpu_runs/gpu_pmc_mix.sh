#!/bin/bash
# Instruction mix and stall counters (one frame per dispatch, one --pmc pass each): the trace
# kernel's LDS / SALU / VMEM / atomic mix (pmcA, pmcB) and the bin kernel's wave-cycle split (pmcC).
source "$(dirname "$0")/gpu_lib.sh"
Q="--steps 50 --warmup 5 --queues 1 --batch 1 --no-extras --no-cpu-baseline"
run pmcA 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-include-regex TraceCullKernel -d gpurun_out/pmcA -o run --output-format csv -- python3 bench.py $Q
run pmcB 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS_ATOMIC SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex TraceCullKernel -d gpurun_out/pmcB -o run --output-format csv -- python3 bench.py $Q
run pmcC 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD --kernel-include-regex PrepareBinKernel -d gpurun_out/pmcC -o run --output-format csv -- python3 bench.py $Q
echo done
