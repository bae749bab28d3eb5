#!/bin/bash
# GPU tests, then an A/B of library builds (LIBS) and one SQ counter pass of the product ($PMC:
# "lds" = the trace kernel's LDS counters, else the bin kernel's wave-cycle split).
LIBS="${LIBS:-base prev}" bash tools/gpu_runs/gpu_ab_check.sh || exit $?
source "$(dirname "$0")/gpu_lib.sh"
Q="--steps 50 --warmup 5 --queues 1 --batch 1 --no-extras --no-cpu-baseline"
if [ "${PMC:-bin}" = lds ]; then
    run pmcA 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-include-regex TraceCullKernel -d gpurun_out/pmcA -o run --output-format csv -- python3 bench.py $Q
else
    run pmcC 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD --kernel-include-regex PrepareBinKernel -d gpurun_out/pmcC -o run --output-format csv -- python3 bench.py $Q
fi
