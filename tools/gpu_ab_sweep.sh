#!/bin/bash
# GPU tests, then an A/B of library builds (LIBS) and the bin kernel's SQ counters of the product.
LIBS="${LIBS:-base prev}" bash tools/gpu_ab_check.sh || exit $?
source "$(dirname "$0")/gpu_lib.sh"
run pmcC 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD --kernel-include-regex PrepareBinKernel -d gpurun_out/pmcC -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --queues 1 --batch 1 --no-extras --no-cpu-baseline
