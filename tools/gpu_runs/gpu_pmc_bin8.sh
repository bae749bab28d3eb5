#!/bin/bash
# SQ counters and kernel times of PrepareBinKernel on a P = 8 share rank (rank simulation, one
# queue): is the replicated record pass VALU-, memory- or latency-bound?
source "$(dirname "$0")/gpu_lib.sh"
R="python3 tools/rank_sim.py --ranks 8 --queues 1 --steps 4 --warmup 2"
run b8_trace 200 rocprofv3 --kernel-trace --stats -d gpurun_out/b8_trace -o run --output-format csv -- $R
run b8_sq 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex PrepareBinKernel -d gpurun_out/b8_sq -o run --output-format csv -- $R
