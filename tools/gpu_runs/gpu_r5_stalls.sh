#!/bin/bash
# Round 5: stall counters of TraceCullKernel in the headline launch shape (8 frames per launch, the
# largest grid), plus a kernel trace of the same bench command whose 8-frame dispatches give the
# roofline's rocprof mean (tools/trace_shapes.py), and the two HBM traffic passes again.
source "$(dirname "$0")/gpu_lib.sh"
B="python3 bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0"
K="--kernel-include-regex TraceCullKernel"
run list 60 rocprofv3 -L
run l8_trace 200 timeout -s KILL 190 rocprofv3 --kernel-trace --stats -d gpurun_out/l8_trace -o run --output-format csv -- $B
run l8_stallA 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS $K -d gpurun_out/l8_stallA -o run --output-format csv -- $B
run l8_stallB 150 timeout -s KILL 140 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SMEM SQ_BUSY_CYCLES $K -d gpurun_out/l8_stallB -o run --output-format csv -- $B
run l8_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE $K -d gpurun_out/l8_fetch -o run --output-format csv -- $B
run l8_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE $K -d gpurun_out/l8_write -o run --output-format csv -- $B
echo done
