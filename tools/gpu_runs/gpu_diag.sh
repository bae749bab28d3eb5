#!/bin/bash
# Diag-build timelines of the cull trace (uniform and random offsets) + a quick bench line.
source "$(dirname "$0")/gpu_lib.sh"
export SRT_LIB=simpleraytracer_amd/lib_diag/libModelRunner.so
run diag_uniform 120 python tools/diag_cull.py
OFFSETS=random run diag_random 120 python tools/diag_cull.py
unset SRT_LIB
run bench_uniform 300 python bench.py --steps 3000 --warmup 20 --no-cpu-baseline --no-e2e --brute-steps 0
run prof_uniform 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_uniform -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --queues 1 --no-cpu-baseline --no-e2e --brute-steps 0
echo done
