#!/bin/bash
# Round-2 starting point: driver-shaped bench line, random-offset leg, rocprof of both.
source "$(dirname "$0")/gpu_lib.sh"
Q=(--no-cpu-baseline --no-e2e --brute-steps 0)
run bench_driver 300 python bench.py --steps 20 --warmup 5 "${Q[@]}"
run bench_uniform 300 python bench.py --steps 3000 --warmup 20 "${Q[@]}"
run bench_random 300 python bench.py --steps 1000 --warmup 20 --offsets random "${Q[@]}"
run prof_random 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_random -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --offsets random --queues 1 "${Q[@]}"
run prof_uniform 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_uniform -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --queues 1 "${Q[@]}"
echo done
