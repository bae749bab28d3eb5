#!/bin/bash
# Table upload by kernel + per-shape cull arenas + per-frame share: GPU tests, the fake-device
# rehearsals (2, 4, 8), and an A/B of the default bench line against lib_ab/head.
source "$(dirname "$0")/gpu_lib.sh"
run up_tests 600 python -u -m pytest tests/ -m gpu -q -x --timeout 200 --timeout-method thread
for n in 2 4 8; do
    SRT_BENCH_ONE_DEVICE=1 run up_rehearse$n 400 python bench.py --gpus $n --steps 20 --warmup 2 --no-e2e --frames-per-step 64
    grep -o '"verified": [a-z]*' gpurun_out/up_rehearse$n.log | head -1
done
VARIANTS="head product" REPS=2 bash "$(dirname "$0")/gpu_ab_variants.sh"
