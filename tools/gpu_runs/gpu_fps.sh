#!/bin/bash
# The driver's bench shape (--steps 20 --warmup 5) at several frames per step, against the default
# 50 steps, interleaved twice: how much of the short run's deficit is its fixed start cost.
source "$(dirname "$0")/gpu_lib.sh"
for rep in 1 2; do
    for cfg in "50 64" "20 64" "20 128" "20 256"; do
        set -- $cfg
        run fps_${1}_${2}_$rep 200 python3 bench.py --steps $1 --warmup 5 --frames-per-step $2 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0
        echo "steps $1 fps $2 #$rep $(grep -o '"value": [0-9.]*' gpurun_out/fps_${1}_${2}_$rep.log)"
    done
done
