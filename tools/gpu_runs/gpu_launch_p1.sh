#!/bin/bash
# P = 1 frames per launch now that tables upload by kernel: the default bench line at 8 (kernel
# arguments), 16, 32, 64 (device tables), twice interleaved.
source "$(dirname "$0")/gpu_lib.sh"
for rep in 1 2; do
    for L in ${LS:-8 16 32 64}; do
        run lp_${L}_$rep 200 python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-e2e --brute-steps 0 --no-extras --launch $L
        echo "L=$L#$rep $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/lp_${L}_$rep.log | head -2 | tr '\n' ' ')"
    done
done
