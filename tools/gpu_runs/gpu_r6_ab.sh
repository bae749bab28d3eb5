#!/bin/bash
# Round 6 A/B of experiment libraries (make exp EXP_NAME=...) in the driver's bench shape, two
# interleaved rounds: LIBS="base nofxy7 ...". Prints value, trace kernel ms (8-frame launch) and
# single-frame trace ms per run.
source "$(dirname "$0")/gpu_lib.sh"
for rep in 1 2; do
    for name in ${LIBS:-base}; do
        if [ "$name" = base ]; then lib=""; else lib="simpleraytracer_amd/lib_exp/$name/libModelRunner.so"; fi
        env SRT_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
            --no-e2e ${BENCH_ARGS:-} > gpurun_out/ab_${name}_${rep}${BENCH_ARGS:+_alt}.log 2>&1 || { echo "rc=$? $name"; exit 1; }
        echo "$name#$rep $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"verified": [a-z]*' gpurun_out/ab_${name}_${rep}${BENCH_ARGS:+_alt}.log | tr '\n' ' ')"
    done
done
