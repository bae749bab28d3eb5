#!/bin/bash
# Same-box A/B of library variants (VARIANTS: names under simpleraytracer_amd/lib_ab/, "product" =
# the in-tree library): rank simulation at P = 8 all-to-all and P = 2 share, and the default bench
# line, REPS times interleaved.
source "$(dirname "$0")/gpu_lib.sh"
for rep in $(seq 1 ${REPS:-2}); do
    for v in ${VARIANTS:-old product}; do
        lib=""; [ $v != product ] && lib=simpleraytracer_amd/lib_ab/$v/libModelRunner.so
        SRT_LIB=$lib run va8_${v}_$rep 300 python3 tools/rank_sim.py --ranks 8 --exchange alltoall
        SRT_LIB=$lib run va2_${v}_$rep 300 python3 tools/rank_sim.py --ranks 2 --exchange share
        SRT_LIB=$lib run vab_${v}_$rep 200 python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-e2e --brute-steps 0 --no-extras
        echo "$v#$rep P8 $(grep -o '"slowest_us": [0-9.]*' gpurun_out/va8_${v}_$rep.log | head -1) P2share $(grep -o '"slowest_us": [0-9.]*' gpurun_out/va2_${v}_$rep.log | head -1) bench $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/vab_${v}_$rep.log | tr '\n' ' ')"
    done
done
