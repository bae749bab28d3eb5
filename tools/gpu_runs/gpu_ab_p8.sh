#!/bin/bash
# Same-box A/B of library variants (VARIANTS, as in tools/gpu_runs/gpu_ab_variants.sh) on the P = 8 rank
# simulation alone, REPS times interleaved, with QUEUES frame queues.
source "$(dirname "$0")/gpu_lib.sh"
for rep in $(seq 1 ${REPS:-2}); do
    for v in ${VARIANTS:-old product}; do
        lib=""; [ $v != product ] && lib=simpleraytracer_amd/lib_ab/$v/libModelRunner.so
        SRT_LIB=$lib run p8_${v}_$rep 300 python3 tools/rank_sim.py --ranks ${P:-8} --exchange ${EX:-alltoall} --queues ${QUEUES:-2}
        echo "$v#$rep P${P:-8} $(grep -o '"us_per_frame": {[^}]*}' gpurun_out/p8_${v}_$rep.log | head -1)"
    done
done
