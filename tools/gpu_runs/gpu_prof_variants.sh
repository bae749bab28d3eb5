#!/bin/bash
# Same-box kernel statistics of the P = 8 rank simulation for library variants (VARIANTS, as in
# tools/gpu_runs/gpu_ab_variants.sh), with QUEUES frame queues (one: each kernel's own time).
source "$(dirname "$0")/gpu_lib.sh"
for q in ${QUEUES:-1 2}; do
    for v in ${VARIANTS:-old product}; do
        lib=""; [ $v != product ] && lib=simpleraytracer_amd/lib_ab/$v/libModelRunner.so
        n=pv_${v}_q$q
        SRT_LIB=$lib run $n 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$n -o run --output-format csv -- \
            python3 tools/rank_sim.py --ranks ${P:-8} --exchange ${EX:-alltoall} --queues $q --steps 20
        python3 tools/kernel_stats.py gpurun_out/$n | head -6
        grep -o '"slowest_us": [0-9.]*' gpurun_out/$n.log | head -1
    done
done
