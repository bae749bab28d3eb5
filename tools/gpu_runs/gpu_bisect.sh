#!/bin/bash
# Rank-simulation bisection over lib_ab builds of intermediate commits (VARIANTS), the product last.
source "$(dirname "$0")/gpu_lib.sh"
for rep in 1 2; do
    for v in ${VARIANTS:-old c_plan c_fab c_share c_tile product x_noempty}; do
        lib=""; [ $v != product ] && lib=simpleraytracer_amd/lib_ab/$v/libModelRunner.so
        SRT_LIB=$lib run bis_${v}_$rep 300 python3 tools/rank_sim.py --ranks 2,8 --exchange alltoall
        grep '^{"P"' gpurun_out/bis_${v}_$rep.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$v#$rep', d['P'], d['slowest_us'])"
    done
done
