#!/bin/bash
# Rank simulation (all-to-all P = 2, 4, 8) for each library of VARIANTS, twice interleaved.
source "$(dirname "$0")/gpu_lib.sh"
for rep in 1 2; do
    for v in ${VARIANTS:-product}; do
        lib=""; [ $v != product ] && lib=simpleraytracer_amd/lib_ab/$v/libModelRunner.so
        SRT_LIB=$lib run ra_${v}_$rep 300 python3 tools/rank_sim.py --ranks ${PS:-2,4,8} --exchange ${EXCH:-alltoall}
        grep '^{"P"' gpurun_out/ra_${v}_$rep.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$v#$rep', d['P'], d['slowest_us'])"
    done
done
