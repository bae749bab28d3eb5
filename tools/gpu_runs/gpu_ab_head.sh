#!/bin/bash
# Same-box A/B of the product library against lib_ab/old (an earlier build): rank simulation at
# P = 2, 8 (all-to-all) and the default bench line, twice interleaved.
source "$(dirname "$0")/gpu_lib.sh"
for rep in 1 2; do
    for v in old product; do
        lib=""; [ $v = old ] && lib=simpleraytracer_amd/lib_ab/old/libModelRunner.so
        SRT_LIB=$lib run hrs_${v}_$rep 300 python3 tools/rank_sim.py --ranks 2,8 --exchange alltoall
        grep '^{"P"' gpurun_out/hrs_${v}_$rep.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$v#$rep', d['P'], d['slowest_us'])"
        SRT_LIB=$lib run hb_${v}_$rep 200 python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-e2e --brute-steps 0 --no-extras
        echo "$v#$rep $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/hb_${v}_$rep.log | tr '\n' ' ')"
    done
done
