#!/bin/bash
# Deferred-shading change check: the shading / band / engine parity tests, then the rank
# simulation (all-to-all P = 2, 8; share at P = 2) against lib_ab/old, twice interleaved.
source "$(dirname "$0")/gpu_lib.sh"
run shade_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py tests/test_gpu_engine_rccl.py \
    tests/test_golden_full.py -m gpu -q -x --timeout 300 --timeout-method thread \
    -k "shad or band or engine or packed or share or interleaved or golden or full or c5"
for rep in 1 2; do
    for v in old product; do
        lib=""; [ $v != product ] && lib=simpleraytracer_amd/lib_ab/$v/libModelRunner.so
        SRT_LIB=$lib run sc_${v}_$rep 300 python3 tools/rank_sim.py --ranks 2,4,8 --exchange alltoall
        grep '^{"P"' gpurun_out/sc_${v}_$rep.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$v#$rep', d['P'], d['slowest_us'])"
    done
done
run sc_share 300 python3 tools/rank_sim.py --ranks 1,2 --exchange share
grep '^{"P"' gpurun_out/sc_share.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('share', d['P'], d['slowest_us'], 'link', d['link_us_per_frame'], 'job', d['job_ceiling_mrays'])"
