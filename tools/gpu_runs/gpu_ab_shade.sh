#!/bin/bash
# Deferred-shading rows per thread (SRT_SHADE_ROWS: lib_ab/shade8, lib_ab/shade16) against the
# product library: the shading parity tests, then the rank simulation at P = 2 and 8.
source "$(dirname "$0")/gpu_lib.sh"
for v in ${VARIANTS:-shade8 shade16}; do
    SRT_LIB=simpleraytracer_amd/lib_ab/$v/libModelRunner.so run tests_$v 300 python -u -m pytest tests/test_gpu_parity.py \
        tests/test_gpu_engine.py tests/test_gpu_engine_rccl.py -m gpu -q -x --timeout 200 --timeout-method thread \
        -k "shad or band or engine or packed or collision"
done
for rep in 1 2; do
    for v in product ${VARIANTS:-shade8 shade16}; do
        lib=""; [ $v != product ] && lib=simpleraytracer_amd/lib_ab/$v/libModelRunner.so
        SRT_LIB=$lib run ranks_${v}_$rep 300 python3 tools/rank_sim.py --ranks 2,8
        grep '^{"P"' gpurun_out/ranks_${v}_$rep.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$v#$rep', d['P'], d['slowest_us'])"
    done
done
