#!/bin/bash
# Same-box A/B of library variants (VARIANTS; "product" = the in-tree library) on the rank
# simulation at the defaults (share exchange) for P = 2, 4, 8 and the default bench line, REPS
# times interleaved; GPU tests of the product first (TESTS=0 skips them).
source "$(dirname "$0")/gpu_lib.sh"
if [ "${TESTS:-1}" = 1 ]; then
    run ar_tests 500 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_full.py tests/test_gpu_engine.py \
        -m gpu -q -x --timeout 200 --timeout-method thread
fi
for rep in $(seq 1 ${REPS:-2}); do
    for v in ${VARIANTS:-head product}; do
        lib=""; [ $v != product ] && lib=simpleraytracer_amd/lib_ab/$v/libModelRunner.so
        SRT_LIB=$lib run ar_rank_${v}_$rep 300 python3 tools/rank_sim.py --ranks 2,4,8
        SRT_LIB=$lib run ar_bench_${v}_$rep 200 python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-e2e --brute-steps 0 --no-extras
        echo "$v#$rep $(grep '^{"P"' gpurun_out/ar_rank_${v}_$rep.log | python3 -c "import sys,json
print(' '.join('P%d=%s' % (d['P'], d['slowest_us']) for d in map(json.loads, sys.stdin)))") bench $(grep -o '"value": [0-9.]*' gpurun_out/ar_bench_${v}_$rep.log)"
    done
done
