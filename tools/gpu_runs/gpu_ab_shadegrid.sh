#!/bin/bash
# Compacted shade grid: GPU parity (parity, golden, engine), one-queue kernel statistics of the rank
# simulations (tools/gpu_runs/gpu_prof_share.sh), then rank simulations (2 queues) of lib_ab/old vs the
# product at P = 2 share / all-to-all and P = 8, twice interleaved.
source "$(dirname "$0")/gpu_lib.sh"
run sg_tests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_full.py tests/test_gpu_engine.py \
    -m gpu -q -x --timeout 200 --timeout-method thread
bash "$(dirname "$0")/gpu_prof_share.sh"
for rep in 1 2; do
    for v in old product; do
        lib=""; [ $v = old ] && lib=simpleraytracer_amd/lib_ab/old/libModelRunner.so
        for ex in share alltoall; do
            SRT_LIB=$lib run sg_${v}_${ex}_$rep 300 python3 tools/rank_sim.py --ranks 2,8 --exchange $ex
            grep '^{"P"' gpurun_out/sg_${v}_${ex}_$rep.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$v $ex #$rep', d['P'], d['slowest_us'])"
        done
    done
done
