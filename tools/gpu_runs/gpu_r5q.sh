#!/bin/bash
# Round 5: the two-device rotated split (band 0 = SRT_ROTATE_OWN per cent): engine tests, then the rank
# simulation at P = 2 for several splits.
source "$(dirname "$0")/gpu_lib.sh"
run own_tests 500 python -u -m pytest tests/test_gpu_engine.py tests/test_golden_full.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "rotated or engine or shade or band"
tail -2 gpurun_out/own_tests.log
for own in 50 62 75 81 88; do
  SRT_ROTATE_OWN=$own run rs_own$own 200 python3 tools/rank_sim.py --ranks 2 --exchange alltoall --rows rotated
  echo "own=$own $(grep '^{"P"' gpurun_out/rs_own$own.log | python3 -c 'import sys,json; print([(d["P"], d["slowest_us"], d["link_us_per_frame"], d["job_ceiling_mrays"]) for d in map(json.loads, sys.stdin)])')"
done
