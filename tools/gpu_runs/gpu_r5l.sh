#!/bin/bash
# Round 5: full GPU suite, the default bench line (driver shape) and the rank simulations at the final code.
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -3 gpurun_out/pytest_gpu.log
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "FAILED\|Error" gpurun_out/pytest_gpu.log || { echo "tests failed"; exit 1; }
run bench 600 python3 bench.py --steps 20 --warmup 5
tail -1 gpurun_out/bench.log | cut -c1-300
for ex in "alltoall rotated" "share interleaved" "alltoall interleaved"; do
  set -- $ex
  run rsf_$1_$2 300 python3 tools/rank_sim.py --exchange $1 --rows $2
  echo "$1 $2: $(grep '^{"P"' gpurun_out/rsf_$1_$2.log | python3 -c 'import sys,json; print([(d["P"], d["slowest_us"]) for d in map(json.loads, sys.stdin)])')"
done
