#!/bin/bash
# Round 5: staggered frame queues (SRT_STAGGER) -- rank simulation (rotated all-to-all, share) and P = 1.
source "$(dirname "$0")/gpu_lib.sh"
for S in 1 0 1 0; do
  SRT_STAGGER=$S run st$S 200 python3 tools/rank_sim.py --ranks 1,2,4,8 --exchange alltoall --rows rotated
  echo "STAGGER $S: $(grep '^{"P"' gpurun_out/st$S.log | python3 -c 'import sys,json; print([(d["P"], d["slowest_us"]) for d in map(json.loads, sys.stdin)])')"
done
for S in 1 0; do
  SRT_STAGGER=$S run sts$S 200 python3 tools/rank_sim.py --ranks 2,8 --exchange share
  echo "STAGGER share $S: $(grep '^{"P"' gpurun_out/sts$S.log | python3 -c 'import sys,json; print([(d["P"], d["slowest_us"]) for d in map(json.loads, sys.stdin)])')"
done
