#!/bin/bash
# Round 5: the two-device split at 80 and 85 % (rank simulation, P = 2, rotated all-to-all).
source "$(dirname "$0")/gpu_lib.sh"
for own in 80 85 75; do
  SRT_ROTATE_OWN=$own run rs_own$own 200 python3 tools/rank_sim.py --ranks 2 --exchange alltoall --rows rotated
  echo "own=$own $(grep '^{"P"' gpurun_out/rs_own$own.log | python3 -c 'import sys,json; print([(d["P"], d["slowest_us"], d["link_us_per_frame"], d["job_ceiling_mrays"]) for d in map(json.loads, sys.stdin)])')"
done
