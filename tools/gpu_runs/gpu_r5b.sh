#!/bin/bash
# Round 5: rotated all-to-all at P = 8 / 4 / 2 -- queue, batch and launch-size sweep of the rank simulation.
source "$(dirname "$0")/gpu_lib.sh"
for cfg in "2 256 0" "3 256 0" "4 256 0" "2 512 0" "2 256 32" "2 256 128" "3 256 128"; do
  set -- $cfg
  run sw_q$1_b$2_l$3 200 python3 tools/rank_sim.py --exchange alltoall --rows rotated --ranks 8,4 --queues $1 --batch $2 --launch $3
  grep '^{"P"' gpurun_out/sw_q$1_b$2_l$3.log | cut -c1-120
done
