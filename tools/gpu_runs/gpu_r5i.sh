#!/bin/bash
# Round 5: does capping the deferred shading's blocks per CU (dynamic LDS) let the other queue's traces
# overlap it? Rotated all-to-all rank simulation, 2 queues, P = 2 and 8.
source "$(dirname "$0")/gpu_lib.sh"
for L in 0 8192 16384 32768; do
  SRT_SHADE_LDS=$L run lds$L 200 python3 tools/rank_sim.py --ranks 2,8 --exchange alltoall --rows rotated
  echo "LDS $L: $(grep '^{"P"' gpurun_out/lds$L.log | cut -c1-60 | tr '\n' ' ')"
done
