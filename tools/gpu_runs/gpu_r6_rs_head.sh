#!/bin/bash
# Round 6: rank simulations at HEAD (after the per-tile division of the tile info).
source "$(dirname "$0")/gpu_lib.sh"
for ex in "alltoall rotated" "share interleaved"; do
  set -- $ex
  run rsh_$1_$2 300 python3 tools/rank_sim.py --exchange $1 --rows $2
  echo "$1 $2: $(grep '^{"P"' gpurun_out/rsh_$1_$2.log | python3 -c 'import sys,json; r=[json.loads(l) for l in sys.stdin]; p1=r[0]["slowest_us"]; print([(d["P"], d["slowest_us"], round(p1/d["slowest_us"],3)) for d in r])')"
done
run rsh_c5 400 python3 tools/rank_sim.py --exchange alltoall --rows rotated --width 3840 --height 2160 --triangles 1000000 --batch 64 --steps 8 --warmup 4
echo "c5: $(grep '^{"P"' gpurun_out/rsh_c5.log | python3 -c 'import sys,json; r=[json.loads(l) for l in sys.stdin]; p1=r[0]["slowest_us"]; print([(d["P"], d["slowest_us"], round(p1/d["slowest_us"],3)) for d in r])')"
