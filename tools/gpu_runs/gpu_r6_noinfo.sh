#!/bin/bash
# Round 6, upper bound: the headline with the tile-info blocks' offset reads removed (measurement build
# noinfo: every offset taken as the tile's first -- exact only for uniform offsets, the headline's), against
# the product's build (base), three alternating rounds; and one frame in flight.
source "$(dirname "$0")/gpu_lib.sh"
L=simpleraytracer_amd/lib_exp
B="python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e"
S="python3 bench.py --steps 400 --warmup 20 --frames-per-step 1 --queues 1 --launch 1 --no-extras --no-cpu-baseline --no-e2e"
for r in 1 2 3; do
  for v in base noinfo; do
    SRT_LIB=$L/$v/libModelRunner.so run ni_${v}_$r 150 $B
  done
  echo "round $r: base $(grep -o '"value": [0-9.]*' gpurun_out/ni_base_$r.log | head -1 | cut -d' ' -f2) noinfo $(grep -o '"value": [0-9.]*' gpurun_out/ni_noinfo_$r.log | head -1 | cut -d' ' -f2) verified $(grep -o '"verified": [a-z]*' gpurun_out/ni_noinfo_$r.log | head -1)"
done
for v in base noinfo; do
  SRT_LIB=$L/$v/libModelRunner.so run ni_${v}_s 150 $S
  echo "$v single $(grep -o '"value": [0-9.]*' gpurun_out/ni_${v}_s.log | head -1) $(grep -o '"bin": [0-9.]*' gpurun_out/ni_${v}_s.log | head -1)"
done
