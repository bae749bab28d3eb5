#!/bin/bash
# Round 6: confirmation of tile-info tiles per block 4 (it4) against 2 (ba4 = the product's build), headline
# driver shape, four more alternating rounds.
source "$(dirname "$0")/gpu_lib.sh"
L=simpleraytracer_amd/lib_exp
B="python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e"
for r in 3 4 5 6; do
  for v in ba4 it4; do
    SRT_LIB=$L/$v/libModelRunner.so run k${v}_h_$r 150 $B
  done
  echo "round $r: ba4 $(grep -o '"value": [0-9.]*' gpurun_out/kba4_h_$r.log | head -1 | cut -d' ' -f2) it4 $(grep -o '"value": [0-9.]*' gpurun_out/kit4_h_$r.log | head -1 | cut -d' ' -f2)"
done
