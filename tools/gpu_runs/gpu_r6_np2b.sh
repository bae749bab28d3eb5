#!/bin/bash
# Round 6: confirmation of split chunks of any size (np2) against power-of-two chunks (p2) on the headline,
# four more alternating rounds, and the C5 leg's shape once each.
source "$(dirname "$0")/gpu_lib.sh"
L=simpleraytracer_amd/lib_exp
B="python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e"
C5="python3 bench.py --triangles 1000000 --width 3840 --height 2160 --frames-per-step 64 --steps 10 --warmup 2 --queues 1 --launch 64 --no-extras --no-cpu-baseline --no-e2e"
for r in 3 4 5 6; do
  for v in p2 np2; do
    SRT_LIB=$L/$v/libModelRunner.so run nb_${v}_$r 150 $B
  done
  echo "round $r: p2 $(grep -o '"value": [0-9.]*' gpurun_out/nb_p2_$r.log | head -1 | cut -d' ' -f2) np2 $(grep -o '"value": [0-9.]*' gpurun_out/nb_np2_$r.log | head -1 | cut -d' ' -f2)"
done
for v in p2 np2; do
  SRT_LIB=$L/$v/libModelRunner.so run nb_${v}_c5 200 $C5
  echo "c5 $v $(grep -o '"value": [0-9.]*' gpurun_out/nb_${v}_c5.log | head -1)"
done
