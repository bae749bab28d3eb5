#!/bin/bash
# Round 6: the C5 leg's launch size at one queue (records recomputed: the one-queue policy), 16 / 32 / 64
# frames per launch of 64-frame steps, two alternating rounds.
source "$(dirname "$0")/gpu_lib.sh"
C5="python3 bench.py --triangles 1000000 --width 3840 --height 2160 --frames-per-step 64 --steps 10 --warmup 2 --queues 1 --no-extras --no-cpu-baseline --no-e2e"
for r in 1 2; do
  for l in 16 32 64; do
    run c5l_${l}_$r 200 $C5 --launch $l
  done
  echo "round $r: l16 $(grep -o '"value": [0-9.]*' gpurun_out/c5l_16_$r.log) l32 $(grep -o '"value": [0-9.]*' gpurun_out/c5l_32_$r.log) l64 $(grep -o '"value": [0-9.]*' gpurun_out/c5l_64_$r.log)"
done
