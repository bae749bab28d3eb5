#!/bin/bash
# Round 6: C5 (1M triangles, 3840 x 2160, one GPU) frame-loop shape sweep: frame queues x frames per
# launch, 64-frame steps (the bench's C5 leg uses 2 queues x 8 frames per launch).
source "$(dirname "$0")/gpu_lib.sh"
C5="python3 bench.py --triangles 1000000 --width 3840 --height 2160 --frames-per-step 64 --steps 8 --warmup 2 --no-extras --no-cpu-baseline --no-e2e"
for q in 1 2 3; do
  for l in 4 8 16; do
    run c5_q${q}_l${l} 200 $C5 --queues $q --launch $l
    echo "q=$q launch=$l $(grep -o '"value": [0-9.]*' gpurun_out/c5_q${q}_l${l}.log)"
  done
done
