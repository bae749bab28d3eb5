#!/bin/bash
# Round 5: frames per trace launch at N = 1 (bench --launch), driver shape, two rounds.
source "$(dirname "$0")/gpu_lib.sh"
for round in 1 2; do
  for L in 8 4 6 12; do
    run l_${L}_$round 200 python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0 --launch $L
    echo "launch=$L $round $(tail -1 gpurun_out/l_${L}_$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"])')"
  done
done
