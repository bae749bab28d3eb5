#!/bin/bash
# Round 6: the headline's frame loop at the final code -- frame queues 2 / 3 x frames per launch 8 / 16 / 32
# (driver shape, 256-frame steps), two alternating rounds.
source "$(dirname "$0")/gpu_lib.sh"
B="python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e"
for r in 1 2; do
  line="round $r:"
  for q in 2 3; do
    for l in 8 16 32; do
      run sh_q${q}_l${l}_$r 150 $B --queues $q --launch $l
      line="$line q$q/l$l $(grep -o '"value": [0-9.]*' gpurun_out/sh_q${q}_l${l}_$r.log | head -1 | cut -d' ' -f2)"
    done
  done
  echo "$line"
done
