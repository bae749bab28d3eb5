#!/bin/bash
# Round 5: split room per launch (SRT_CULL_SPLIT extra descriptors, default = resident trace blocks) at N = 1.
source "$(dirname "$0")/gpu_lib.sh"
for round in 1 2; do
  for S in default 0 768 3072 6144; do
    if [ $S = default ]; then unset SRT_CULL_SPLIT; else export SRT_CULL_SPLIT=$S; fi
    run sp_${S}_$round 200 python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0
    echo "split=$S $round $(tail -1 gpurun_out/sp_${S}_$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["roofline_single_frame"]["kernel_ms"])')"
  done
  unset SRT_CULL_SPLIT
done
