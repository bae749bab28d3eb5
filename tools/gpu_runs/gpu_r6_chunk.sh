#!/bin/bash
# Round 6: one frame in flight (records recomputed) against the smallest candidate chunk of a split tile part
# (SRT_CULL_CHUNK 128 / 256 (default) / 512 / 1024), two alternating rounds.
source "$(dirname "$0")/gpu_lib.sh"
S="python3 bench.py --steps 400 --warmup 20 --frames-per-step 1 --queues 1 --launch 1 --no-extras --no-cpu-baseline --no-e2e"
for r in 1 2; do
  line="round $r:"
  for c in 128 256 512 1024; do
    SRT_CULL_CHUNK=$c run ch${c}_$r 150 $S
    line="$line c$c $(grep -o '"value": [0-9.]*' gpurun_out/ch${c}_$r.log | head -1 | cut -d' ' -f2) trace $(grep -o '"trace_kernel": [0-9.]*' gpurun_out/ch${c}_$r.log | head -1 | cut -d' ' -f2)"
  done
  echo "$line"
done
