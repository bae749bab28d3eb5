#!/bin/bash
# Round 5: mlInfer end to end vs the NUMA node the process (and so its pinned host images) lives on.
source "$(dirname "$0")/gpu_lib.sh"
for n in -1 0 1 -1 0 1; do
  run e2e_node$n 120 python3 tools/e2e_probe.py --chunks 4 --reps 10 --node $n
  grep -E "numa|pinned|chunks" gpurun_out/e2e_node$n.log | cut -c1-300
done
