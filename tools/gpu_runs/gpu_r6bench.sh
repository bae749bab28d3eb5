#!/bin/bash
# Round 6: the default bench line (driver shape) at the final code, after the final traffic passes.
source "$(dirname "$0")/gpu_lib.sh"
run bench 900 python3 bench.py --steps 20 --warmup 5
tail -1 gpurun_out/bench.log | cut -c1-200
