#!/bin/bash
# Round 6: the fake-device N = 2 line at HEAD (every N > 1 field prints with the last bench changes).
source "$(dirname "$0")/gpu_lib.sh"
SRT_BENCH_ONE_DEVICE=1 run fake2_head 600 python3 bench.py --gpus 2 --steps 10 --warmup 2 --cpu-seconds 4
tail -1 gpurun_out/fake2_head.log | cut -c1-300
