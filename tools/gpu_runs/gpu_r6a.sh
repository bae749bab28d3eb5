#!/bin/bash
# Round 6, first check: the GPU suite at the split / stage-timing fixes and the stripped render.hip,
# the driver-shape bench line (binned CPU baseline beside the oracle) and a fake-device N = 2 line.
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread
run bench 600 python bench.py --steps 20 --warmup 5
run fake2 400 env SRT_BENCH_ONE_DEVICE=1 python bench.py --gpus 2 --steps 10 --warmup 2 --no-extras --no-e2e --cpu-seconds 4
