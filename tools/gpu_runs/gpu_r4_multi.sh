#!/bin/bash
# Multi-GPU path evidence on a one-GPU box: the engine / band GPU tests, then the rank simulation
# (per-rank GPU time + the modelled exchange, tools/rank_sim.py) at C3 and C5.
source "$(dirname "$0")/gpu_lib.sh"
run multi_tests 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_engine_rccl.py tests/test_golden_full.py \
    -m gpu -q -x --timeout 300 --timeout-method thread
run rank_sim 400 python3 tools/rank_sim.py --all-ranks
run rank_sim_c5 500 python3 tools/rank_sim.py --width 3840 --height 2160 --triangles 1000000 --steps 8 --ranks 1,8
