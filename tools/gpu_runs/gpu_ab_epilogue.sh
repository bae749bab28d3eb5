#!/bin/bash
# Trace epilogue A/B: GPU parity of the RGBA path (parity, golden, engine), then the same-box
# A/B of tools/gpu_runs/gpu_ab_head.sh (rank simulation at P = 2, 8 and the default bench line).
source "$(dirname "$0")/gpu_lib.sh"
run ep_tests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_full.py tests/test_gpu_engine.py \
    -m gpu -q -x --timeout 200 --timeout-method thread
bash "$(dirname "$0")/gpu_ab_head.sh"
