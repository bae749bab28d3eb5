#!/bin/bash
# Round 6: the split trace launch (regular-tile kernel at 7 blocks per CU + the other tiles' kernel):
# its parity tests, then A/B against the previous library (prev) and the persistent variant (persist),
# uniform and jittered offsets.
source "$(dirname "$0")/gpu_lib.sh"
run pytest_split 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
    -k "trace_batch or work_plan or mixed or headline or engine_c3 or rotated or cull"
LIBS="prev base persist" bash tools/gpu_runs/gpu_r6_ab.sh
LIBS="prev base persist" BENCH_ARGS="--offsets random" bash tools/gpu_runs/gpu_r6_ab.sh
