#!/bin/bash
# Iteration session: GPU parity tests (PYTEST_K filter optional), then bench lines for uniform
# and random offsets and a one-queue rocprofv3 kernel-stats pass of each.
source "$(dirname "$0")/gpu_lib.sh"
Q=(--no-cpu-baseline --no-e2e --brute-steps 0)
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
fi
run bench_uniform 300 python bench.py --steps 3000 --warmup 20 "${Q[@]}"
run bench_random 300 python bench.py --steps 1000 --warmup 20 --offsets random "${Q[@]}"
run prof_uniform 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_uniform -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --queues 1 "${Q[@]}"
run prof_random 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_random -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --offsets random --queues 1 "${Q[@]}"
echo done
