#!/bin/bash
# Chunk-size sweep of the split trace work items (bench lines + one-queue rocprof each).
source "$(dirname "$0")/gpu_lib.sh"
Q=(--no-cpu-baseline --no-e2e --brute-steps 0)
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
fi
for c in ${CHUNKS:-256 512 1024 128}; do
    SRT_CULL_CHUNK=$c run bench_c$c 300 python bench.py --steps 3000 --warmup 20 "${Q[@]}"
    SRT_CULL_CHUNK=$c run prof_c$c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c$c -o run --output-format csv -- \
        python3 bench.py --steps 50 --warmup 5 --queues 1 "${Q[@]}"
done
echo done
