#!/bin/bash
# Multi-GPU path on a one-GPU box: GPU parity tests, the default bench line, the per-rank band
# simulation (compute ceiling of bands x P) and 2- / 4-rank rehearsals of bench.py over gloo.
source "$(dirname "$0")/gpu_lib.sh"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
fi
run bench_default 600 python bench.py --no-cpu-baseline
run band_sim 300 python tools/band_sim.py
for n in 2 4; do
    SRT_BENCH_BACKEND=gloo SRT_BENCH_ONE_DEVICE=1 run rehearse$n 300 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2953$n bench.py --gpus $n --steps 20 --warmup 2 \
        --no-extras
done
echo done
