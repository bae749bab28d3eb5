#!/bin/bash
# Batched band gather: its parity tests, then 2- and 4-rank gloo rehearsals of bench.py.
source "$(dirname "$0")/gpu_lib.sh"
run t_batch 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "batched_band or deferred"
for n in 2 4; do
    SRT_BENCH_BACKEND=gloo SRT_BENCH_ONE_DEVICE=1 run rehearse$n 300 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2953$n bench.py --gpus $n --steps 48 \
        --warmup 2 --no-extras
done
echo done
