#!/bin/bash
# Batched launches: parity tests, bench at N = 1 with 1 and 8 frames per launch, the band
# simulation with batch 8 and 1, and a 2-rank gloo rehearsal of the batched band path.
source "$(dirname "$0")/gpu_lib.sh"
run t_batch 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread \
    -k "batch or deferred or setup_state or variants_bitwise or split"
run bench_b1 300 python bench.py --no-extras --no-cpu-baseline --batch 1
run bench_b8 300 python bench.py --no-extras --no-cpu-baseline --batch 8
run band_sim_b8 300 python tools/band_sim.py --steps 2000 --batch 8
run band_sim_b1 300 python tools/band_sim.py --steps 2000 --batch 1
SRT_BENCH_BACKEND=gloo SRT_BENCH_ONE_DEVICE=1 run rehearse2 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 48 --warmup 2 --no-extras
echo done
