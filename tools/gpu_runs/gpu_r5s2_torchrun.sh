#!/bin/bash
# Round 5 (second session): the driver's launch form rehearsed on the one-GPU box at the final code --
# torch.distributed.run with one rank (N = 1) and two ranks on the one GPU (fake devices: RCCL refuses two
# ranks on one device, so the run must end in bench's error record or the device-copy path, never a hang).
source "$(dirname "$0")/gpu_lib.sh"
run tr1 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 \
    bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --brute-steps 0
tail -1 gpurun_out/tr1.log | cut -c1-300
SRT_BENCH_ONE_DEVICE=1 run tr2 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29542 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline
tail -1 gpurun_out/tr2.log | cut -c1-600
