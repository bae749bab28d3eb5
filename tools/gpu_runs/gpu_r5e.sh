#!/bin/bash
# Round 5: bench lines -- N = 1 (the driver's shape, with the mlInfer host-link roofline) and the fake-device
# rehearsals at N = 2 / 4 / 8 (every N > 1 field: exchange timing, legs, one frame in flight, ml_multi).
source "$(dirname "$0")/gpu_lib.sh"
run b1 400 python3 bench.py --steps 20 --warmup 5
tail -1 gpurun_out/b1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"], d.get("e2e_ml_api"))'
for N in 2 8; do
  SRT_BENCH_ONE_DEVICE=1 run r$N 400 python3 bench.py --gpus $N --steps 10 --warmup 2 --no-cpu-baseline
  tail -1 gpurun_out/r$N.log | cut -c1-400
done
python3 tools/e2e_probe.py --chunks 2,4,8,12,16 > gpurun_out/e2e_chunks.log 2>&1; tail -6 gpurun_out/e2e_chunks.log
