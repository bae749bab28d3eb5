#!/bin/bash
# Round 5: mlInfer end to end -- chunk counts, with / without torch's context, SDMA vs blit-kernel copies.
source "$(dirname "$0")/gpu_lib.sh"
run e2e_plain 120 python3 tools/e2e_probe.py --chunks 4,6,8 --reps 12
run e2e_torch 120 python3 tools/e2e_probe.py --chunks 4,6,8 --reps 12 --torch
HSA_ENABLE_SDMA=0 run e2e_nosdma 120 python3 tools/e2e_probe.py --chunks 4,6,8 --reps 12
HSA_ENABLE_SDMA=0 run e2e_nosdma_torch 120 python3 tools/e2e_probe.py --chunks 4,6,8 --reps 12 --torch
for f in e2e_plain e2e_torch e2e_nosdma e2e_nosdma_torch; do echo "== $f"; grep chunks gpurun_out/$f.log; done
HSA_ENABLE_SDMA=0 run bench_nosdma 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --brute-steps 0
tail -1 gpurun_out/bench_nosdma.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], json.dumps(d.get("e2e_ml_api")))'
