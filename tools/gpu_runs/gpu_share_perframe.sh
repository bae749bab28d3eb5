#!/bin/bash
# Per-frame share exchange (frame f composited on f % P in its compositor's row pattern): engine GPU
# tests, rank simulations (share vs all-to-all, C3 and C5 at P = 8) and the fake-device rehearsals.
source "$(dirname "$0")/gpu_lib.sh"
run pf_tests 400 python -u -m pytest tests/test_gpu_engine.py -m gpu -q -x --timeout 200 --timeout-method thread
run pf_rank 400 python tools/rank_sim.py --ranks 1,2,4,8
run pf_rank_b256 400 python tools/rank_sim.py --ranks 2,4,8 --batch 256 --steps 8 --warmup 4
run pf_rank_c5 500 python tools/rank_sim.py --ranks 8 --width 3840 --height 2160 --triangles 1000000 --steps 16 --warmup 8
for n in 2 4 8; do
    SRT_BENCH_ONE_DEVICE=1 run pf_rehearse$n 400 python bench.py --gpus $n --steps 20 --warmup 2 --no-e2e --frames-per-step 64
done
for f in pf_rank pf_rank_b256 pf_rank_c5; do
    grep '^{"P"' gpurun_out/$f.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$f', d['P'], d['us_per_frame'], d['link_us_per_frame'])"
done
for n in 2 4 8; do grep -o '"verified": [a-z]*' gpurun_out/pf_rehearse$n.log | head -1; done
