#!/bin/bash
# Share exchange at the library's k (srtShareAuto) as the bands default: rank simulations (share and
# all-to-all; C3, and C5 at P = 1, 8) and the multi-GPU rehearsals (fake devices, verified frames).
source "$(dirname "$0")/gpu_lib.sh"
run se_rank_share 400 python tools/rank_sim.py --all-ranks
run se_rank_alltoall 400 python tools/rank_sim.py --ranks 2,4,8 --exchange alltoall
run se_rank_c5 500 python tools/rank_sim.py --ranks 1,8 --width 3840 --height 2160 --triangles 1000000 --steps 16 --warmup 8
run se_rank_c5_alltoall 400 python tools/rank_sim.py --ranks 8 --width 3840 --height 2160 --triangles 1000000 --steps 16 --warmup 8 --exchange alltoall
for n in 2 4 8; do
    SRT_BENCH_ONE_DEVICE=1 run se_rehearse$n 400 python bench.py --gpus $n --steps 20 --warmup 2 --no-e2e --frames-per-step 64
done
for f in se_rank_share se_rank_alltoall se_rank_c5 se_rank_c5_alltoall; do
    grep '^{"P"' gpurun_out/$f.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$f', d['P'], d['slowest_us'], d['link_us_per_frame'], d['bound'])"
done
