#!/bin/bash
# Round 5: C5 (1M-triangle soup, 3840 x 2160) -- the bench leg at N = 1 and the rank simulation of the
# rotated all-to-all at P = 1 / 2 / 4 / 8 (64-frame batches).
source "$(dirname "$0")/gpu_lib.sh"
run c5_bench 400 python3 bench.py --triangles 1000000 --width 3840 --height 2160 --steps 4 --warmup 2 --frames-per-step 64 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0
tail -1 gpurun_out/c5_bench.log | cut -c1-300
run c5_rank 600 python3 tools/rank_sim.py --triangles 1000000 --width 3840 --height 2160 --batch 64 --steps 6 --warmup 3 --exchange alltoall --rows rotated
echo "c5 rotated: $(grep '^{"P"' gpurun_out/c5_rank.log | python3 -c 'import sys,json; print([(d["P"], d["slowest_us"], d["link_us_per_frame"]) for d in map(json.loads, sys.stdin)])')"
