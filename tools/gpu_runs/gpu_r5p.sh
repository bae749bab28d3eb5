#!/bin/bash
# Round 5 (second half): the default bench line (driver shape), fake-device N > 1 rehearsals of the
# line's every field, and the rank simulations at this code.
source "$(dirname "$0")/gpu_lib.sh"
run bench 600 python3 bench.py --steps 20 --warmup 5
tail -1 gpurun_out/bench.log | cut -c1-300
SRT_BENCH_ONE_DEVICE=1 run fake2 400 python3 bench.py --gpus 2 --steps 4 --warmup 2 --no-cpu-baseline
SRT_BENCH_ONE_DEVICE=1 run fake8 400 python3 bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu-baseline
for ex in "alltoall rotated" "share interleaved" "alltoall interleaved"; do
  set -- $ex
  run rsf_$1_$2 300 python3 tools/rank_sim.py --exchange $1 --rows $2
  echo "$1 $2: $(grep '^{"P"' gpurun_out/rsf_$1_$2.log | python3 -c 'import sys,json; print([(d["P"], d["slowest_us"]) for d in map(json.loads, sys.stdin)])')"
done
