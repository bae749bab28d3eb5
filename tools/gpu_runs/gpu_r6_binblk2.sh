#!/bin/bash
# Round 6: confirmation of the bin block size A/B (gpu_r6_binblk.sh read 128-record blocks +1.2 % on the
# headline in both rounds): three more alternating rounds of the driver shape, 256 (product) against 128
# (one tile-info tile per block), plus a P = 8 rank simulation of each (the band skip's block granularity).
source "$(dirname "$0")/gpu_lib.sh"
B="python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e"
for r in 3 4 5; do
  for v in bt256 bt128; do
    SRT_LIB=simpleraytracer_amd/lib_exp/$v/libModelRunner.so run ${v}_h_$r 150 $B
  done
  echo "round $r: bt256 $(grep -o '"value": [0-9.]*' gpurun_out/bt256_h_$r.log) bt128 $(grep -o '"value": [0-9.]*' gpurun_out/bt128_h_$r.log)"
done
for v in bt256 bt128; do
  SRT_LIB=simpleraytracer_amd/lib_exp/$v/libModelRunner.so run ${v}_rs8 200 python3 tools/rank_sim.py --ranks 1,8 --rows rotated --exchange alltoall
  grep -hE "\"P\": (1|8)," gpurun_out/${v}_rs8.log | cut -c1-120
done
