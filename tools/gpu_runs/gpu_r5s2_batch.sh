#!/bin/bash
# Round 5 (second session): packet-walk batches of 64 candidates (22.8 KB of LDS: 7 blocks per CU fit at
# 72 VGPRs, b64o7; b64 = 6 blocks per CU) against the product's 128 (26.4 KB: 6 per CU).
# Alternating bench rounds with uniform and random offsets.
source "$(dirname "$0")/gpu_lib.sh"
for round in 1 2; do
  for v in ${VARIANTS:-product b64o7 b64}; do
    if [ $v = product ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
    for off in uniform random; do
      SRT_LIB=$L run k_${v}_${off}_$round 200 python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0 --offsets $off
      echo "$v $off $round $(tail -1 gpurun_out/k_${v}_${off}_$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["roofline_single_frame"]["kernel_ms"])')"
    done
  done
done
