#!/bin/bash
# Round 5: trace-kernel A/B (make exp builds) -- bench value, launch8 and single-frame kernel time,
# alternating rounds. VARIANTS="product la ..." (lib_exp/<name>).
source "$(dirname "$0")/gpu_lib.sh"
for round in ${ROUNDS:-1 2}; do
  for v in ${VARIANTS:-product la}; do
    if [ $v = product ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
    SRT_LIB=$L run k_${v}_$round 200 python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0
    echo "$v $round $(tail -1 gpurun_out/k_${v}_$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["roofline_single_frame"]["kernel_ms"])')"
  done
done
