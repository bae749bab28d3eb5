#!/bin/bash
# Round 5 (second session): render.hip built under LLVM's other AMDGPU machine schedulers
# (-mllvm -amdgpu-sched-strategy = max-ilp / iterative-ilp / max-memory-clause) against the default
# (max-occupancy). Scheduling only: the explicit fmaf / -ffp-contract=off numerics are unchanged.
source "$(dirname "$0")/gpu_lib.sh"
for round in 1 2; do
  for v in ${VARIANTS:-product ilp iter mml}; do
    if [ $v = product ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
    for off in uniform random; do
      SRT_LIB=$L run k_${v}_${off}_$round 200 python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0 --offsets $off
      echo "$v $off $round $(tail -1 gpurun_out/k_${v}_${off}_$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["roofline_single_frame"]["kernel_ms"])')"
    done
  done
done
