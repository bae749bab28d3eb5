#!/bin/bash
# Round 5: trace-kernel knob variants (make exp builds) at the current code -- bench value and launch8
# kernel time, alternating twice.
source "$(dirname "$0")/gpu_lib.sh"
for round in 1; do
  for v in product ilp2 lp1 lp3 occ5; do
    if [ $v = product ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
    SRT_LIB=$L run k_${v}_$round 200 python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0
    echo "$v $round $(tail -1 gpurun_out/k_${v}_$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["roofline_single_frame"]["kernel_ms"])')"
  done
done
for v in product tids; do
  if [ $v = product ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
  for P in 2 8; do
    SRT_LIB=$L run t${P}_$v 200 rocprofv3 --kernel-trace --stats -d gpurun_out/t${P}_$v -o run --output-format csv -- \
        python3 tools/rank_sim.py --ranks $P --exchange alltoall --rows rotated --queues 1 --steps 6 --warmup 2
    echo "P=$P $v $(python3 tools/trace_shapes.py gpurun_out/t${P}_$v --kernel ShadeIds | cut -c1-120)"
  done
done
