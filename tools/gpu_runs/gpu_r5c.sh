#!/bin/bash
# Round 5: deferred-shading kernel variants (make exp builds) in the P = 2 rotated rank simulation,
# one queue: ShadeIdsKernel's own time per launch (128 frames of 540 rows).
source "$(dirname "$0")/gpu_lib.sh"
for v in product store_only no_record rows2 thr256; do
  if [ $v = product ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
  SRT_LIB=$L run sh_$v 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sh_$v -o run --output-format csv -- \
      python3 tools/rank_sim.py --ranks 2 --exchange alltoall --rows rotated --queues 1 --steps 6 --warmup 2
  python3 tools/trace_shapes.py gpurun_out/sh_$v --kernel ShadeIds
done
