#!/bin/bash
# Round 5: bin-launch LDS padding probe (bench A/B) and 8 shading rows per thread (rank simulation).
source "$(dirname "$0")/gpu_lib.sh"
VARIANTS="product binpad" ROUNDS="1 2" bash tools/gpu_runs/gpu_r5m.sh
for v in product rows8; do
  if [ $v = product ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
  for P in 2 8; do
    SRT_LIB=$L run t${P}_$v 200 rocprofv3 --kernel-trace --stats -d gpurun_out/t${P}_$v -o run --output-format csv -- \
        python3 tools/rank_sim.py --ranks $P --exchange alltoall --rows rotated --queues 1 --steps 6 --warmup 2
    echo "P=$P $v $(python3 tools/trace_shapes.py gpurun_out/t${P}_$v --kernel ShadeIds | cut -c1-120)"
  done
done
