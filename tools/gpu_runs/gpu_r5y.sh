#!/bin/bash
# Round 5: deferred shading with write-back (plain) framebuffer stores instead of nontemporal ones.
source "$(dirname "$0")/gpu_lib.sh"
for v in product plainst; do
  if [ $v = product ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
  for P in 2 8; do
    SRT_LIB=$L run t${P}_$v 200 rocprofv3 --kernel-trace --stats -d gpurun_out/t${P}_$v -o run --output-format csv -- \
        python3 tools/rank_sim.py --ranks $P --exchange alltoall --rows rotated --queues 1 --steps 6 --warmup 2
    echo "P=$P $v $(python3 tools/trace_shapes.py gpurun_out/t${P}_$v --kernel ShadeIds | cut -c1-120)"
  done
  SRT_LIB=$L run rs_$v 300 python3 tools/rank_sim.py --ranks 2,8 --exchange alltoall --rows rotated
  echo "$v $(grep '^{"P"' gpurun_out/rs_$v.log | python3 -c 'import sys,json; print([(d["P"], d["slowest_us"]) for d in map(json.loads, sys.stdin)])')"
done
