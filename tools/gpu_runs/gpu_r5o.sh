#!/bin/bash
# Round 5: deferred-shading kernel A/B (tile offset pinned with the id loads, exact float row division):
# the shading parity tests, then ShadeIdsKernel per launch in rank simulations at P = 2 and 8.
source "$(dirname "$0")/gpu_lib.sh"
run sh_tests 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "shade or band or engine or rotated or share"
for v in ${VARIANTS:-product nopin}; do
  if [ $v = product ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
  for P in 2 8; do
    SRT_LIB=$L run t${P}_$v 200 rocprofv3 --kernel-trace --stats -d gpurun_out/t${P}_$v -o run --output-format csv -- \
        python3 tools/rank_sim.py --ranks $P --exchange alltoall --rows rotated --queues 1 --steps 6 --warmup 2
    echo "P=$P $v $(python3 tools/trace_shapes.py gpurun_out/t${P}_$v --kernel ShadeIds | cut -c1-120)"
  done
done
for v in ${VARIANTS:-product nopin}; do
  if [ $v = product ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
  SRT_LIB=$L run rs_$v 300 python3 tools/rank_sim.py --ranks 2,8 --exchange alltoall --rows rotated
  grep '"P"' gpurun_out/rs_$v.log | cut -c1-60
done
