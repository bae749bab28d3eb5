#!/bin/bash
# Round 5: the wave-persistent deferred shading (ShadeIdsLoopKernel) -- parity, then its time in the
# P = 2 rotated rank simulation (one queue) against the grid kernel (noloop) and prefetch depths.
source "$(dirname "$0")/gpu_lib.sh"
run t_shade 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py \
    "tests/test_gpu_parity.py::test_deferred_shading_bitwise" "tests/test_gpu_parity.py::test_batched_band_shading_bitwise" \
    "tests/test_gpu_parity.py::test_interleaved_bands_bitwise" "tests/test_gpu_engine_rccl.py"
grep -q " passed" gpurun_out/t_shade.log && ! grep -q "FAILED\|Error" gpurun_out/t_shade.log || { echo "tests failed"; exit 1; }
for v in product noloop loop_a4 loop_a8 blk4096; do
  if [ $v = product ] || [ $v = blk1024 ] || [ $v = blk4096 ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
  B=0; [ $v = blk1024 ] && B=1024; [ $v = blk4096 ] && B=4096
  for P in 2 8; do
    SRT_SHADE_LOOP_BLOCKS=$B SRT_LIB=$L run sh${P}_$v 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sh${P}_$v -o run --output-format csv -- \
        python3 tools/rank_sim.py --ranks $P --exchange alltoall --rows rotated --queues 1 --steps 6 --warmup 2
    echo "P=$P $v $(python3 tools/trace_shapes.py gpurun_out/sh${P}_$v --kernel ShadeIds | cut -c1-120)"
  done
done
for v in product noloop; do
  if [ $v = product ] || [ $v = blk1024 ] || [ $v = blk4096 ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
  SRT_LIB=$L run rs2_$v 200 python3 tools/rank_sim.py --ranks 2,4,8 --exchange alltoall --rows rotated
  grep '^{"P"' gpurun_out/rs2_$v.log | cut -c1-90
done
