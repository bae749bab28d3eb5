#!/bin/bash
# Round 5: deferred shading with 32-bit id-buffer offsets (SRT_SHADE_OFF32): parity, then the
# compositor's ShadeIdsKernel per launch at P = 2 / 4 / 8 (rank simulation, one queue), then its SALU count.
source "$(dirname "$0")/gpu_lib.sh"
SRT_LIB=simpleraytracer_amd/lib_exp/o32/libModelRunner.so run o32_tests 400 python -u -m pytest tests/test_gpu_engine.py tests/test_golden_full.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "shade or band or engine or rotated or share"
tail -1 gpurun_out/o32_tests.log
for v in product o32; do
  if [ $v = product ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
  for P in 2 4 8; do
    SRT_LIB=$L run t${P}_$v 200 rocprofv3 --kernel-trace --stats -d gpurun_out/t${P}_$v -o run --output-format csv -- \
        python3 tools/rank_sim.py --ranks $P --exchange alltoall --rows rotated --queues 1 --steps 6 --warmup 2
    echo "P=$P $v $(python3 tools/trace_shapes.py gpurun_out/t${P}_$v --kernel ShadeIds | cut -c1-120)"
  done
done
R="python3 tools/rank_sim.py --ranks 4 --exchange alltoall --rows rotated --queues 1 --steps 3 --warmup 1"
SRT_LIB=simpleraytracer_amd/lib_exp/o32/libModelRunner.so run o32_sq2 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU --kernel-include-regex ShadeIdsKernel -d gpurun_out/o32_sq2 -o run --output-format csv -- $R
python3 tools/pmc_sq.py --key o32 --dir gpurun_out/o32_sq2 --kernel ShadeIdsKernel --out gpurun_out/o32_pmc.json && cat gpurun_out/o32_pmc.json
