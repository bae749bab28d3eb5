#!/bin/bash
# Round 6: tile info by a lean one-wave kernel (TileInfoWaveKernel, 24 VGPRs, no LDS: lib_exp/fw, SRT_INFO_WAVE=1)
# launched before the bin launch (SRT_FUSED_INFO=0) so its waves fit beside the other queue's trace blocks,
# against the product's fused tile info (base) and the unfused 256-thread kernel: the GPU suite on fw unfused
# first, then the headline (three alternating rounds) and one frame in flight.
source "$(dirname "$0")/gpu_lib.sh"
L=simpleraytracer_amd/lib_exp
SRT_LIB=$L/fw/libModelRunner.so SRT_FUSED_INFO=0 run fw_pytest 600 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --deselect "tests/test_gpu_parity.py::test_stage_timing_does_not_change_the_frame[cull]"
tail -1 gpurun_out/fw_pytest.log
grep -q " passed" gpurun_out/fw_pytest.log && ! grep -q "FAILED\|Error" gpurun_out/fw_pytest.log || { echo "tests failed"; exit 1; }
B="python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e"
S="python3 bench.py --steps 400 --warmup 20 --frames-per-step 1 --queues 1 --launch 1 --no-extras --no-cpu-baseline --no-e2e"
for r in 1 2 3; do
  SRT_LIB=$L/base/libModelRunner.so run fw_base_$r 150 $B
  SRT_LIB=$L/base/libModelRunner.so SRT_FUSED_INFO=0 run fw_unf_$r 150 $B
  SRT_LIB=$L/fw/libModelRunner.so SRT_FUSED_INFO=0 run fw_wave_$r 150 $B
  echo "round $r: fused $(grep -o '"value": [0-9.]*' gpurun_out/fw_base_$r.log | head -1 | cut -d' ' -f2) unfused $(grep -o '"value": [0-9.]*' gpurun_out/fw_unf_$r.log | head -1 | cut -d' ' -f2) wave $(grep -o '"value": [0-9.]*' gpurun_out/fw_wave_$r.log | head -1 | cut -d' ' -f2) (trace $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/fw_wave_$r.log | head -1 | cut -d' ' -f2))"
done
SRT_LIB=$L/base/libModelRunner.so run fw_base_s 150 $S
SRT_LIB=$L/fw/libModelRunner.so SRT_FUSED_INFO=0 run fw_wave_s 150 $S
echo "single: fused $(grep -o '"value": [0-9.]*' gpurun_out/fw_base_s.log | head -1) wave $(grep -o '"value": [0-9.]*' gpurun_out/fw_wave_s.log | head -1)"
