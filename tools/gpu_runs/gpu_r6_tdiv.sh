#!/bin/bash
# Round 6: the tile info's box divided once per tile (the extremes of fl(x + o) divided after the reduction,
# monotone: the same bits) instead of two divisions per pixel: the GPU suite at that code, then the headline
# A/B against the previous build (base), four alternating rounds, and one frame in flight.
source "$(dirname "$0")/gpu_lib.sh"
L=simpleraytracer_amd/lib_exp
run td_pytest 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/td_pytest.log
grep -q " passed" gpurun_out/td_pytest.log && ! grep -q "FAILED\|Error" gpurun_out/td_pytest.log || { echo "tests failed"; exit 1; }
B="python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e"
S="python3 bench.py --steps 400 --warmup 20 --frames-per-step 1 --queues 1 --launch 1 --no-extras --no-cpu-baseline --no-e2e"
for r in 1 2 3 4; do
  for v in base tdiv; do
    SRT_LIB=$L/$v/libModelRunner.so run td_${v}_$r 150 $B
  done
  echo "round $r: base $(grep -o '"value": [0-9.]*' gpurun_out/td_base_$r.log | head -1 | cut -d' ' -f2) tdiv $(grep -o '"value": [0-9.]*' gpurun_out/td_tdiv_$r.log | head -1 | cut -d' ' -f2)"
done
for v in base tdiv; do
  SRT_LIB=$L/$v/libModelRunner.so run td_${v}_s 150 $S
  echo "$v single $(grep -o '"value": [0-9.]*' gpurun_out/td_${v}_s.log | head -1) $(grep -o '"bin": [0-9.]*' gpurun_out/td_${v}_s.log | head -1)"
done
