#!/bin/bash
# Round 6: records recomputed by the trace (SRT_TRACE_RECOMPUTE=1: the bin kernel writes a 16-B screen box
# per position instead of the 64-B cull record) against the product's record reads (rc0): the GPU suite
# on the rc library first, then alternating A/B rounds -- headline (driver shape), one frame in flight,
# C5 leg shape (1 queue x 16-frame launches).
source "$(dirname "$0")/gpu_lib.sh"
L=simpleraytracer_amd/lib_exp
SRT_LIB=$L/rc/libModelRunner.so run rc_pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
grep -E "passed|failed" gpurun_out/rc_pytest.log | tail -1
B="python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e"
S="python3 bench.py --steps 400 --warmup 20 --frames-per-step 1 --queues 1 --launch 1 --no-extras --no-cpu-baseline --no-e2e"
C5="python3 bench.py --triangles 1000000 --width 3840 --height 2160 --frames-per-step 64 --steps 10 --warmup 2 --queues 1 --launch 16 --no-extras --no-cpu-baseline --no-e2e"
for r in 1 2 3; do
  for v in rc0 rc; do
    SRT_LIB=$L/$v/libModelRunner.so run ${v}_h_$r 150 $B
    SRT_LIB=$L/$v/libModelRunner.so run ${v}_c5_$r 200 $C5
  done
  echo "round $r: headline rc0 $(grep -o '"value": [0-9.]*' gpurun_out/rc0_h_$r.log) rc $(grep -o '"value": [0-9.]*' gpurun_out/rc_h_$r.log); C5 rc0 $(grep -o '"value": [0-9.]*' gpurun_out/rc0_c5_$r.log) rc $(grep -o '"value": [0-9.]*' gpurun_out/rc_c5_$r.log)"
done
for v in rc0 rc; do
  SRT_LIB=$L/$v/libModelRunner.so run ${v}_s 150 $S
  echo "$v single $(grep -o '"value": [0-9.]*' gpurun_out/${v}_s.log) $(grep -o '"stages_ms": {[^}]*' gpurun_out/${v}_s.log | cut -c1-120)"
done
