#!/bin/bash
# Round 6: split chunks of any size (SRT_CHUNK_POW2=0, lib_exp/np2: S = max(min_chunk, C / (D - P)) itself
# instead of the power of two above it) against the product (p2): the GPU suite on np2, then one frame in
# flight at min_chunk 160 / 192 / 224 / 256 and the headline at 192 / 256, two alternating rounds.
source "$(dirname "$0")/gpu_lib.sh"
L=simpleraytracer_amd/lib_exp
SRT_LIB=$L/np2/libModelRunner.so run np2_pytest 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 gpurun_out/np2_pytest.log
grep -q " passed" gpurun_out/np2_pytest.log && ! grep -q "FAILED\|Error" gpurun_out/np2_pytest.log || { echo "tests failed"; exit 1; }
B="python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e"
S="python3 bench.py --steps 400 --warmup 20 --frames-per-step 1 --queues 1 --launch 1 --no-extras --no-cpu-baseline --no-e2e"
for r in 1 2; do
  line="round $r single:"
  SRT_LIB=$L/p2/libModelRunner.so run np_p2_s_$r 150 $S
  line="$line p2 $(grep -o '"value": [0-9.]*' gpurun_out/np_p2_s_$r.log | head -1 | cut -d' ' -f2)"
  for c in 160 192 224 256; do
    SRT_LIB=$L/np2/libModelRunner.so SRT_CULL_CHUNK=$c run np_${c}_s_$r 150 $S
    line="$line np2/$c $(grep -o '"value": [0-9.]*' gpurun_out/np_${c}_s_$r.log | head -1 | cut -d' ' -f2)"
  done
  echo "$line"
  line="round $r headline:"
  SRT_LIB=$L/p2/libModelRunner.so run np_p2_h_$r 150 $B
  line="$line p2 $(grep -o '"value": [0-9.]*' gpurun_out/np_p2_h_$r.log | head -1 | cut -d' ' -f2)"
  for c in 192 256; do
    SRT_LIB=$L/np2/libModelRunner.so SRT_CULL_CHUNK=$c run np_${c}_h_$r 150 $B
    line="$line np2/$c $(grep -o '"value": [0-9.]*' gpurun_out/np_${c}_h_$r.log | head -1 | cut -d' ' -f2)"
  done
  echo "$line"
done
