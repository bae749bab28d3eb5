#!/bin/bash
# Round 5 (second session): a 128-candidate batch spread over the first 32 lanes of all four waves (SRT_BATCH_SPREAD=1)
# against the product's first 128 threads (waves 0 and 1).
# Parity subset on the spread build first, then alternating bench rounds with uniform and random offsets.
source "$(dirname "$0")/gpu_lib.sh"
SRT_LIB=simpleraytracer_amd/lib_exp/spread/libModelRunner.so run pytest_spread 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_golden_full.py tests/test_gpu_engine.py -m gpu -x -q --timeout 200 --timeout-method thread
tail -2 gpurun_out/pytest_spread.log
grep -q " passed" gpurun_out/pytest_spread.log && ! grep -q "FAILED\|Error" gpurun_out/pytest_spread.log || { echo "tests failed"; exit 1; }
for round in 1 2; do
  for v in ${VARIANTS:-product spread}; do
    if [ $v = product ]; then L=simpleraytracer_amd/lib/libModelRunner.so; else L=simpleraytracer_amd/lib_exp/$v/libModelRunner.so; fi
    for off in uniform random; do
      SRT_LIB=$L run k_${v}_${off}_$round 200 python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0 --offsets $off
      echo "$v $off $round $(tail -1 gpurun_out/k_${v}_${off}_$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["roofline_single_frame"]["kernel_ms"])')"
    done
  done
done
