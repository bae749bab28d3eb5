#!/bin/bash
# Round 5: packed ids carry spatial positions (position-ordered shading table at the compositor): the
# GPU suite, then ShadeIdsKernel per launch at P = 2 / 4 / 8 (C3) and the C5 P = 8 rank breakdown, then
# the rank simulations.
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread
tail -2 gpurun_out/pytest_gpu.log
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "FAILED\|Error" gpurun_out/pytest_gpu.log || { echo "tests failed"; exit 1; }
for P in 2 4 8; do
  run tp${P} 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tp${P} -o run --output-format csv -- \
      python3 tools/rank_sim.py --ranks $P --exchange alltoall --rows rotated --queues 1 --steps 6 --warmup 2
  echo "P=$P $(python3 tools/trace_shapes.py gpurun_out/tp${P} --kernel ShadeIds | cut -c1-120)"
done
run c5p8 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c5p8 -o run --output-format csv -- \
    python3 tools/rank_sim.py --ranks 8 --triangles 1000000 --width 3840 --height 2160 --batch 64 --steps 4 --warmup 2 --queues 1 --exchange alltoall --rows rotated
python3 tools/trace_shapes.py gpurun_out/c5p8 | head -6
run rsx 300 python3 tools/rank_sim.py --exchange alltoall --rows rotated
echo "c3 rotated: $(grep '^{"P"' gpurun_out/rsx.log | python3 -c 'import sys,json; print([(d["P"], d["slowest_us"]) for d in map(json.loads, sys.stdin)])')"
run c5x 600 python3 tools/rank_sim.py --triangles 1000000 --width 3840 --height 2160 --batch 64 --steps 6 --warmup 3 --exchange alltoall --rows rotated
echo "c5 rotated: $(grep '^{"P"' gpurun_out/c5x.log | python3 -c 'import sys,json; print([(d["P"], d["slowest_us"]) for d in map(json.loads, sys.stdin)])')"
