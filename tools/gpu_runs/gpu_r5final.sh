#!/bin/bash
# Round 5 final evidence: full GPU suite, the default bench line (driver shape), fake-device N > 1
# rehearsals, the rank simulations, and the launch8 kernel trace + HBM traffic passes of the roofline.
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread
tail -2 gpurun_out/pytest_gpu.log
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "FAILED\|Error" gpurun_out/pytest_gpu.log || { echo "tests failed"; exit 1; }
run bench 600 python3 bench.py --steps 20 --warmup 5
tail -1 gpurun_out/bench.log | cut -c1-200
SRT_BENCH_ONE_DEVICE=1 run fake2 400 python3 bench.py --gpus 2 --steps 4 --warmup 2 --no-cpu-baseline
SRT_BENCH_ONE_DEVICE=1 run fake8 400 python3 bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu-baseline
for ex in "alltoall rotated" "share interleaved" "alltoall interleaved"; do
  set -- $ex
  run rsf_$1_$2 300 python3 tools/rank_sim.py --exchange $1 --rows $2
  echo "$1 $2: $(grep '^{"P"' gpurun_out/rsf_$1_$2.log | python3 -c 'import sys,json; print([(d["P"], d["slowest_us"]) for d in map(json.loads, sys.stdin)])')"
done
B="python3 bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0"
K="--kernel-include-regex TraceCullKernel"
run l8_trace 200 timeout -s KILL 190 rocprofv3 --kernel-trace --stats -d gpurun_out/l8_trace -o run --output-format csv -- $B
tail -1 gpurun_out/l8_trace.log | cut -c1-200
run l8_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE $K -d gpurun_out/l8_fetch -o run --output-format csv -- $B
run l8_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE $K -d gpurun_out/l8_write -o run --output-format csv -- $B
echo done
