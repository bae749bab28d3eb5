#!/bin/bash
# Round 6 evidence at the final code (record sources, 48-B spatial inputs, C5 leg at one queue x 64-frame
# launches). PART a: full GPU suite, smoke, the default bench line (driver shape, every leg), fake-device
# N = 2 / 8 lines. PART b: rank simulations, the rocprofv3 kernel trace of the bench's launch shapes, HBM
# traffic passes of the launch shapes the line's roofline blocks quote (C3 8-frame, C3 one-frame, C5 leg).
source "$(dirname "$0")/gpu_lib.sh"
PART=${PART:-a}
if [ "$PART" = a ]; then
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread
tail -2 gpurun_out/pytest_gpu.log
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "FAILED\|Error" gpurun_out/pytest_gpu.log || { echo "tests failed"; exit 1; }
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
run bench 900 python3 bench.py --steps 20 --warmup 5
tail -1 gpurun_out/bench.log | cut -c1-200
SRT_BENCH_ONE_DEVICE=1 run fake2 600 python3 bench.py --gpus 2 --steps 10 --warmup 2 --cpu-seconds 4
SRT_BENCH_ONE_DEVICE=1 run fake8 600 python3 bench.py --gpus 8 --steps 4 --warmup 1 --cpu-seconds 4
exit 0
fi
for ex in "alltoall rotated" "share interleaved" "alltoall interleaved"; do
  set -- $ex
  run rsf_$1_$2 300 python3 tools/rank_sim.py --exchange $1 --rows $2
  echo "$1 $2: $(grep '^{"P"' gpurun_out/rsf_$1_$2.log | python3 -c 'import sys,json; print([(d["P"], d["slowest_us"]) for d in map(json.loads, sys.stdin)])')"
done
run rsf_c5 400 python3 tools/rank_sim.py --exchange alltoall --rows rotated --width 3840 --height 2160 --triangles 1000000 --batch 64 --steps 8 --warmup 4
B="python3 bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0"
B1="python3 bench.py --steps 300 --warmup 20 --frames-per-step 1 --queues 1 --launch 1 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0"
B5="python3 bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline --no-e2e --brute-steps 0 --triangles 1000000 --width 3840 --height 2160 --frames-per-step 64 --queues 1 --launch 64"
K="--kernel-include-regex TraceCullKernel"
run l8_trace 200 timeout -s KILL 190 rocprofv3 --kernel-trace --stats -d gpurun_out/l8_trace -o run --output-format csv -- $B
run l8_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE $K -d gpurun_out/l8_fetch -o run --output-format csv -- $B
run l8_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE $K -d gpurun_out/l8_write -o run --output-format csv -- $B
run l1_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE $K -d gpurun_out/l1_fetch -o run --output-format csv -- $B1
run l1_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE $K -d gpurun_out/l1_write -o run --output-format csv -- $B1
run c5_trace 300 timeout -s KILL 290 rocprofv3 --kernel-trace --stats -d gpurun_out/c5_trace -o run --output-format csv -- $B5
run c5_fetch 300 timeout -s KILL 290 rocprofv3 --pmc FETCH_SIZE $K -d gpurun_out/c5_fetch -o run --output-format csv -- $B5
run c5_write 300 timeout -s KILL 290 rocprofv3 --pmc WRITE_SIZE $K -d gpurun_out/c5_write -o run --output-format csv -- $B5
echo done
