#!/bin/bash
# Round 5 closing check at the committed code: GPU suite, smoke, default bench line (driver shape).
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread
tail -2 gpurun_out/pytest_gpu.log
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "FAILED\|Error" gpurun_out/pytest_gpu.log || { echo "tests failed"; exit 1; }
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
tail -1 gpurun_out/smoke.log
run bench 600 python3 bench.py --steps 20 --warmup 5
tail -1 gpurun_out/bench.log | cut -c1-200
