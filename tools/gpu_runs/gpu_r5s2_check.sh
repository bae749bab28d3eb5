#!/bin/bash
# Round 5, second session: the GPU suite, smoke() and the default bench line at the restored HEAD
# (the container was re-created; the .so files were rebuilt here from the committed sources).
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread
tail -2 gpurun_out/pytest_gpu.log
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "FAILED\|Error" gpurun_out/pytest_gpu.log || { echo "tests failed"; exit 1; }
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 600 python3 bench.py --steps 20 --warmup 5
tail -1 gpurun_out/bench.log | cut -c1-300
echo done
