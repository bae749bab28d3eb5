#!/bin/bash
# Round 6: the GPU suite and smoke at HEAD (after the bench config change).
source "$(dirname "$0")/gpu_lib.sh"
run pytest_head 900 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread
tail -1 gpurun_out/pytest_head.log
run smoke_head 300 python3 -c "import __graft_entry__ as g; g.smoke()"
tail -1 gpurun_out/smoke_head.log
