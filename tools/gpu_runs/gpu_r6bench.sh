#!/bin/bash
# Round 6: smoke and the default bench line (driver shape) at the final code.
source "$(dirname "$0")/gpu_lib.sh"
run smoke_head 300 python3 -c "import __graft_entry__ as g; g.smoke()"
tail -1 gpurun_out/smoke_head.log
run bench 900 python3 bench.py --steps 20 --warmup 5
tail -1 gpurun_out/bench.log | cut -c1-200
