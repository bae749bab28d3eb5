#!/bin/bash
# Frames per trace launch (FrameEngine launch option): GPU tests, then rank_sim and the bench line
# for each LAUNCHES value.
source "$(dirname "$0")/gpu_lib.sh"
if [ "${TESTS:-1}" = 1 ]; then
    run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
fi
for l in ${LAUNCHES:-8 16 32 64}; do
    run rs_l$l 300 python tools/rank_sim.py --ranks ${RANKS:-1,8} --launch $l
    run bench_l$l 300 python bench.py --no-extras --no-cpu-baseline --launch $l
done
for l in ${LAUNCHES:-8 16 32 64}; do
    echo "== launch $l"; grep '"P"' gpurun_out/rs_l$l.log
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_l$l.log').read().strip().splitlines()[-1]); print('bench', d['value'], d['verified'])"
done
