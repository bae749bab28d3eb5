#!/bin/bash
# Fused tile info for bands (SRT_FUSED_INFO=bands: tile info in the bin launch, every cull record
# written) against the default (a TileInfoKernel launch per band launch, band-restricted records):
# the band parity tests under it, then the rank simulation at P = 2, 4, 8 both ways.
source "$(dirname "$0")/gpu_lib.sh"
SRT_FUSED_INFO=bands run fused_tests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -m gpu -q -x \
    --timeout 200 --timeout-method thread -k "band or interleaved or cull_modes or setup_state or engine or extreme or uniform"
for v in default bands; do
    SRT_FUSED_INFO=$([ $v = bands ] && echo bands || echo 1) run ranks_$v 300 python3 tools/rank_sim.py --ranks 2,4,8
    grep '^{"P"' gpurun_out/ranks_$v.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$v', d['P'], d['slowest_us'], d['us_per_frame'])"
done
