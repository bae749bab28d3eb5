#!/bin/bash
# The share exchange: its GPU tests (fake devices, the RCCL tests) and the rank simulation at P = 2
# (share 1 / 3 / 7 against all-to-all) and P = 4, 8.
source "$(dirname "$0")/gpu_lib.sh"
run share_tests 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_engine_rccl.py tests/test_gpu_parity.py -m gpu -q -x \
    --timeout 300 --timeout-method thread -k "share or fake_devices or interleaved or band or engine or packed or shad"
for cfg in "alltoall 0" "share 2" "share 4" "share 8"; do
    set -- $cfg
    run rs_${1}_$2 300 python3 tools/rank_sim.py --ranks 2 --exchange $1 --share $2
    grep '^{"P"' gpurun_out/rs_${1}_$2.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$1/$2', d['P'], d['slowest_us'], 'link', d['link_us_per_frame'], 'job', d['job_ceiling_mrays'])"
done
for cfg in "share 4" "alltoall 0"; do
    set -- $cfg
    run rs48_${1}_$2 300 python3 tools/rank_sim.py --ranks 4,8 --exchange $1 --share $2
    grep '^{"P"' gpurun_out/rs48_${1}_$2.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$1/$2', d['P'], d['slowest_us'], 'link', d['link_us_per_frame'], 'job', d['job_ceiling_mrays'])"
done
