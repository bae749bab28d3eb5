#!/bin/bash
# Quick GPU check after a kernel change: full parity suite, the main bench line (no extras),
# one-queue rocprofv3 kernel stats, and (setup) the setup probe and band simulation.
# STEPS=tests,bench,prof,setup selects.
source "$(dirname "$0")/gpu_lib.sh"
STEPS=${STEPS:-tests,bench,prof}
if [[ $STEPS == *tests* ]]; then
    run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
fi
if [[ $STEPS == *bench* ]]; then
    run bench 400 python bench.py --no-extras --no-cpu-baseline
fi
if [[ $STEPS == *setup* ]]; then
    run setup_probe 300 python tools/setup_probe.py
    run band_sim 300 python tools/band_sim.py --steps 2000
fi
if [[ $STEPS == *prof* ]]; then
    run prof_q1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q1 -o run --output-format csv -- \
        python3 bench.py --steps 300 --warmup 5 --queues 1 --no-extras --no-cpu-baseline
fi
echo done
