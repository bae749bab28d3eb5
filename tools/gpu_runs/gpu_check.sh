#!/bin/bash
# The usual check of a change on the one-GPU box: GPU parity tests, one-frame-in-flight kernel stats
# of the product library, the rank simulation at P = 1 and 8, and a bench line without the CPU
# baseline (STEPS: any of tests, q1, ranks, bench).
source "$(dirname "$0")/gpu_lib.sh"
STEPS=${STEPS:-tests,q1,ranks,bench}
if [[ $STEPS == *tests* ]]; then
    run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
fi
if [[ $STEPS == *q1* ]]; then
    run prof_q1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q1 -o run --output-format csv -- \
        python3 bench.py --steps 300 --warmup 20 --queues 1 --frames-per-step 1 --no-extras --no-cpu-baseline
    python3 tools/kernel_stats.py gpurun_out/prof_q1
fi
if [[ $STEPS == *ranks* ]]; then
    run rank_sim 300 python tools/rank_sim.py --ranks 1,8
fi
if [[ $STEPS == *bench* ]]; then
    run bench 300 python bench.py --no-cpu-baseline --no-e2e --brute-steps 0
    python3 tools/bench_summary.py gpurun_out/bench.log
fi
