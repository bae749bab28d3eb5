#!/bin/bash
# Frame-engine check on the GPU box: engine tests, the full GPU suite, the bench in the driver's
# shape, and the multi-device rehearsal (fake devices: GPU 0 repeated) at N = 2, 4, 8.
# STEPS=engine,tests,bench,rehearse selects.
source "$(dirname "$0")/gpu_lib.sh"
STEPS=${STEPS:-engine,tests,bench,rehearse}
if [[ $STEPS == *engine* ]]; then
    run pytest_engine 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v --timeout 120 --timeout-method thread
fi
if [[ $STEPS == *tests* ]]; then
    run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
fi
if [[ $STEPS == *bench* ]]; then
    run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
    run bench_long 300 python bench.py --no-extras --no-cpu-baseline
fi
if [[ $STEPS == *rehearse* ]]; then
    for n in 2 4 8; do
        SRT_BENCH_ONE_DEVICE=1 run rehearse$n 300 python bench.py --gpus $n --steps 20 --warmup 3 --no-e2e
    done
fi
echo done
