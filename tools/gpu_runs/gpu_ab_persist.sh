#!/bin/bash
# A/B of the persistent cull trace (render.hip TraceGrid, env SRT_TRACE_GRID; SRT_DESC_PREFETCH):
# correctness of the cull paths first, then the driver-shape bench and one queue per setting.
source "$(dirname "$0")/gpu_lib.sh"
run persist_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_full.py tests/test_gpu_engine_rccl.py \
    -m gpu -q -x --timeout 300 --timeout-method thread
for g in ${GRIDS:-0 1 2}; do
    SRT_TRACE_GRID=$g run persist_bench_g$g 300 python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline
    SRT_TRACE_GRID=$g run persist_q1_g$g 300 python3 bench.py --queues 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline
done
for lib in ${LIBS:-static}; do
    SRT_LIB=simpleraytracer_amd/lib_ab/$lib/libModelRunner.so run persist_bench_$lib 300 python3 bench.py --steps 20 \
        --warmup 5 --no-extras --no-cpu-baseline
done
python3 tools/bench_summary.py gpurun_out/persist_*bench*.log gpurun_out/persist_q1*.log
