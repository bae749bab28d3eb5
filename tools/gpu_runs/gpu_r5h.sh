#!/bin/bash
# Round 5: mlInfer with the trace storing straight into the mapped host image (SRT_E2E_DIRECT=1).
source "$(dirname "$0")/gpu_lib.sh"
run e2e_copy 120 python3 tools/e2e_probe.py --chunks 2,4,8 --reps 10
SRT_E2E_DIRECT=1 run e2e_direct 120 python3 tools/e2e_probe.py --chunks 1,2,4,8,16 --reps 10
grep chunks gpurun_out/e2e_copy.log gpurun_out/e2e_direct.log
SRT_E2E_DIRECT=1 run t_direct 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
    "tests/test_gpu_parity.py::test_ml_pipelined_chunks_bitwise" "tests/test_gpu_parity.py::test_c2_cornell_1080p_ml_api" \
    "tests/test_gpu_parity.py::test_c1_single_triangle_256_ml_api" "tests/test_gpu_parity.py::test_float16_images"
tail -2 gpurun_out/t_direct.log
