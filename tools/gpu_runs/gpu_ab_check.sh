#!/bin/bash
# Parity first (the GPU test suite, stopping at the first failure), then -- only if it is green --
# an A/B of library builds (tools/gpu_runs/gpu_libs.sh; LIBS="base NAME ...", NAME from lib_ab/).
source "$(dirname "$0")/gpu_lib.sh"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -n 3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then
    echo "pytest rc=$rc: no A/B"
    exit $rc
fi
LIBS="${LIBS:-base old}" LIBDIR_AB=lib_ab bash tools/gpu_runs/gpu_libs.sh
