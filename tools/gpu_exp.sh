#!/bin/bash
# Diagnostic GPU session: the `make diag` library's per-block cull phase counters
# (tools/diag_cull.py) and rocprofv3 kernel stats of bench.py under SRT_EXP experiment bits
# (render.hip BinParams::exp; timing only, results are wrong with any bit set).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export SRT_LIB=simpleraytracer_amd/lib_diag/libModelRunner.so
timeout -k 10 120 python tools/diag_cull.py > gpurun_out/diag.json 2> gpurun_out/diag.err || { echo "diag rc=$?"; tail -5 gpurun_out/diag.err; exit 1; }
for e in ${EXPS:-0 1 2 4 8}; do
    SRT_EXP=$e timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/exp$e -o run --output-format csv -- \
        python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/exp$e.log 2>&1 || { echo "exp $e rc=$?"; exit 1; }
    echo "exp $e"; cut -d, -f1,4 gpurun_out/exp$e/run_kernel_stats.csv | cut -c1-120
done
echo done
