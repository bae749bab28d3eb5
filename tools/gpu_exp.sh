#!/bin/bash
# Experiment GPU session: parity tests, then bench lines + rocprofv3 kernel stats under each
# env configuration in $CFGS (space-separated; each entry's '+' separates VAR=VALUE pairs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
    rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
fi
for cfg in ${CFGS:-NONE=0}; do
    tag=$(echo "$cfg" | tr '+=/' '___' | cut -c1-80)
    env $(echo "$cfg" | tr '+' ' ') timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/e_$tag -o run --output-format csv -- \
        python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e ${BENCH_ARGS:-} > gpurun_out/e_$tag.log 2>&1 || { echo "rc=$? $cfg"; exit 1; }
    echo "== $cfg"; grep -o '"value": [0-9.]*\|"single_queue": {"mrays_per_s": [0-9.]*' gpurun_out/e_$tag.log | tr '\n' ' '; echo
    cut -d, -f1,3,4 gpurun_out/e_$tag/run_kernel_stats.csv | sed 's/(srt::(anonymous namespace)::[A-Za-z]*)//; s/srt::(anonymous namespace):://' | head -8
done
echo done
