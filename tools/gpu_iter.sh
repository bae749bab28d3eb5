#!/bin/bash
# Quick GPU iteration: parity tests (optionally filtered) then bench lines per variant / cull mode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 4 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -x ${PYTEST_K:+-k "$PYTEST_K"}
for v in ${BENCH_VARIANTS:-cull}; do
    if [ "$v" = cull ]; then
        for b in ${CULL_BINS:-1}; do
            SRT_CULL_BIN=$b step "bench_cull_bin$b" 300 python bench.py --steps 50 --warmup 5 --variant cull --no-cpu-baseline --no-e2e
        done
    else
        step "bench_$v" 300 python bench.py --steps 10 --warmup 2 --variant "$v" --no-cpu-baseline --no-e2e
    fi
done
echo done
