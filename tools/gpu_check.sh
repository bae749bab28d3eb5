#!/bin/bash
# One GPU-box session: parity tests, smoke, bench lines, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash-type exit (fault, abort, segfault, timeout)
# ends the script (test failures, rc 1, do not). Output under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
}
STEPS=${STEPS:-all}
if [[ $STEPS == all || $STEPS == *tests* ]]; then
    run pytest_gpu 900 python -m pytest tests -m gpu -q -x
fi
if [[ $STEPS == all || $STEPS == *smoke* ]]; then
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
    run bench_lds 600 python bench.py --steps 10 --warmup 2 --variant lds
    run bench_scalar 300 python bench.py --steps 10 --warmup 2 --variant scalar --no-cpu-baseline --no-e2e
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
    run rocprof_stats 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e
fi
echo done
