#!/bin/bash
# Full GPU-box session for a round's evidence: parity tests, smoke, the default bench line
# (with cpu_baseline + e2e), rocprofv3 kernel stats of the same bench command, and the two
# PMC traffic passes (FETCH_SIZE, WRITE_SIZE, separate runs) for the trace kernel.
# Each GPU step has its own time limit; a crash-type exit (fault, abort, segfault, timeout)
# ends the script; test failures (rc 1) do not. Output under gpurun_out/.
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
STEPS=${STEPS:-tests,smoke,bench,prof,pmc}
KERNEL_RE=${KERNEL_RE:-TraceCullKernel}
BENCH=(python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-e2e --brute-steps 0)
if [[ $STEPS == *tests* ]]; then
    run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
fi
if [[ $STEPS == *smoke* ]]; then
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $STEPS == *bench* ]]; then
    run bench 600 python bench.py
fi
if [[ $STEPS == *rehearse* ]]; then
    SRT_BENCH_BACKEND=gloo SRT_BENCH_ONE_DEVICE=1 run rehearse2 300 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2
fi
if [[ $STEPS == *quick* ]]; then
    run bench_quick 300 "${BENCH[@]}"
fi
if [[ $STEPS == *prof* ]]; then
    run prof_stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- "${BENCH[@]}"
    # one frame in flight: per-kernel durations without the frame-queue overlap (the bench's
    # roofline/stage times come from its single-queue instrumented pass)
    run prof_stats_q1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q1 -o run --output-format csv -- \
        "${BENCH[@]}" --queues 1
fi
if [[ $STEPS == *pmc* ]]; then
    run pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KERNEL_RE" -d gpurun_out/pmc_fetch -o run --output-format csv -- "${BENCH[@]}"
    run pmc_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KERNEL_RE" -d gpurun_out/pmc_write -o run --output-format csv -- "${BENCH[@]}"
    python3 tools/pmc_traffic.py --key "soup-100k 1920x1080 1spp|cull" --kernel "$KERNEL_RE" \
        --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --out gpurun_out/pmc_traffic.json
fi
echo done
