#!/bin/bash
# rocprofv3 session on the GPU box for one bench configuration:
#   1. kernel trace + stats (per-kernel durations)       -> gpurun_out/prof_<tag>/
#   2. PMC pass FETCH_SIZE, 3. PMC pass WRITE_SIZE         -> profiles/pmc_traffic.json (tools/pmc_traffic.py)
#   4. PMC pass of SQ counters (issue/wait breakdown)     -> gpurun_out/pmc_sq_<tag>/
# Counters are collected in their own runs with --kernel-trace/--stats only (never with
# sys/runtime traces). Each GPU step has its own time limit; a crash-type exit ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANT=${VARIANT:-cull}
TAG=${TAG:-$VARIANT}
BENCH_ARGS=${BENCH_ARGS:-}
KERNEL_RE=${KERNEL_RE:-Trace}
WORKLOAD=${WORKLOAD:-soup-100k 1920x1080 1spp}
run() {
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
    return $rc
}
BENCH=(python3 bench.py --steps 20 --warmup 3 --variant "$VARIANT" --no-cpu-baseline --no-e2e $BENCH_ARGS)
run "prof_stats_$TAG" 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$TAG" -o run --output-format csv -- "${BENCH[@]}"
run "pmc_fetch_$TAG" 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KERNEL_RE" -d "gpurun_out/pmc_fetch_$TAG" -o run --output-format csv -- "${BENCH[@]}"
run "pmc_write_$TAG" 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KERNEL_RE" -d "gpurun_out/pmc_write_$TAG" -o run --output-format csv -- "${BENCH[@]}"
python3 tools/pmc_traffic.py --key "$WORKLOAD|$VARIANT" --kernel "$KERNEL_RE" --fetch "gpurun_out/pmc_fetch_$TAG" --write "gpurun_out/pmc_write_$TAG" --out gpurun_out/pmc_traffic.json
if [ -n "${SQ_COUNTERS:-}" ]; then
    run "pmc_sq_$TAG" 600 rocprofv3 --pmc $SQ_COUNTERS --kernel-include-regex "$KERNEL_RE" -d "gpurun_out/pmc_sq_$TAG" -o run --output-format csv -- "${BENCH[@]}"
fi
echo done
