#!/bin/bash
# A/B throughput of experiment libraries (make exp EXP_NAME=...): the default bench frame loop
# (three frame queues + single queue), no CPU baseline / e2e / brute-force legs, each library
# run twice in interleaved order. LIBS = space-separated entries NAME[@VAR=VAL,VAR=VAL]: NAME an
# exp build or "base" (the product lib), the optional env settings applied to that run only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
    for entry in ${LIBS:-base}; do
        name=${entry%%@*}
        envs=""
        [ "$entry" != "$name" ] && envs=$(echo "${entry#*@}" | tr ',' ' ')
        if [ "$name" = base ]; then lib=""; else lib="simpleraytracer_amd/lib_exp/$name/libModelRunner.so"; fi
        name=$(echo "$entry" | tr '@=,' '___')
        env SRT_LIB=$lib $envs timeout -k 10 120 python3 bench.py --steps ${STEPS:-2000} --warmup 10 --no-cpu-baseline --no-e2e \
            --brute-steps 0 ${BENCH_ARGS:-} > gpurun_out/ab_${name}_$rep.log 2>&1 || { echo "rc=$? $name"; exit 1; }
        echo "$name#$rep $(grep -o '"value": [0-9.]*\|"single_queue": {"mrays_per_s": [0-9.]*\|"trace_kernel": [0-9.]*' gpurun_out/ab_${name}_$rep.log | tr '\n' ' ')"
    done
done
