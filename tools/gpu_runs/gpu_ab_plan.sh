#!/bin/bash
# Work plan A/B (render.hip WorkPlan): the GPU parity tests of the plan, then the default bench
# (headline + single queue) for the previous library (lib_ab/old, if built) and the product
# library under SRT_WORK_PLAN = auto / reuse / order, twice in interleaved order; then the rank
# simulation at P = 8 under auto and reuse.
source "$(dirname "$0")/gpu_lib.sh"
run plan_tests 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread \
    -k "work_plan or split_items or trace_batch or setup_state or cull_modes or interleaved"
for rep in 1 2; do
    for v in ${VARIANTS:-old auto reuse order}; do
        lib=""
        mode=$v
        if [ "$v" = old ]; then
            [ -f simpleraytracer_amd/lib_ab/old/libModelRunner.so ] || continue
            lib=simpleraytracer_amd/lib_ab/old/libModelRunner.so
            mode=auto
        fi
        SRT_LIB=$lib SRT_WORK_PLAN=$mode run ab_${v}_$rep 200 python3 bench.py --steps ${STEPS:-200} --warmup 10 \
            --no-cpu-baseline --no-e2e --brute-steps 0
        echo "$v#$rep $(grep -o '"value": [0-9.]*\|"single_queue": {"mrays_per_s": [0-9.]*\|"kernel_ms": [0-9.]*\|"bin": [0-9.]*' gpurun_out/ab_${v}_$rep.log | tr '\n' ' ')"
    done
done
for v in auto reuse; do
    SRT_WORK_PLAN=$v run rank_sim_$v 300 python3 tools/rank_sim.py --ranks 1,8
done
