#!/bin/bash
# Split-part merge A/B: lib_ab/atomic (SRT_SPLIT_ATOMIC=1: atomic maxima into one slice per part)
# against the product library: its parity tests, the one-queue kernel statistics and the default
# bench (headline + single queue), twice interleaved.
source "$(dirname "$0")/gpu_lib.sh"
A=simpleraytracer_amd/lib_ab/atomic/libModelRunner.so
SRT_LIB=$A run atomic_tests 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_full.py -m gpu -q -x \
    --timeout 200 --timeout-method thread -k "split or work_plan or cull_modes or c3 or full or trace_batch or interleaved"
for v in product atomic; do
    lib=""; [ $v = atomic ] && lib=$A
    SRT_LIB=$lib run q1_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q1_$v -o run --output-format csv -- \
        python3 bench.py --steps 300 --warmup 20 --queues 1 --frames-per-step 1 --no-extras --no-cpu-baseline
    python3 tools/kernel_stats.py gpurun_out/q1_$v | grep -E "TraceCull|PrepareBin|WorkOrder"
done
for rep in 1 2; do
    for v in product atomic; do
        lib=""; [ $v = atomic ] && lib=$A
        SRT_LIB=$lib run ab_${v}_$rep 200 python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-e2e --brute-steps 0
        echo "$v#$rep $(grep -o '"value": [0-9.]*\|"single_queue": {"mrays_per_s": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/ab_${v}_$rep.log | tr '\n' ' ')"
    done
done
