#!/bin/bash
# Where the per-frame setup's cost goes at C3:
#  * q1b8: one queue, 8-frame launches, kernel trace (each batched stage alone on the chip);
#  * setup_only: the frame pipeline with the trace kernel returning at once (make exp
#    EXP_NAME=setup EXP_FLAGS=-DSRT_EXP_SETUP_ONLY, copied to lib_ab/setup): setup's throughput cost;
#  * exp_N: the diag build's PrepareBinKernel with SRT_EXP bit N (2: no tile tests / lists,
#    4: no global list reservations, 512: no screen-box solve), one frame per dispatch.
source "$(dirname "$0")/gpu_lib.sh"
Q="--steps 50 --warmup 5 --queues 1 --batch 1 --no-extras --no-cpu-baseline"
run q1b8 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q1b8 -o run --output-format csv -- \
    python3 bench.py --steps 400 --warmup 8 --queues 1 --batch 8 --no-extras --no-cpu-baseline
SRT_LIB=simpleraytracer_amd/lib_ab/setup/libModelRunner.so run setup_only 300 python bench.py --no-extras --no-cpu-baseline
for e in ${EXPS:-0 2 4 512}; do
    SRT_LIB=simpleraytracer_amd/lib_diag/libModelRunner.so SRT_EXP=$e run exp_$e 200 rocprofv3 --kernel-trace --stats \
        -d gpurun_out/exp_$e -o run --output-format csv -- python3 bench.py $Q
done
echo done
