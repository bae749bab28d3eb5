#!/bin/bash
# Diag-build block timeline of one C3 trace (tools/diag_cull.py), then the product library with
# one queue and 8-frame launches under rocprofv3 (each batched stage alone on the chip).
source "$(dirname "$0")/gpu_lib.sh"
SRT_LIB=simpleraytracer_amd/lib_diag/libModelRunner.so DIAG_RAW=gpurun_out/diag_raw.npy run diag_uniform 120 python tools/diag_cull.py
run q1b8 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q1b8 -o run --output-format csv -- \
    python3 bench.py --steps 400 --warmup 8 --queues 1 --batch 8 --no-extras --no-cpu-baseline
echo done
