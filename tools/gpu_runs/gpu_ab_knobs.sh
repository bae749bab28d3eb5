#!/bin/bash
# Throughput A/B of compile-time knobs (make ab AB_NAME=... AB_FLAGS=...): the driver-shape bench for
# the product library and each lib_ab build, alternating, twice.
source "$(dirname "$0")/gpu_lib.sh"
for rep in 1 2; do
    run knob_base_$rep 300 python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline
    for lib in ${LIBS:-$(ls simpleraytracer_amd/lib_ab)}; do
        SRT_LIB=simpleraytracer_amd/lib_ab/$lib/libModelRunner.so run knob_${lib}_$rep 300 python3 bench.py --steps 20 \
            --warmup 5 --no-extras --no-cpu-baseline
    done
done
python3 tools/bench_summary.py gpurun_out/knob_*.log
