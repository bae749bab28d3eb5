#!/bin/bash
# GPU tests, a bench A/B of LIBS and the band simulation of each library (C3, and C5 when C5=1).
LIBS="${LIBS:-base prev}" bash tools/gpu_runs/gpu_ab_check.sh || exit $?
source "$(dirname "$0")/gpu_lib.sh"
for name in ${LIBS:-base prev}; do
    if [ "$name" = base ]; then unset SRT_LIB; else export SRT_LIB=simpleraytracer_amd/lib_ab/$name/libModelRunner.so; fi
    run band_sim_$name 300 python tools/band_sim.py
    if [ "${C5:-0}" = 1 ]; then
        run band_c5_$name 600 python tools/band_sim.py --width 3840 --height 2160 --triangles 1000000 --steps 200 --warmup 5
    fi
done
echo done
