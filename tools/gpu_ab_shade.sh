#!/bin/bash
# A/B of deferred-shading builds (LIBS in lib_ab/): whole frames traced to ids and shaded by
# ShadeIdsKernel (SRT_DEFER_SHADE=1, verified bit for bit), and the P = 8 rank simulation.
source "$(dirname "$0")/gpu_lib.sh"
for name in $LIBS; do
    SRT_DEFER_SHADE=1 SRT_LIB=simpleraytracer_amd/lib_ab/$name/libModelRunner.so run defer_$name 300 \
        python bench.py --no-extras --no-cpu-baseline --steps 50
    SRT_LIB=simpleraytracer_amd/lib_ab/$name/libModelRunner.so run rank8_$name 300 python tools/rank_sim.py --ranks 8
done
for name in $LIBS; do
    echo "== $name"; python3 tools/bench_summary.py gpurun_out/defer_$name.log; grep '"P": 8' gpurun_out/rank8_$name.log
done
