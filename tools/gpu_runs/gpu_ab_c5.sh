#!/bin/bash
# A/B of library builds (LIBS in lib_ab/) at C5 (1M triangles, 3840 x 2160): one-frame-in-flight kernel
# stats and the default-shape bench line (no extras).
source "$(dirname "$0")/gpu_lib.sh"
C5="--width 3840 --height 2160 --triangles 1000000"
for name in $LIBS; do
    L=simpleraytracer_amd/lib_ab/$name/libModelRunner.so
    SRT_LIB=$L run c5q1_$name 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c5q1_$name -o run --output-format csv -- \
        python3 bench.py $C5 --steps 30 --warmup 3 --queues 1 --frames-per-step 1 --no-extras --no-cpu-baseline || exit 1
    SRT_LIB=$L run c5_$name 300 python bench.py $C5 --steps 20 --warmup 2 --no-extras --no-cpu-baseline || exit 1
done
for name in $LIBS; do
    echo "== $name"; python3 tools/bench_summary.py gpurun_out/c5_$name.log; python3 tools/kernel_stats.py gpurun_out/c5q1_$name | grep -E "Cull|Bin|Order"
done
