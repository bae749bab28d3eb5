#!/bin/bash
# A/B of library builds on the bench line: for each NAME in $LIBS (lib_ab/NAME, `make ab`), one
# bench.py run (value, stage times; BENCH_ARGS appended), summarised at the end.
source "$(dirname "$0")/gpu_lib.sh"
for name in $LIBS; do
    SRT_LIB=simpleraytracer_amd/lib_ab/$name/libModelRunner.so run ab_$name 300 \
        python bench.py --no-extras --no-cpu-baseline --steps ${STEPS:-50} ${BENCH_ARGS:-}
done
for name in $LIBS; do
    echo "== $name"; python3 tools/bench_summary.py gpurun_out/ab_$name.log
done
