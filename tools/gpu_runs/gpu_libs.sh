#!/bin/bash
# A/B of library builds: for each NAME in $LIBS ("base" = the product library, else
# simpleraytracer_amd/lib_exp/NAME from `make exp`), a bench line and a one-queue rocprof pass.
source "$(dirname "$0")/gpu_lib.sh"
for name in $LIBS; do
    if [ "$name" = base ]; then unset SRT_LIB; else export SRT_LIB=simpleraytracer_amd/${LIBDIR_AB:-lib_exp}/$name/libModelRunner.so; fi
    run bench_$name 300 python bench.py --no-extras --no-cpu-baseline ${BENCH_ARGS:-}
    run prof_$name 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv -- \
        python3 bench.py --steps 50 --warmup 5 --queues 1 --no-extras --no-cpu-baseline ${BENCH_ARGS:-}
done
echo done
