#!/bin/bash
# Kernel statistics of a P = 8 rank simulation for each library of VARIANTS (lib_ab/<name> or
# "product"), to see which kernel an A/B difference comes from.
source "$(dirname "$0")/gpu_lib.sh"
for v in ${VARIANTS:-c_share c_tile}; do
    lib=""; [ $v != product ] && lib=simpleraytracer_amd/lib_ab/$v/libModelRunner.so
    SRT_LIB=$lib run pab_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pab_$v -o run --output-format csv -- \
        python3 tools/rank_sim.py --ranks ${PS:-8} --steps 20
    echo "== $v"; python3 tools/kernel_stats.py gpurun_out/pab_$v | grep -E "Kernel"
done
