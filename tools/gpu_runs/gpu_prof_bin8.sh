#!/bin/bash
# PrepareBinKernel of a P = 8 rank under the diag build's SRT_EXP knock-outs (timing only, the
# frames are not valid): 0 = as built, 512 = no screen-box solve, 1 = no tile ranges (no binning),
# 513 = neither -- rocprofv3 kernel statistics of the rank simulation.
source "$(dirname "$0")/gpu_lib.sh"
for e in ${EXPS:-0 512 1 513}; do
    SRT_LIB=simpleraytracer_amd/lib_diag/libModelRunner.so SRT_EXP=$e run bin8_$e 200 rocprofv3 --kernel-trace --stats \
        -d gpurun_out/bin8_$e -o run --output-format csv -- python3 tools/rank_sim.py --ranks 8 --steps 10
    echo "exp $e"; python3 tools/kernel_stats.py gpurun_out/bin8_$e | grep -E "PrepareBin|TraceCull|TileInfo|ShadeIds"
done
