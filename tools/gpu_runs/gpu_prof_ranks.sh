#!/bin/bash
# Kernel statistics of the rank simulation (tools/rank_sim.py) at P = 2 and P = 8: per-kernel time
# of one rank's stream (rocprofv3 --kernel-trace --stats), to split a rank's frame into setup,
# trace and compositing.
source "$(dirname "$0")/gpu_lib.sh"
for P in ${PS:-2 8}; do
    run prof_rank$P 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rank$P -o run --output-format csv -- \
        python3 tools/rank_sim.py --ranks $P --steps 20
    python3 tools/kernel_stats.py gpurun_out/prof_rank$P
done
