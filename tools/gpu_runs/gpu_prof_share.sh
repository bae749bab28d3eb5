#!/bin/bash
# Kernel statistics of one-queue rank simulations (no overlap between a rank's kernels, so the
# rocprofv3 averages are each kernel's own time): P = 1, P = 2 share and all-to-all, P = 8.
source "$(dirname "$0")/gpu_lib.sh"
for cfg in "1 alltoall" "2 share" "2 alltoall" "8 alltoall"; do
    set -- $cfg
    n=ps_$1_$2
    run $n 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$n -o run --output-format csv -- \
        python3 tools/rank_sim.py --ranks $1 --exchange $2 --queues 1 --steps 10
    python3 tools/kernel_stats.py gpurun_out/$n
    grep '^{"P"' gpurun_out/$n.log || true
done
