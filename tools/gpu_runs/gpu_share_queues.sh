#!/bin/bash
# Share exchange with as many frame queues as ranks (every compositor busy at once in the real job:
# a batch's senders cannot run more than Q batches ahead of its compositor), against all-to-all at
# the bench's 256-frame batches: rank simulation at P = 4, 8.
source "$(dirname "$0")/gpu_lib.sh"
for cfg in ${CFGS:-"4 4 64 share" "4 2 256 alltoall" "4 2 64 alltoall" "8 8 32 share" "8 4 32 share" "8 2 256 alltoall" "8 2 64 alltoall"}; do
    set -- $cfg
    n=sq_p$1_q$2_b$3_$4
    run $n 300 python3 tools/rank_sim.py --ranks $1 --queues $2 --batch $3 --exchange $4 --warmup 8 --steps 16
    echo "P=$1 Q=$2 batch=$3 $4 $(grep -o '"us_per_frame": {[^}]*}' gpurun_out/$n.log | head -1)"
done
