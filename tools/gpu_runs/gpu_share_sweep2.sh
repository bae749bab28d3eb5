#!/bin/bash
# Share exchange at larger k (P = 2) and at P = 4, 8 (frame queues a multiple of P or not),
# against all-to-all.
source "$(dirname "$0")/gpu_lib.sh"
for cfg in "2 2 32" "2 2 64" "4 2 0" "4 2 16" "4 4 16" "8 2 0" "8 2 16" "8 8 16"; do
    set -- $cfg
    ex=share; [ $3 = 0 ] && ex=alltoall
    n=s2_p$1_q$2_k$3
    run $n 300 python3 tools/rank_sim.py --ranks $1 --exchange $ex --share $3 --queues $2
    echo "P=$1 q=$2 k=$3 $(grep -o '"us_per_frame": {[^}]*}\|"link_us_per_frame": [0-9.]*' gpurun_out/$n.log | head -2 | tr '\n' ' ')"
done
