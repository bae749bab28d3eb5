#!/bin/bash
# Share exchange vs all-to-all with balanced batch counts (warmup and timed batches multiples of P):
# rank simulation at P = 2, 4, 8 over the compositor's rows per cycle (k; 0 = all-to-all).
source "$(dirname "$0")/gpu_lib.sh"
for cfg in ${CFGS:-"2 16" "2 32" "4 0" "4 8" "4 16" "4 32" "8 0" "8 8" "8 16" "8 32"}; do
    set -- $cfg
    ex=share; [ $2 = 0 ] && ex=alltoall
    n=s3_p$1_k$2
    run $n 300 python3 tools/rank_sim.py --ranks $1 --exchange $ex --share $2 --warmup 8 --steps 32 ${EXTRA:-}
    echo "P=$1 k=$2 $(grep -o '"us_per_frame": {[^}]*}\|"link_us_per_frame": [0-9.]*' gpurun_out/$n.log | head -2 | tr '\n' ' ')"
done
