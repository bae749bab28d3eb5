#!/bin/bash
# P = 2 share exchange: rank simulation over the compositor's rows per cycle (k) and frame queues.
source "$(dirname "$0")/gpu_lib.sh"
for q in ${QS:-2 4}; do
    for k in ${KS:-2 4 8 16}; do
        run ss_q${q}_k$k 300 python3 tools/rank_sim.py --ranks 2 --exchange share --share $k --queues $q
        echo "q=$q k=$k $(grep -o '"us_per_frame": {[^}]*}\|"link_us_per_frame": [0-9.]*' gpurun_out/ss_q${q}_k$k.log | head -2 | tr '\n' ' ')"
    done
done
