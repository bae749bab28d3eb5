#!/bin/bash
# Frame queues at N = 1: the default bench (3000 steps) and the driver's 20-step shape for each
# queue count in $QS.
source "$(dirname "$0")/gpu_lib.sh"
for q in ${QS:-1 2 3}; do
    run qb_q$q 300 python bench.py --no-extras --no-cpu-baseline --queues $q
    run qd_q$q 200 python bench.py --no-extras --no-cpu-baseline --queues $q --steps 20 --warmup 5
done
echo done
