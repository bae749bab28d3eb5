#!/bin/bash
# Frame-pipeline shape at N = 1: bench value for each "QUEUES:BATCH" in $SHAPES (default 3:8).
source "$(dirname "$0")/gpu_lib.sh"
for sh in ${SHAPES:-3:8}; do
    q=${sh%%:*}; b=${sh#*:}
    run pipe_q${q}_b${b} 200 python bench.py --no-extras --no-cpu-baseline --queues $q --batch $b
done
echo done
