#!/bin/bash
# The driver's 20-step shape at N = 1 for queue / batch pairs in $SHAPES ("Q:B", B 0 = auto).
source "$(dirname "$0")/gpu_lib.sh"
for sh in ${SHAPES:-3:0 4:0 5:0 3:4 2:0}; do
    q=${sh%%:*}; b=${sh#*:}
    run short_q${q}_b${b} 200 python bench.py --no-extras --no-cpu-baseline --steps 20 --warmup 5 --queues $q --batch $b
done
echo done
