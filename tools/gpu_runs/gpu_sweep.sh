#!/bin/bash
# Sweep of library env settings: for each "NAME:VAR=V,VAR2=V2" entry of $CFGS, a bench line
# (main value + single queue, no extras), a one-queue rocprof pass and (BANDSIM=1) the band
# simulation.
source "$(dirname "$0")/gpu_lib.sh"
for cfg in $CFGS; do
    name=${cfg%%:*}
    envs=${cfg#*:}
    (
        IFS=','
        for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
        run bench_$name 300 python bench.py --no-extras --no-cpu-baseline --steps ${STEPS:-3000}
        run prof_$name 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv -- \
            python3 bench.py --steps 50 --warmup 5 --queues 1 --no-extras --no-cpu-baseline
        if [ "${BANDSIM:-0}" = 1 ]; then
            run band_sim_$name 300 python tools/band_sim.py --steps 1000
        fi
    ) || exit $?
done
echo done
