#!/bin/bash
# Round 6: the compositor's deferred shading carried by the next trace launch (SRT_CARRY_SHADE): engine
# parity tests, rank simulation carried / own launch (rotated all-to-all P = 2, 8; share P = 8), a bench
# line and the fake-device N = 2 line.
source "$(dirname "$0")/gpu_lib.sh"
run pytest_engine 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "engine or trace_batch or shade"
for rep in 1 2; do
    SRT_CARRY_SHADE=1 run rs_carry_$rep 300 python3 tools/rank_sim.py --exchange alltoall --rows rotated --ranks 2,4,8
    SRT_CARRY_SHADE=0 run rs_own_$rep 300 python3 tools/rank_sim.py --exchange alltoall --rows rotated --ranks 2,4,8
done
run bench 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e
run fake2 400 env SRT_BENCH_ONE_DEVICE=1 python bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e
for f in gpurun_out/rs_carry_?.log gpurun_out/rs_own_?.log; do echo "$f $(grep -o '"P": [0-9]*\|"slowest_us": [0-9.]*' $f | tr '\n' ' ')"; done
grep -o '"value": [0-9.]*' gpurun_out/bench.log gpurun_out/fake2.log
