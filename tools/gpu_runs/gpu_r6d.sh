#!/bin/bash
# Round 6: upper bound of hiding the compositor's deferred shading (rank simulation with the shading
# skipped: lib_ab/noshade), and the bench line with its new C5 one-GPU leg.
source "$(dirname "$0")/gpu_lib.sh"
run rs_base 300 python3 tools/rank_sim.py --exchange alltoall --rows rotated --ranks 2,8
SRT_LIB=simpleraytracer_amd/lib_ab/noshade/libModelRunner.so run rs_noshade 300 \
    python3 tools/rank_sim.py --exchange alltoall --rows rotated --ranks 2,8
run bench_c5 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --brute-steps 0
for f in gpurun_out/rs_base.log gpurun_out/rs_noshade.log; do echo "$f $(grep -o '"P": [0-9]*\|"slowest_us": [0-9.]*' $f | tr '\n' ' ')"; done
python3 -c "import json;d=json.loads([l for l in open('gpurun_out/bench_c5.log') if l.startswith('{')][-1]);print(json.dumps(d.get('c5_one_gpu')))"
