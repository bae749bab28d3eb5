#!/bin/bash
# Round 6: record modes in the product (render.h RecordMode): the GPU suite and smoke at the code, then
# alternating A/B of the recomputed records against stored ones (SRT_TRACE_RECORDS) where the policy picks
# recompute -- one frame in flight, the C5 leg's one-queue shape -- and the headline (stored either way).
source "$(dirname "$0")/gpu_lib.sh"
run rm_pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
grep -E "passed|failed" gpurun_out/rm_pytest.log | tail -1
run rm_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
B="python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e"
S="python3 bench.py --steps 400 --warmup 20 --frames-per-step 1 --queues 1 --launch 1 --no-extras --no-cpu-baseline --no-e2e"
C5="python3 bench.py --triangles 1000000 --width 3840 --height 2160 --frames-per-step 64 --steps 10 --warmup 2 --queues 1 --launch 16 --no-extras --no-cpu-baseline --no-e2e"
for r in 1 2; do
  run rm_h_$r 150 $B
  for m in policy stored; do
    v=$([ $m = policy ] && echo "" || echo $m)  # empty: the product's policy (one queue: recompute)
    SRT_TRACE_RECORDS=$v run rm_s_${m}_$r 150 $S
    SRT_TRACE_RECORDS=$v run rm_c5_${m}_$r 200 $C5
  done
  echo "round $r: headline $(grep -o '"value": [0-9.]*' gpurun_out/rm_h_$r.log) single policy $(grep -o '"value": [0-9.]*' gpurun_out/rm_s_policy_$r.log) stored $(grep -o '"value": [0-9.]*' gpurun_out/rm_s_stored_$r.log) C5 policy $(grep -o '"value": [0-9.]*' gpurun_out/rm_c5_policy_$r.log) stored $(grep -o '"value": [0-9.]*' gpurun_out/rm_c5_stored_$r.log)"
done
