#!/bin/bash
# Round 6: a recomputing trace with its entry-holding waves walking LIGHT packets fewer per window
# (SRT_RC_LIGHT), so they build the next batch's records while the other waves walk: the headline
# (driver shape, 2 queues) with records recomputed for every launch, against stored records, two rounds.
source "$(dirname "$0")/gpu_lib.sh"
L=simpleraytracer_amd/lib_exp
B="python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-e2e"
for r in 1 2; do
  SRT_LIB=$L/light0/libModelRunner.so SRT_TRACE_RECORDS=stored run st_$r 150 $B
  line="round $r: stored $(grep -o '"value": [0-9.]*' gpurun_out/st_$r.log | head -1)"
  for b in 0 1 2 4 8; do
    SRT_LIB=$L/light$b/libModelRunner.so SRT_TRACE_RECORDS=recompute run rc${b}_$r 150 $B
    line="$line | rc light$b $(grep -o '"value": [0-9.]*' gpurun_out/rc${b}_$r.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/rc${b}_$r.log | head -1)"
  done
  echo "$line"
done
