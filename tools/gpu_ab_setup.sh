#!/bin/bash
# A/B of the setup launches under trace load: work-order block size (lib_ab/{base,ord256,ord512})
# x setup stream (SRT_SETUP_STREAM 0 / 1 / 2): the default bench line (value, stage times) and the
# one-frame-in-flight latency (queues 1, one frame per step).
source "$(dirname "$0")/gpu_lib.sh"
LIBS=${LIBS:-base ord256 ord512}
MODES=${MODES:-0 1 2}
for lib in $LIBS; do
  for m in $MODES; do
    SRT_LIB=simpleraytracer_amd/lib_ab/$lib/libModelRunner.so SRT_SETUP_STREAM=$m \
      run ab_${lib}_s$m 200 python bench.py --no-extras --no-cpu-baseline --steps 100 || exit 1
    SRT_LIB=simpleraytracer_amd/lib_ab/$lib/libModelRunner.so SRT_SETUP_STREAM=$m \
      run ab_${lib}_s${m}_q1 200 python bench.py --no-extras --no-cpu-baseline --steps 1000 --queues 1 --frames-per-step 1 || exit 1
  done
done
for lib in $LIBS; do for m in $MODES; do
  python - "$lib" "$m" <<'PY'
import json, sys
lib, m = sys.argv[1:]
d = json.loads(open(f"gpurun_out/ab_{lib}_s{m}.log").read().strip().splitlines()[-1])
q = json.loads(open(f"gpurun_out/ab_{lib}_s{m}_q1.log").read().strip().splitlines()[-1])
s = d["stages_ms"]
print(f"{lib:7s} setup_stream={m}: value {d['value']:9.1f}  q1 {q['value']:8.1f}  stages {s['prepare']*1e3:.1f}/{s['bin']*1e3:.1f}/{s['trace_kernel']*1e3:.1f} us  verified {d['verified']}")
PY
done; done
