#!/bin/bash
# Env / option sweep of the default bench line: CFGS="name:VAR=V,VAR2=V2[:bench args] ..." (one run
# each, value and stage times summarised at the end).
source "$(dirname "$0")/gpu_lib.sh"
for cfg in $CFGS; do
  name=${cfg%%:*}; rest=${cfg#*:}; envs=${rest%%:*}; args=""
  [[ $rest == *:* ]] && args=${rest#*:}
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --steps ${STEPS:-100} ${args//,/ } \
      > gpurun_out/sw_$name.log 2>&1; rc=$?
  echo "$name rc=$rc"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
for cfg in $CFGS; do
  name=${cfg%%:*}
  python - "$name" <<'PY'
import json, sys
n = sys.argv[1]
try:
    d = json.loads(open(f"gpurun_out/sw_{n}.log").read().strip().splitlines()[-1])
    s = d["stages_ms"]
    print(f"{n:14s} value {d['value']:9.1f}  ms/frame {d['ms_per_frame']*1e3:6.2f} us  stages {s['prepare']*1e3:.1f}/{s['bin']*1e3:.1f}/{s['trace_kernel']*1e3:.1f} us  verified {d['verified']}")
except Exception as e:
    print(n, "failed", e)
PY
done
