#!/usr/bin/env python3
"""Summarise a gpurun_out/ directory: bench JSON lines (value, single queue, stages) and
rocprofv3 kernel stats (calls, mean us, share) of every prof_* subdirectory."""
import csv
import json
import sys
from pathlib import Path

root = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
for f in sorted(root.glob("bench*.log")):
    lines = [x for x in f.read_text().splitlines() if x.startswith("{")]
    if not lines:
        print(f"{f.name}: no JSON line")
        continue
    d = json.loads(lines[-1])
    sq = d.get("single_queue", {}).get("mrays_per_s")
    st = d.get("stages_ms", {})
    print(f"{f.name}: value {d['value']:.0f} {d['unit']} ms/step {d['ms_per_step']} single {sq} "
          f"prep {st.get('prepare')} bin {st.get('bin')} trace {st.get('trace_kernel')}")
    for k in ("bands", "frames", "offsets_random", "c2_cornell"):
        if k in d:
            print(f"   {k}: {json.dumps(d[k])[:300]}")
for f in sorted(root.glob("*/run_kernel_stats.csv")):
    print(f"== {f.parent.name}")
    for x in csv.DictReader(open(f)):
        print(f"   {x['Name'][:58]:58s} {x['Calls']:>6} {float(x['AverageNs']) / 1000:9.2f} us {float(x['Percentage']):5.1f}%")
