#!/usr/bin/env python3
"""The main fields of a bench.py JSON line (the last one in the file).

    python tools/bench_summary.py gpurun_out/bench.log
"""
import json
import sys

line = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(line)
print(f"value {d['value']:.1f} {d['unit']}  ms/frame {d['ms_per_frame'] * 1e3:.2f} us  verified {d.get('verified')}  "
      f"roofline frac {d['roofline']['frac']}  stages {d['stages_ms']['prepare']*1e3:.2f}/{d['stages_ms']['bin']*1e3:.2f}/"
      f"{d['stages_ms']['trace_kernel']*1e3:.2f} us")
for k in ("single_queue", "rotating_inputs", "offsets_random", "c2_cornell", "variant_bvh", "e2e_ml_api", "frames"):
    if k in d:
        print(f"  {k}: {d[k].get('mrays_per_s')}")
