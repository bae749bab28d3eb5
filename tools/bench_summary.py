#!/usr/bin/env python3
"""The main fields of a bench.py JSON line (the last one in each file).

    python tools/bench_summary.py gpurun_out/bench.log [more logs]
"""
import json
import sys


def summary(path):
    lines = [x for x in open(path) if x.startswith("{")]
    if not lines:
        print(f"== {path}: no JSON line")
        return
    d = json.loads(lines[-1])
    if d.get("value") is None:
        print(f"== {path}: error {d.get('error')}")
        return
    print(f"== {path}")
    show(d)


def show(d):
    roof = d["roofline"]
    print(f"value {d['value']:.1f} {d['unit']}  ms/frame {d['ms_per_frame'] * 1e3:.2f} us  verified {d.get('verified')}  "
          f"roofline frac {roof['frac']} (trace {roof['kernel_ms'] * 1e3:.1f} us / {roof.get('frames_per_launch', 1)} "
          f"frames)")
    st = d["stages_ms"]
    print(f"  single-frame stages {st['prepare'] * 1e3:.2f}/{st['bin'] * 1e3:.2f}/{st['trace_kernel'] * 1e3:.2f} us")
    for k in ("single_queue", "rotating_inputs", "offsets_random", "c2_cornell", "variant_bvh", "e2e_ml_api", "frames"):
        if k in d:
            print(f"  {k}: {d[k].get('mrays_per_s')}")


for path in sys.argv[1:]:
    summary(path)
