#!/usr/bin/env python3
"""Per-kernel HBM-side bytes per dispatch from two rocprofv3 --pmc passes over every kernel
(FETCH_SIZE x 2 x 1024 and WRITE_SIZE x 1024, the MI355X_MICROARCH.md corrections, as
tools/pmc_traffic.py), averaged over each kernel's dispatches.

    python tools/pmc_kernels.py gpurun_out/pmc_fetch_all gpurun_out/pmc_write_all
"""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path


def load(d, counter):
    per = defaultdict(dict)
    for f in sorted(Path(d).rglob("*counter_collection.csv")):
        for r in csv.DictReader(open(f, newline="")):
            if r.get("Counter_Name") != counter:
                continue
            m = re.search(r"(\w+)(<[^(]*)?\(", r.get("Kernel_Name", ""))
            name = m.group(1) if m else r.get("Kernel_Name", "")[:40]
            key = (r.get("Dispatch_Id"), r.get("Agent_Id"))
            per[name][key] = per[name].get(key, 0.0) + float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in per.items()}


fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE")
for name in sorted(set(fetch) | set(write), key=lambda n: -(fetch.get(n, (0, 0))[0] * 2 + write.get(n, (0, 0))[0])):
    f, nf = fetch.get(name, (0.0, 0))
    w, nw = write.get(name, (0.0, 0))
    print(f"{name:28s} dispatches {max(nf, nw):5d}  read {f * 2 * 1024 / 1e6:8.2f} MB  write {w * 1024 / 1e6:8.2f} MB")
