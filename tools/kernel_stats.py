#!/usr/bin/env python3
"""Short table of a rocprofv3 --stats run: kernel, calls, mean / min us, total ms.

    python tools/kernel_stats.py gpurun_out/prof_q1 [more dirs]
"""
import csv
import glob
import re
import sys

for d in sys.argv[1:]:
    files = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)
    if not files:
        print(f"== {d}: no kernel_stats.csv")
        continue
    print(f"== {d}")
    for r in csv.DictReader(open(files[0])):
        m = re.search(r"(\w+)(<[^(]*)?\(", r["Name"])
        n = m.group(1) if m else r["Name"][:40]
        print(f"{n:28s} calls {r['Calls']:>6s} avg {float(r['AverageNs']) / 1e3:9.2f} us  min "
              f"{float(r['MinNs']) / 1e3:9.2f}  tot {float(r['TotalDurationNs']) / 1e6:9.3f} ms")
