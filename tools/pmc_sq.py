#!/usr/bin/env python3
"""Turn a rocprofv3 --pmc pass of SQ counters into per-launch means (bench.py "valu_issue").

    python tools/pmc_sq.py --key "soup-100k 1920x1080 1spp|cull" --dir gpurun_out/pmc_sq \
        [--kernel TraceCullKernel] [--out profiles/pmc_sq.json]

Every counter of the pass is averaged over the dispatches of the kernel; SQ_INSTS_VALU is also
stored as sq_insts_valu_per_launch. VALU issue time = SQ_INSTS_VALU x 2 cycles per wave64
instruction (SIMD-32, MI355X_MICROARCH.md "Wave scheduling") / (1024 SIMDs x 2.4 GHz).
SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / SQ_WAIT_* are reported as read (their units are not
calibrated here). Result merged into --out under --key.
"""
from __future__ import annotations

import argparse
import csv
import json
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", required=True)
    ap.add_argument("--dir", type=Path, required=True)
    ap.add_argument("--kernel", default="TraceCullKernel")
    ap.add_argument("--out", type=Path, default=REPO / "profiles" / "pmc_sq.json")
    ap.add_argument("--source", default="")
    ap.add_argument("--largest-grid", action="store_true", help="only the dispatches of the largest grid")
    a = ap.parse_args()
    per, grid = {}, {}
    for f in sorted(a.dir.rglob("*counter_collection.csv")):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                if a.kernel not in r.get("Kernel_Name", ""):
                    continue
                key = (r["Counter_Name"], r.get("Dispatch_Id"), r.get("Agent_Id"))
                per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
                grid[key] = int(r.get("Grid_Size") or 0)
    if per and a.largest_grid:
        g = max(grid.values())
        per = {k: v for k, v in per.items() if grid[k] == g}
    if not per:
        raise SystemExit(f"no {a.kernel} counters under {a.dir}")
    sums, counts = {}, {}
    for (name, _, _), v in per.items():
        sums[name] = sums.get(name, 0.0) + v
        counts[name] = counts.get(name, 0) + 1
    entry = {name: sums[name] / counts[name] for name in sorted(sums)}
    entry["dispatches"] = max(counts.values())
    entry["kernel"] = a.kernel
    if "SQ_INSTS_VALU" in entry:
        entry["sq_insts_valu_per_launch"] = entry["SQ_INSTS_VALU"]
        entry["valu_issue_us"] = entry["SQ_INSTS_VALU"] * 2 / (1024 * 2.4e9) * 1e6
    if a.source:
        entry["source"] = a.source
    out = json.loads(a.out.read_text()) if a.out.exists() else {}
    out[a.key] = entry
    a.out.write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print(json.dumps({a.key: entry}, indent=1))


if __name__ == "__main__":
    main()
