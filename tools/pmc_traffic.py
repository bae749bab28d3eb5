#!/usr/bin/env python3
"""Turn rocprofv3 --pmc counter CSVs into HBM bytes per trace launch (bench.py "traffic").

    python tools/pmc_traffic.py --key "soup-100k 1920x1080 1spp|cull" \
        --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write [--kernel TraceCullKernel]

FETCH_SIZE and WRITE_SIZE come from separate passes (they do not fit one TCC pass together,
MI355X_MICROARCH.md "rocprofv3 PMC slots"). Corrections from MI355X_MICROARCH.md "HBM": both
counters are in KiB (x1024), and on gfx950 FETCH_SIZE reports half of the bytes of a wide
coalesced streaming read, so it is doubled. The per-dispatch values of every dispatch of the
kernel are averaged. Result merged into profiles/pmc_traffic.json under --key.
"""
from __future__ import annotations

import argparse
import csv
import json
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def counter_rows(d: Path):
    files = sorted(d.rglob("*counter_collection.csv"))
    if not files:
        raise SystemExit(f"no *counter_collection.csv under {d}")
    for f in files:
        with open(f, newline="") as fh:
            yield from csv.DictReader(fh)


def per_dispatch(d: Path, counter: str, kernel: str, largest_grid: bool = False):
    vals, grid = {}, {}
    for r in counter_rows(d):
        if r.get("Counter_Name") != counter or kernel not in r.get("Kernel_Name", ""):
            continue
        key = (r.get("Dispatch_Id"), r.get("Agent_Id"))
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
        grid[key] = int(r.get("Grid_Size") or 0)
    if not vals:
        raise SystemExit(f"{counter}: no dispatch of a kernel matching {kernel!r} under {d}")
    if largest_grid:  # only the dispatches of the largest grid (bench's multi-frame launches)
        g = max(grid.values())
        return [v for k, v in vals.items() if grid[k] == g]
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", required=True, help='"<workload>|<variant>" as bench.py looks it up')
    ap.add_argument("--fetch", type=Path, required=True)
    ap.add_argument("--write", type=Path, required=True)
    ap.add_argument("--kernel", default="Trace")
    ap.add_argument("--out", type=Path, default=REPO / "profiles" / "pmc_traffic.json")
    ap.add_argument("--largest-grid", action="store_true",
                    help="keep the dispatches of the largest grid only (a key ending in |launch8: bench's 8-frame launches)")
    ap.add_argument("--source", default="", help="the command the passes profiled (recorded with the entry)")
    a = ap.parse_args()
    fetch = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel, a.largest_grid)
    write = per_dispatch(a.write, "WRITE_SIZE", a.kernel, a.largest_grid)
    fetch_b = 2.0 * 1024.0 * sum(fetch) / len(fetch)
    write_b = 1024.0 * sum(write) / len(write)
    entry = {
        "kernel": a.kernel,
        "dispatches": {"fetch_pass": len(fetch), "write_pass": len(write)},
        "fetch_bytes_per_launch": fetch_b,
        "write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "corrections": "FETCH_SIZE x2 x1024, WRITE_SIZE x1024 (MI355X_MICROARCH.md HBM section)",
    }
    if a.largest_grid:
        entry["dispatch_filter"] = "largest grid only"
    if a.source:
        entry["source"] = a.source
    data = json.loads(a.out.read_text()) if a.out.exists() else {}
    data[a.key] = entry
    a.out.write_text(json.dumps(data, indent=1, sort_keys=True) + "\n")
    print(json.dumps({a.key: entry}))


if __name__ == "__main__":
    main()
