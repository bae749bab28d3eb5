#!/usr/bin/env python3
"""Per-frame kernel timeline from a rocprofv3 --kernel-trace CSV: duration of each kernel and
the idle gap before it (the last N kernels), plus mean busy / gap per frame.

    python tools/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv [--last 12]
    python tools/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv --overlap 150 --skip 100

--overlap N: over the last N kernels (frame queues: kernels of different streams overlap),
the wall time they span, the time with at least one kernel running, and the mean number of
kernels running while any is.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=12)
    ap.add_argument("--frame-kernel", default="PrepareKernel", help="kernel that starts a frame")
    ap.add_argument("--overlap", type=int, default=0)
    ap.add_argument("--skip", type=int, default=-1, help="--overlap over kernels [skip, skip + N) instead")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "srt::" in r["Kernel_Name"]]
    if a.overlap:
        overlap(rows[a.skip:a.skip + a.overlap] if a.skip >= 0 else rows[-a.overlap:])
        return
    prev = None
    frames, cur = [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("srt::", "")
        gap = 0 if prev is None else max(0, s - prev)
        if a.frame_kernel in name:
            cur = {"busy": 0, "gap": 0}
            frames.append(cur)
        if cur is not None:
            cur["busy"] += e - s
            cur["gap"] += gap if a.frame_kernel not in name else 0
        r["_line"] = f"{name:28s} dur {(e - s) / 1e3:8.2f} us  gap before {gap / 1e3:7.2f} us"
        prev = e
    for r in rows[-a.last:]:
        print(r["_line"])
    full = frames[1:-1] or frames
    if full:
        busy = sum(f["busy"] for f in full) / len(full) / 1e3
        gap = sum(f["gap"] for f in full) / len(full) / 1e3
        print(f"frames {len(full)}: mean kernel time {busy:.2f} us, mean in-frame gaps {gap:.2f} us")


def overlap(rows):
    ev = sorted([(int(r["Start_Timestamp"]), 1) for r in rows] + [(int(r["End_Timestamp"]), -1) for r in rows])
    active, last, busy, weighted = 0, ev[0][0], 0, 0
    for t, d in ev:
        if active:
            busy += t - last
            weighted += active * (t - last)
        active += d
        last = t
    span = ev[-1][0] - ev[0][0]
    kern = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
    print(f"{len(rows)} kernels over {span / 1e3:.1f} us: some kernel running {100 * busy / span:.1f} % of it, "
          f"{weighted / max(busy, 1):.2f} kernels running on average meanwhile; summed kernel durations "
          f"{kern / 1e3:.1f} us")


if __name__ == "__main__":
    main()
