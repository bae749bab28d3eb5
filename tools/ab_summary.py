#!/usr/bin/env python3
"""Summary of a tools/gpu_runs/gpu_libs.sh A/B in gpurun_out/: per library the bench value, the single-queue
rate, the HIP-event stage times and the one-queue rocprofv3 kernel means / minima.

    python tools/ab_summary.py base old ...
"""
import csv
import json
import sys


def main():
    for name in sys.argv[1:]:
        try:
            line = [l for l in open(f"gpurun_out/bench_{name}.log") if l.startswith("{")][-1]
            d = json.loads(line)
            st = d["stages_ms"]
            print(f"{name:8s} value {d['value']:9.0f}  single {d['single_queue']['mrays_per_s']:8.0f}  "
                  f"stages prep {st['prepare'] * 1e3:5.2f} bin {st['bin'] * 1e3:5.2f} trace {st['trace_kernel'] * 1e3:5.2f} us")
        except (OSError, IndexError, KeyError, ValueError) as e:
            print(f"{name:8s} no bench line ({e})")
        try:
            for r in csv.DictReader(open(f"gpurun_out/prof_{name}/run_kernel_stats.csv")):
                n = r["Name"]
                if "srt::" not in n:
                    continue
                n = n[n.find("namespace)::") + 12:].split("(")[0]
                print(f"    {n:18s} calls {r['Calls']:>5s} mean {float(r['AverageNs']) / 1e3:7.2f} min {float(r['MinNs']) / 1e3:7.2f} us")
        except OSError:
            pass


if __name__ == "__main__":
    main()
