#!/usr/bin/env python3
"""Cut a rocprofv3 kernel trace to the launches of bench.py's in-situ timing pass.

mp_hip_profile_ops_kev brackets its launches with two empty profile_mark_kernel
dispatches. This script keeps the dispatches between the first such pair and
writes per-kernel statistics in rocprofv3's kernel_stats column layout, so the
profiler's average for the roofline kernel can be set beside bench.py's
"avg_launch_us" for the same launches.

usage: prof_phase.py <prof_kernel_trace.csv> <out_stats.csv>
"""
import csv
import sys

import numpy as np


def main(trace_path, out_path):
    rows = list(csv.DictReader(open(trace_path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "profile_mark_kernel" in r["Kernel_Name"]]
    if len(marks) < 2:
        sys.exit(f"{trace_path}: no profile_mark_kernel pair (run bench.py under rocprofv3 --kernel-trace)")
    a, b = marks[0], marks[1]
    per = {}
    for r in rows[a + 1:b]:
        per.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    total = sum(sum(v) for v in per.values())
    out = []
    for name, d in per.items():
        d = np.array(d, dtype=np.float64)
        out.append({"Name": name, "Calls": len(d), "TotalDurationNs": int(d.sum()), "AverageNs": round(d.mean(), 1),
                    "Percentage": round(100.0 * d.sum() / total, 3), "MinNs": int(d.min()), "MaxNs": int(d.max()),
                    "StdDev": round(d.std(), 1)})
    out.sort(key=lambda r: -r["TotalDurationNs"])
    with open(out_path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(out[0]))
        w.writeheader()
        w.writerows(out)
    for r in out[:12]:
        print(f"{r['Name'][:64]:64s} {r['Calls']:6d} avg {r['AverageNs'] / 1000:7.3f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
