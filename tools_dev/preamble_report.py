"""Summarise a rocprofv3 kernel trace of tools_dev/preamble_prof.py: per kernel name,
launches and device time per preamble (the trace holds 1 + REPS preambles; the first,
which allocates, is dropped). usage: preamble_report.py TRACE_CSV REPS"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# preambles start with embed_text_kernel
starts = [i for i, r in enumerate(rows) if "embed_text_kernel" in r["Kernel_Name"]]
assert len(starts) >= reps + 1, len(starts)
seg = rows[starts[1]:]
agg = defaultdict(lambda: [0, 0.0])
t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
for r in seg:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = agg[r["Kernel_Name"][:100]]
    a[0] += 1
    a[1] += d
tot = sum(v[1] for v in agg.values())
print(f"{reps} preambles: {len(seg) / reps:.0f} launches each, busy {tot / reps:.1f} us, span {(t1 - t0) / 1e3 / reps:.1f} us per preamble")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k:100s} {v[0] / reps:6.1f} x {v[1] / v[0]:8.2f} us = {v[1] / reps:8.1f} us")
