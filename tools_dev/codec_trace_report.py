"""Per-dispatch codec times from a rocprofv3 kernel-trace CSV (last of the 3 decodes
of tools_dev/codec_prof.py), in launch order, plus per-kernel totals."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "mpc::" in r["Kernel_Name"]]
per = len(rows) // 3
last = rows[-per:]
tot = 0.0
by = {}
for i, r in enumerate(last):
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += us
    k = r["Kernel_Name"].split("(")[0].replace("void mpc::", "")
    by[k] = by.get(k, 0.0) + us
    print(f"{i:3d} {us:8.1f} us  {k}")
span = (int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])) / 1e3
print(f"{per} dispatches, sum {tot:.1f} us, span {span:.1f} us")
for k, v in sorted(by.items(), key=lambda kv: -kv[1]):
    print(f"  {v:8.1f} us  {k}")
