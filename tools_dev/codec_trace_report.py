"""Per-dispatch codec times from a rocprofv3 kernel-trace CSV (last decode of
tools_dev/codec_prof.py): pre, then per stage convT + 3 x (in_conv, sk_conv), post."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "mpc::" in r["Kernel_Name"]]
per = len(rows) // 3
last = rows[-per:]
names = ["pre"]
for s in range(5):
    names.append(f"s{s} convT")
    for k in range(3):
        names += [f"s{s} k{k} in", f"s{s} k{k} sk"]
names.append("post")
tot = 0.0
stage = {}
for n, r in zip(names, last):
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += us
    stage[n.split()[0]] = stage.get(n.split()[0], 0.0) + us
    print(f"{n:12s} {us:8.1f} us  {r['Kernel_Name'][:60]}")
print(f"total {tot:.1f} us;", {k: round(v, 1) for k, v in stage.items()})
