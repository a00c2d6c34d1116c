"""Print the per-op table of bench JSON lines: optable.py FILE..."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], "fps", d["ms_per_step"], "ms/step")
    ot = d.get("op_table") or d.get("ops") or {}
    for k, v in sorted(ot.items(), key=lambda kv: -kv[1]["us_per_frame"]):
        print("  %-12s %3d %7.2f us %8.1f us/frame" % (k, v["launches_per_frame"], v["avg_us"], v["us_per_frame"]))
