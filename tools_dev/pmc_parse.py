"""Per-op HBM traffic of the decode iteration from the two PMC passes of
tools_dev/pmc_traffic.sh: pmc_parse.py TAG -> profiles/TAG_pmc_traffic.json.

FETCH_SIZE and WRITE_SIZE are rocprofv3 derived counters in KiB per dispatch.
MI355X_MICROARCH.md ("HBM"): on gfx950 FETCH_SIZE reports exactly half of the
bytes of a wide coalesced streaming read (16 B/lane) -> doubled here; WRITE_SIZE
reads the bytes exactly for 16 B/lane streaming stores. Infinity-Cache hits are
counted, so these are fabric (L2-miss) bytes, an upper bound on HBM bytes.
The decode dispatches (preamble and copy kernels filtered out) repeat the op
order of one iteration (gpurun_out/pmc_ops.json); op i of every iteration is
averaged."""
import csv
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
ops = json.load(open(os.path.join(REPO, "gpurun_out", "pmc_ops.json")))["ops"]
DECODE = ("gemv_kernel", "sa_attn_kernel", "xa_part_kernel", "lt_finalize_kernel", "gemm_b16_kernel",
          "gemv_q8_kernel", "row_xa_kernel", "lt_ffn_kernel", "lt_merge_kernel", "lt_pick_kernel", "xa_q8_kernel")


def per_op(kind):
    rows = list(csv.DictReader(open(os.path.join(REPO, "gpurun_out", f"{tag}_pmc_{kind}", "pmc_counter_collection.csv"))))
    seq = []
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        name = r["Kernel_Name"]
        if any(k in name for k in DECODE) and not (name.startswith("mp::row_xa") and "row_xa" not in " ".join(ops)):
            seq.append((name, float(r["Counter_Value"])))
    n = len(ops)
    it = len(seq) // n
    assert it >= 2 and len(seq) == it * n, (len(seq), n)
    out = {}
    for i, op in enumerate(ops):
        vals = [seq[j * n + i][1] for j in range(it)]
        out.setdefault(op, {"kernel": seq[i][0], "kib": []})["kib"].extend(vals)
    return out, it


fetch, it = per_op("fetch")
write, _ = per_op("write")
res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), eager decode, Magpie-357M f32 B=1",
       "correction": "bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 (gfx950 FETCH_SIZE halves 16 B/lane streaming reads)",
       "iterations": it, "ops": {}}
for op in fetch:
    f = float(np.mean(fetch[op]["kib"])) * 1024 * 2
    w = float(np.mean(write[op]["kib"])) * 1024
    res["ops"][op] = {"kernel": fetch[op]["kernel"], "fetch_bytes": round(f), "write_bytes": round(w),
                      "traffic_bytes": round(f + w), "launches_averaged": len(fetch[op]["kib"])}
os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
json.dump(res, open(os.path.join(REPO, "profiles", f"{tag}_pmc_traffic.json"), "w"), indent=1)
for op, v in res["ops"].items():
    print(f"{op:10s} fetch {v['fetch_bytes'] / 1e6:8.3f} MB  write {v['write_bytes'] / 1e6:7.3f} MB  {v['kernel'][:60]}")
