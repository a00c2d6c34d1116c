"""Per-dispatch counters of the last codec decode from tools_dev/codec_pmc.sh passes."""
import csv, glob, os, sys
out = sys.argv[1]
names = ["pre"]
for s in range(5):
    names.append(f"s{s} convT")
    for k in range(3):
        names += [f"s{s} k{k} in", f"s{s} k{k} sk"]
names.append("post")
table = {}
for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if "mpc::" in r["Kernel_Name"]]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    last = ids[-len(names):]
    for r in rows:
        d = int(r["Dispatch_Id"])
        if d in last:
            table.setdefault(last.index(d), {})[r["Counter_Name"]] = table.get(last.index(d), {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
cols = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
        "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS", "SQ_INSTS_VALU",
        "SQ_INSTS_VMEM_RD", "SQ_VALU_MFMA_BUSY_CYCLES", "TCC_HIT_sum", "TCC_MISS_sum", "GRBM_GUI_ACTIVE",
        "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "TCP_PENDING_STALL_CYCLES_sum", "TCP_TCR_TCP_STALL_CYCLES_sum"]
print("op " + " ".join(c.replace("SQ_", "").replace("_sum", "")[:14] for c in cols))
for i, n in enumerate(names):
    t = table.get(i, {})
    print(f"{n:11s} " + " ".join(f"{t.get(c, float('nan')):.3g}" for c in cols))
