"""Per-dispatch counters of the last codec decode from tools_dev/codec_pmc.sh passes."""
import csv, glob, os, sys
out = sys.argv[1]
table = {}
names = []
for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if "mpc::" in r["Kernel_Name"]]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    per = len(ids) // 3  # tools_dev/codec_prof.py: the last of its 3 decodes
    last = ids[-per:]
    if not names:
        kn = {int(r["Dispatch_Id"]): r["Kernel_Name"].split("(")[0].replace("void mpc::", "") for r in rows}
        names = [kn[d][:22] for d in last]
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
    print(f"{n:22s} " + " ".join(f"{t.get(c, float('nan')):.3g}" for c in cols))
