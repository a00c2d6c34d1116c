#!/usr/bin/env python3
"""PMC report of tools_dev/pmc_collect.sh's passes: pmc_report.py TAG writes
  profiles/TAG_pmc_decode_f32_b1.json    per decode op: HBM-side bytes per launch
  profiles/TAG_pmc_decode_bf16_b16.json  per decode op: bytes + MFMA busy / util
  profiles/TAG_pmc_codec.json            per codec kernel shape: bytes + MFMA

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB per dispatch.
MI355X_MICROARCH.md ("HBM"): on gfx950 FETCH_SIZE reports exactly half of the bytes
of a wide coalesced streaming read (16 B/lane) -> doubled here, but only for the
kernels whose bulk loads are 16 B per lane (WIDE below); other kernels' fetch is
reported raw and marked uncalibrated. WRITE_SIZE is exact for 16 B/lane stores.
Infinity-Cache hits are counted: these are L2-miss (fabric) bytes, an upper bound
on HBM bytes. MFMA utilisation = sum SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x
1024 SIMDs): GRBM_GUI_ACTIVE is the sum over the 8 XCDs, so / 8 gives the dispatch's
cycles (round 5 divided by the sum, 8x too low); MFMA FLOPs = MOPS x 512. Under
per-dispatch PMC collection GRBM_GUI_ACTIVE includes the profiler's own per-dispatch
overhead, so with a kernel trace of the same workload (TRACE_CSV, e.g. the bench's
rocprofv3 --kernel-trace run) the codec utilisation is also given against the traced
duration: busy / (duration x 2.4 GHz x 1024).
usage: pmc_report.py TAG [TRACE_CSV]"""
import csv
import json
import os
import sys
from collections import defaultdict

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
SIMDS = 256 * 4
XCDS = 8  # GRBM_GUI_ACTIVE is reported summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS row)
CLK = 2.4e9  # shader clock (MI355X_MICROARCH.md)
# kernels whose bulk global loads are 16 B per lane (float4 / uint4 / half8)
WIDE = ("gemv_kernel", "gemm_b16_kernel", "xa_part_kernel", "sa_attn_kernel", "lt_ffn2_kernel", "lt_ffn_kernel",
        "conv_mfma_kernel", "gemm_q8_kernel_dec")
DECODE = ("gemv_kernel", "sa_attn_kernel", "xa_part_kernel", "lt_finalize_kernel", "gemm_b16_kernel", "gemm_q8_kernel_dec",
          "lt_ffn_kernel", "lt_ffn2_kernel", "lt_merge_kernel", "lt_pick_kernel", "xa_q8_kernel", "xa_f32_kernel",
          "lt_slot_kernel", "lt_slot_q8_kernel", "lt_front_kernel")
# (embed_kernel runs once per decode, for the BOS frame, outside the iteration)


def rows(tag, name):
    """{dispatch_id: (kernel, grid, {counter: value})} of one pass"""
    d = {}
    for r in csv.DictReader(open(os.path.join(OUT, f"{tag}_pmc_{name}", "pmc_counter_collection.csv"))):
        k = int(r["Dispatch_Id"])
        e = d.setdefault(k, (r["Kernel_Name"], int(r["Grid_Size"]), {}))
        e[2][r["Counter_Name"]] = e[2].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [d[k] for k in sorted(d)]


def wide(kernel):
    return any(w in kernel for w in WIDE)


def decode_ops(tag, pre, ops_file, mfma):
    ops = json.load(open(os.path.join(OUT, ops_file)))["ops"]
    passes = {"fetch": rows(tag, pre + "_fetch"), "write": rows(tag, pre + "_write")}
    if mfma:
        passes["mfma"] = rows(tag, pre + "_mfma")
    n = len(ops)
    seqs = {}
    for k, v in passes.items():
        seq = [e for e in v if any(t in e[0] for t in DECODE)]
        it = len(seq) // n
        assert it >= 2 and len(seq) == it * n, (k, len(seq), n)
        seqs[k] = (seq, it)
    res = {}
    for i, op in enumerate(ops):
        rec = res.setdefault(op, defaultdict(list))
        for k, (seq, it) in seqs.items():
            for j in range(it):
                kern, grid, c = seq[j * n + i]
                rec["kernel"] = kern
                for cn, cv in c.items():
                    rec[cn].append(cv)
    out = {}
    for op, rec in res.items():
        f = float(np.mean(rec["FETCH_SIZE"])) * 1024
        w = float(np.mean(rec["WRITE_SIZE"])) * 1024
        o = {"kernel": rec["kernel"], "launches_averaged": len(rec["FETCH_SIZE"]),
             "fetch_bytes_raw": round(f), "fetch_bytes": round(2 * f if wide(rec["kernel"]) else f),
             "fetch_corrected": wide(rec["kernel"]), "write_bytes": round(w)}
        o["traffic_bytes"] = o["fetch_bytes"] + o["write_bytes"]
        if mfma:
            busy, gui = float(np.mean(rec["SQ_VALU_MFMA_BUSY_CYCLES"])), float(np.mean(rec["GRBM_GUI_ACTIVE"]))
            o["mfma_busy_cycles"] = round(busy)
            o["gui_active_cycles"] = round(gui)
            o["mfma_util"] = round(busy / (gui / XCDS * SIMDS), 4) if gui else None
            mops = [v for k, v in rec.items() if k.startswith("SQ_INSTS_VALU_MFMA_MOPS_")]
            if mops:
                o["mfma_ops"] = round(float(np.mean(mops[0])) * 512)  # MOPS x 512 = multiply-adds x 2
        out[op] = o
    return out


def trace_durations(path):
    """{(kernel, grid threads): mean duration us} from a rocprofv3 kernel trace"""
    d = defaultdict(list)
    if path:
        for r in csv.DictReader(open(path)):
            g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            d[(r["Kernel_Name"], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    return {k: float(np.mean(v)) for k, v in d.items()}


def codec(tag, trace=None):
    dur = trace_durations(trace)
    passes = {k: rows(tag, "codec_" + k) for k in ("fetch", "write", "mfma")}
    groups = {}
    for k, v in passes.items():
        for kern, grid, c in v:
            if "mpc::" not in kern and "conv" not in kern:
                continue
            g = groups.setdefault((kern, grid), defaultdict(list))
            for cn, cv in c.items():
                g[cn].append(cv)
    out, tot = [], defaultdict(float)
    for (kern, grid), g in groups.items():
        f = float(np.mean(g["FETCH_SIZE"])) * 1024
        w = float(np.mean(g["WRITE_SIZE"])) * 1024
        busy, gui = float(np.mean(g["SQ_VALU_MFMA_BUSY_CYCLES"])), float(np.mean(g["GRBM_GUI_ACTIVE"]))
        flops = float(np.mean(g.get("SQ_INSTS_VALU_MFMA_MOPS_F16", [0.0]))) * 512
        n = len(g["FETCH_SIZE"])
        fb = 2 * f if wide(kern) else f
        rec = {"kernel": kern, "grid": grid, "dispatches": n, "fetch_bytes": round(fb), "fetch_corrected": wide(kern),
               "write_bytes": round(w), "mfma_flops": round(flops), "mfma_busy_cycles": round(busy),
               "gui_active_cycles": round(gui), "mfma_util": round(busy / (gui / XCDS * SIMDS), 4) if gui else None}
        if flops:
            rec["busy_cycles_per_mfma_16x16x32"] = round(busy / (flops / 16384), 2)
        t = dur.get((kern, grid))
        if t:
            rec["traced_us"] = round(t, 2)
            rec["mfma_util_traced"] = round(busy / (t * 1e-6 * CLK * SIMDS), 4)
            rec["tflops_traced"] = round(flops / (t * 1e-6) / 1e12, 1)
            rec["hbm_tbs_traced"] = round((fb + w) / (t * 1e-6) / 1e12, 2)
            tot["t"] += n * t
        tot["bytes"] += n * (fb + w)
        tot["flops"] += n * flops
        tot["busy"] += n * busy
        tot["gui"] += n * gui
        out.append(rec)
    out.sort(key=lambda r: -r["dispatches"] * r["gui_active_cycles"])
    decodes = 4
    summary = {"chunks": 8, "per_decode_bytes": round(tot["bytes"] / decodes), "per_decode_mfma_flops": round(tot["flops"] / decodes),
               "mfma_util_gui_active": round(tot["busy"] / (tot["gui"] / XCDS * SIMDS), 4) if tot["gui"] else None}
    if tot["t"]:
        summary["per_decode_traced_us"] = round(tot["t"] / decodes, 1)
        summary["mfma_util_traced"] = round(tot["busy"] / (tot["t"] * 1e-6 * CLK * SIMDS), 4)
        summary["tflops_traced"] = round(tot["flops"] / (tot["t"] * 1e-6) / 1e12, 1)
        summary["hbm_tbs_traced"] = round(tot["bytes"] / (tot["t"] * 1e-6) / 1e12, 2)
    return {"summary": summary, "kernels": out}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    src = ("rocprofv3 --pmc, separate passes per counter group (tools_dev/pmc_collect.sh), eager launches; "
           "bytes = FETCH_SIZE x 1024 (x2 for 16 B/lane kernels, gfx950) + WRITE_SIZE x 1024")
    for pre, ops_file, mfma, name in (("f32b1", "pmc_ops_f32_1.json", False, "decode_f32_b1"),
                                      ("b16b16", "pmc_ops_bf16_16.json", True, "decode_bf16_b16"),
                                      ("q8b16", "pmc_ops_q8_16.json", True, "decode_q8_b16")):
        res = {"source": src, "workload": name, "ops": decode_ops(tag, pre, ops_file, mfma),
               "lib_sha16": json.load(open(os.path.join(OUT, ops_file))).get("lib_sha16")}
        json.dump(res, open(os.path.join(REPO, "profiles", f"{tag}_pmc_{name}.json"), "w"), indent=1)
        print(f"== {name}")
        for op, v in res["ops"].items():
            extra = f" mfma util {v['mfma_util']}" if "mfma_util" in v else ""
            print(f"  {op:10s} fetch {v['fetch_bytes'] / 1e6:8.3f} MB write {v['write_bytes'] / 1e6:7.3f} MB{extra}")
    c = codec(tag, sys.argv[2] if len(sys.argv) > 2 else None)
    c["source"] = src
    bj = os.path.join(OUT, "pmc_codec_build.json")
    c["lib_sha16"] = json.load(open(bj)).get("lib_sha16") if os.path.exists(bj) else None
    json.dump(c, open(os.path.join(REPO, "profiles", f"{tag}_pmc_codec.json"), "w"), indent=1)
    print("== codec", c["summary"])
    for r in c["kernels"][:14]:
        print(f"  {r['kernel'][:48]:48s} grid {r['grid']:9d} x{r['dispatches']:3d} bytes {(r['fetch_bytes'] + r['write_bytes']) / 1e6:8.2f} MB"
              f" GF {r['mfma_flops'] / 1e9:7.2f} util {r['mfma_util']}")


if __name__ == "__main__":
    main()
