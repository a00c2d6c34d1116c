#!/usr/bin/env python3
"""Timeline of one fused Q8_0 O-projection + XA launch (oproj_xa_q8: EPI_RESID_XQ8 rows,
then the q_net tails, then the attention + o_net tails) from the raw in-kernel stamps
(MAGPIE_TS_DUMP), us after the launch's first wave start: when the O-projection's
workgroups end, when the q_net tails see x1 / publish q, when the attention tails finish
the attention / end. Usage: python tools_dev/diag_handoff_q8.py [iters] [B]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
import magpie_amd as ma  # noqa: E402

TS_WAVES, TS_BLOCKS = 8, 1024
XQG, XQ8A, XQ8_QIN_NB = 8, 12, 2


def rng(a):
    return f"{a.min():6.2f}-{a.max():6.2f}" if a.size else "   -   "


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
    os.makedirs(cache, exist_ok=True)
    model = ma.synth_gguf(os.path.join(cache, "magpie_357m_q8_k32.gguf"), dtype="q8_0", lt_head_scale=ma.DECISIVE)
    dump = os.path.join(REPO, "gpurun_out", "ts_dump.bin")
    os.makedirs(os.path.dirname(dump), exist_ok=True)
    os.environ["MAGPIE_TS_DUMP"] = dump
    os.environ["MAGPIE_EAGER"] = "1"
    dev = ma.Device(model, weights="q8")
    dev.synthesize([ma.synthetic_tokens(64, seed=b + 1) for b in range(B)], max_dec_steps=128, ignore_eos=True)
    names = dev.ops()
    for it in range(iters):
        dev.profile_ops_ts(iters=1)
        raw = np.fromfile(dump, dtype=np.uint64).reshape(len(names), TS_BLOCKS, TS_WAVES, 2).astype(np.int64)
        seen = False
        for i, n in enumerate(names):
            if n == "oproj_xa_q8" and seen:
                continue
            if n not in ("oproj_xa_q8", "lt_slot_q8"):
                continue
            r = raw[i]
            live = r[:, 0, 1] > 0
            t0 = r[:, :, 0][r[:, :, 1] > 0].min()
            rel = (r - t0) * 0.01
            if n == "lt_slot_q8":
                print(f"iter {it} op {i} {n}: start {rng(rel[live, :4, 0])} y seen {rng(rel[live, 4, 1])} "
                      f"end {rng(rel[live, :4, 1])}")
                continue
            ids = np.nonzero(live)[0]
            nxq = 0 if B <= XQ8_QIN_NB else XQG * B  # small batches: q in the attention workgroups
            nrow = len(ids) - nxq - XQ8A * B
            rows, xq, at = ids[:nrow], ids[nrow:nrow + nxq], ids[nrow + nxq:]
            if nxq == 0:  # small batches: the q-in-attention workgroups' phase stamps (ts_phase 0..3)
                print(f"iter {it} op {i}: oproj {len(rows)} wg end {rng(rel[rows, :4, 1])} | attn {len(at)} start "
                      f"{rng(rel[at, :4, 0])} x1 seen {rng(rel[at, 4, 1])} ln+quant {rng(rel[at, 5, 1])} "
                      f"q {rng(rel[at, 6, 1])} attn {rng(rel[at, 7, 1])} end {rng(rel[at, :4, 1])}")
                seen = True
                continue
            print(f"iter {it} op {i}: oproj {len(rows)} wg end {rng(rel[rows, :4, 1])} | xq {len(xq)} "
                  f"start {rng(rel[xq, :4, 0])} x1 seen {rng(rel[xq, 4, 1])} end {rng(rel[xq, 0, 1])} | "
                  f"attn {len(at)} start {rng(rel[at, :4, 0])} attn done {rng(rel[at, 4:, 1])} "
                  f"end {rng(rel[at, :4, 1])}")
            seen = True
    dev.close()


if __name__ == "__main__":
    main()
