#!/usr/bin/env python3
"""Per-op timeline from the raw in-kernel stamps (MAGPIE_TS_DUMP): for every op
of one decode iteration, the spread of workgroup start / intermediate mark
(ts_mark: e.g. the bf16 kernels' staged activation tile, the fused XA's x1 seen) /
end times, us after the op's first wave start.
usage: diag_timeline.py WEIGHTS B [op ...]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
import magpie_amd as ma  # noqa: E402

TS_WAVES, TS_BLOCKS = 8, 1024
ROLE_SPLIT = {}  # op name -> row workgroups (set per batch in main)


def main():
    weights, B = sys.argv[1], int(sys.argv[2])
    only = set(sys.argv[3:])
    cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
    os.makedirs(cache, exist_ok=True)
    fn, dt = {"q8": ("magpie_357m_q8_k32.gguf", "q8_0"), "q4": ("magpie_357m_q4_k32.gguf", "q4_0"),
              "f16": ("magpie_357m_f16_k32.gguf", "f16")}.get(weights, ("magpie_357m_f32_k32.gguf", "f32"))
    model = ma.synth_gguf(os.path.join(cache, fn), dtype=dt, lt_head_scale=ma.DECISIVE)
    dump = os.path.join(REPO, "gpurun_out", "ts_dump.bin")
    os.makedirs(os.path.dirname(dump), exist_ok=True)
    os.environ["MAGPIE_TS_DUMP"] = dump
    dev = ma.Device(model, weights=weights)
    toks = [ma.synthetic_tokens(64, seed=1000 + b) for b in range(B)]
    dev.synthesize(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=128, ignore_eos=True)
    names = dev.ops()
    ROLE_SPLIT.update({"oproj_xa": 48, "qkv_sa": 144})
    dev.profile_ops_ts(iters=2)
    raw = np.fromfile(dump, dtype=np.uint64).reshape(len(names), TS_BLOCKS, TS_WAVES, 2).astype(np.int64)
    seen = set()
    for i, n in enumerate(names):
        if (only and n not in only) or n in seen:
            continue
        seen.add(n)
        r = raw[i]
        ok = r[:, :, 1] > 0
        if not ok.any():
            continue
        t0 = r[:, :, 0][ok].min()
        rel = (r - t0) * 0.01
        nb = int(ok[:, :4].any(axis=1).sum())
        st, en = rel[:nb, :4, 0], rel[:nb, :4, 1]
        mk = rel[:nb, 4:, 1][ok[:nb, 4:]]
        mk0 = rel[:nb, 4:, 0][ok[:nb, 4:]]
        line = (f"{n:10s} wgs {nb:4d} start p50 {np.median(st):5.2f} max {st.max():5.2f} | "
                f"end p50 {np.median(en):5.2f} max {en.max():5.2f}")
        if mk.size:
            line += f" | mark p50 {np.median(mk):5.2f} max {mk.max():5.2f} (first stamp p50 {np.median(mk0):5.2f})"
        if os.environ.get("PHASES") and not ROLE_SPLIT.get(n):  # ts_phase<k> of every workgroup
            for k in range(4):
                okk = ok[:nb, 4 + k]
                if okk.any():
                    v = rel[:nb, 4 + k, 1][okk]
                    line += f" | ph{k} {np.median(v):5.2f}/{v.max():5.2f}"
        print(line)
        # launches with two roles (row workgroups, then the attention tail): each apart
        nrow = ROLE_SPLIT.get(n)
        if nrow and nb > nrow:
            for lo, hi, role in ((0, nrow, "rows"), (nrow, nb, "tail")):
                okr = ok[lo:hi, :4]
                e2 = rel[lo:hi, :4, 1][okr]
                m2 = rel[lo:hi, 4:, 1][ok[lo:hi, 4:]]
                txt = f"   {role:5s} wgs {hi - lo:4d} end p50 {np.median(e2):5.2f} max {e2.max():5.2f}"
                if m2.size:
                    txt += f" | mark p50 {np.median(m2):5.2f} min {m2.min():5.2f} max {m2.max():5.2f}"
                if os.environ.get("PHASES"):  # ts_phase<k> stamps: slot 4 + k, p50 / max per phase
                    for k in range(4):
                        okk = ok[lo:hi, 4 + k]
                        if okk.any():
                            v = rel[lo:hi, 4 + k, 1][okk]
                            txt += f" | ph{k} {np.median(v):5.2f}/{v.max():5.2f}"
                print(txt)
    dev.close()


if __name__ == "__main__":
    main()
