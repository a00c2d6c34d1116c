#!/usr/bin/env python3
"""Timeline of one fused O-projection + XA launch (EPI_RESID_XA) from the raw
in-kernel stamps (MAGPIE_TS_DUMP): when the O-projection's workgroups end, when
each XA wave has seen all of x1, and when the XA workgroups end (us after the
launch's first wave start). Usage: python tools_dev/diag_handoff.py [iters]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
import magpie_amd as ma  # noqa: E402

TS_WAVES, TS_BLOCKS = 8, 1024


def main():
    cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
    os.makedirs(cache, exist_ok=True)
    model = ma.synth_gguf(os.path.join(cache, "magpie_357m_f32_k32.gguf"), lt_head_scale=ma.DECISIVE)
    dump = os.path.join(REPO, "gpurun_out", "ts_dump.bin")
    os.makedirs(os.path.dirname(dump), exist_ok=True)
    os.environ["MAGPIE_TS_DUMP"] = dump
    os.environ["MAGPIE_EAGER"] = "1"
    dev = ma.Device(model)
    dev.synthesize([ma.synthetic_tokens(64, seed=1)], max_dec_steps=128, ignore_eos=True)
    names = dev.ops()
    for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        dev.profile_ops_ts(iters=1)
        raw = np.fromfile(dump, dtype=np.uint64).reshape(len(names), TS_BLOCKS, TS_WAVES, 2).astype(np.int64)
        for i, n in enumerate(names):
            if n != "oproj_xa":
                continue
            r = raw[i]
            t0 = r[:, :, 0][r[:, :, 1] > 0].min()
            rel = (r - t0) * 0.01
            nrow = 192
            g_end = rel[:nrow, :4, 1]
            xa_seen = rel[nrow:nrow + 4, 4:, 1]
            xa_end = rel[nrow:nrow + 4, :4, 1]
            xa_start = rel[nrow:nrow + 4, :4, 0]
            print(f"iter {it} layer-op {i}: oproj wg end p50 {np.median(g_end):.2f} max {g_end.max():.2f} | "
                  f"xa start {xa_start.min():.2f}-{xa_start.max():.2f} seen {xa_seen.min():.2f}-{xa_seen.max():.2f} "
                  f"end {xa_end.min():.2f}-{xa_end.max():.2f}")
            break
    dev.close()


if __name__ == "__main__":
    main()
