#!/usr/bin/env python3
"""Phase timeline of the codec's per-block residual kernel (rb_kernel), from its in-kernel
stamps (MAGPIE_CODEC_TS): per stage (first residual block), per branch, the workgroups'
durations of A (x rows -> HalfSnake -> LDS), B (conv_d), C (intermediate -> LDS),
D (conv_1), E (residual + store), wave 0's own part of C and of E's loads, and how the launch's workgroups spread in time.
usage: codec_rb_timeline.py [stages...]   (default 1 2 3 4; 8 x 32-frame chunks)"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
import magpie_amd as ma  # noqa: E402

GX = 16384
cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
os.makedirs(cache, exist_ok=True)
stages = [int(a) for a in sys.argv[1:]] or [1, 2, 3, 4]
cdc = ma.Codec(ma.synth_gguf(os.path.join(cache, "nano_codec.gguf"), kind="codec"))
codes = np.random.default_rng(0).integers(0, 2016, (8, 8, 32)).astype(np.int32)
cdc.decode_chunks(codes)
dump = os.path.join(REPO, "gpurun_out", "codec_ts.bin")
os.makedirs(os.path.dirname(dump), exist_ok=True)
for st in stages:
    os.environ["MAGPIE_CODEC_TS"] = f"{st},0,{dump}"
    cdc.decode_chunks(codes)
    del os.environ["MAGPIE_CODEC_TS"]
    ts = np.fromfile(dump, dtype=np.uint64).reshape(3, GX, 48).astype(np.int64)
    live = ts[:, :, 0] > 0
    t_min = ts[:, :, 0][live].min()
    t_max = ts[:, :, 5][live].max()
    waves = []
    print(f"stage {st}: {live.sum()} workgroups, launch span {(t_max - t_min) * 0.01:.1f} us")
    for br in range(3):
        r = ts[br][live[br]]
        if not len(r):
            continue
        d = np.diff(r[:, :6], axis=1) * 0.01
        tot = (r[:, 5] - r[:, 0]) * 0.01
        st0 = (r[:, 0] - t_min) * 0.01
        names = ["A rows", "B conv_d", "C stage", "D conv_1", "E store"]
        parts = " | ".join(f"{n} {np.median(d[:, i]):5.2f}" for i, n in enumerate(names))
        if (r[:, 6] > 0).all() and (r[:, 7] > 0).all():  # wave 0's own part of C / E
            c0 = np.median(r[:, 6] - r[:, 2]) * 0.01
            e0 = np.median(r[:, 7] - r[:, 4]) * 0.01
            b0 = np.median(r[:, 9] - r[:, 1]) * 0.01
            s0 = np.median(r[:, 8] - r[:, 7]) * 0.01
            parts += f" || wave 0: conv_d {b0:5.2f} C {c0:4.2f} E rows {e0:4.2f} stores {s0:4.2f}"
            # every wave's conv_d / conv_1 end (from the phase start), median per wave
            nw = int(((r[:, 16:48:2] > 0).sum(axis=1)).max())
            wd = [np.median(r[:, 16 + 2 * k] - r[:, 1]) * 0.01 for k in range(nw)]
            w1 = [np.median(r[:, 17 + 2 * k] - r[:, 3]) * 0.01 for k in range(nw)]
            waves.append((br, wd, w1))
        print(f"  branch {br} ({len(r)} wgs): per workgroup p50 {parts} | total {np.median(tot):5.2f} "
              f"(max {tot.max():5.2f}); starts spread {st0.max():5.1f} us")
    for br, wd, w1 in waves:
        print(f"  branch {br} per wave conv_d end: " + " ".join(f"{x:5.2f}" for x in wd))
        print(f"  branch {br} per wave conv_1 end: " + " ".join(f"{x:5.2f}" for x in w1))
os.remove(dump)  # 3 x GX x 48 stamps: not for the trip back
cdc.close()
