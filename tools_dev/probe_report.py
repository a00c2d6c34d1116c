"""Report of a MP_TS_PROBE build's stamps (ab_libs/probe.so): per op, the p50 over
workgroups of (loads landed, statistics done, rows put) in the batched LN staging,
us after the op's first wave start. usage: probe_report.py WEIGHTS B [op ...]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
import magpie_amd as ma  # noqa: E402

TS_WAVES, TS_BLOCKS = 8, 1024
weights, B = sys.argv[1], int(sys.argv[2])
only = set(sys.argv[3:])
cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
os.makedirs(cache, exist_ok=True)
model = ma.synth_gguf(os.path.join(cache, "magpie_357m_f32_k32.gguf"), lt_head_scale=ma.DECISIVE)
dump = os.path.join(REPO, "gpurun_out", "ts_dump.bin")
os.environ["MAGPIE_TS_DUMP"] = dump
dev = ma.Device(model, weights=weights)
toks = [ma.synthetic_tokens(64, seed=1000 + b) for b in range(B)]
dev.synthesize(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=128, ignore_eos=True)
names = dev.ops()
dev.profile_ops_ts(iters=2)
raw = np.fromfile(dump, dtype=np.uint64).reshape(len(names), TS_BLOCKS, TS_WAVES, 2).astype(np.int64)
seen = set()
for i, n in enumerate(names):
    if (only and n not in only) or n in seen:
        continue
    seen.add(n)
    r = raw[i]
    ok = r[:, :4, 1] > 0
    if not ok.any():
        continue
    t0 = r[:, :4, 0][ok].min()
    nb = int(ok.any(axis=1).sum())
    rel = (r[:nb] - t0) * 0.01
    mk = r[:nb, 4:, 1] > 0
    if not mk.any():
        continue
    A = rel[:, 4:6, 0][mk[:, :2]]
    Bs = rel[:, 4:6, 1][mk[:, :2]]
    C = rel[:, 6:8, 1][mk[:, 2:]]
    E = rel[:, :4, 1][ok[:nb]]
    print(f"{n:10s} wgs {nb:4d} loads landed p50 {np.median(A):5.2f} | stats p50 {np.median(Bs):5.2f} | "
          f"rows put p50 {np.median(C):5.2f} | end p50 {np.median(E):5.2f} max {E.max():5.2f}")
dev.close()
