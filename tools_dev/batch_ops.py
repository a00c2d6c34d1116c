"""In-situ per-op table of the decode iteration at a given batch / weight mode:
batch_ops.py WEIGHTS B [B ...]  (fixed-length greedy, T=64, mid-utterance state)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
import magpie_amd as ma  # noqa: E402

cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
os.makedirs(cache, exist_ok=True)
weights = sys.argv[1]
path = ma.synth_gguf(os.path.join(cache, "magpie_357m_q8.gguf" if weights == "q8" else "magpie_357m_f32.gguf"),
                     dtype="q8_0" if weights == "q8" else "f32")
dev = ma.Device(path, weights=weights)
for B in [int(b) for b in sys.argv[2:]]:
    toks = [ma.synthetic_tokens(64, seed=1000 + b) for b in range(B)]
    r = dev.synthesize(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=256, ignore_eos=True)
    r = dev.decode(B, 256)
    fps = B * 256 * 1e3 / r.decode_ms
    dev.synthesize(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=128, ignore_eos=True)
    names = dev.ops()
    us = dev.profile_ops_kev(iters=16)
    span = dev.profile_ops_ts(iters=16)
    groups, spans = {}, {}
    for i, n in enumerate(names):
        groups.setdefault(n, []).append(us[i])
        spans.setdefault(n, []).append(span[i])
    print(f"== {weights} B={B}: {fps:.0f} fps, {r.decode_ms / 256 * 1e3:.1f} us/iteration (graph)")
    tot = 0.0
    for n, v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        tot += sum(v)
        print(f"  {n:12s} {len(v):3d} x {np.mean(v):7.2f} us (wave span {np.mean(spans[n]):6.2f}) = {sum(v):8.1f} us/iter")
    print(f"  dispatch-timed total {tot:.1f} us/iter")
dev.close()
