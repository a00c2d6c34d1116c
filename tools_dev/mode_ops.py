"""Per-op launch times of one weight mode / batch size (diagnostic): decode the
batch to mid-utterance, then time whole eager iterations op by op
(mp_hip_profile_ops_kev: the dispatch's own begin/end stamps) and the in-kernel
wave spans (mp_hip_profile_ops_ts), plus the graph-replayed frames/s.

usage: python tools_dev/mode_ops.py WEIGHTS B [model] [ENV=VAL ...]
  WEIGHTS: f32 | bf16 | q8 | q4 | f16;  model: f32 (default) | q8 | q4 | f16 file
  MODE_XA=auto|reassoc|direct, MODE_KV=f32|bf16: the Device's cross-attention form / SA cache type"""
import os
import sys

args = [a for a in sys.argv[1:] if "=" not in a]
for a in sys.argv[1:]:
    if "=" in a:
        k, v = a.split("=", 1)
        os.environ[k] = v
weights, B = args[0], int(args[1])
kind = args[2] if len(args) > 2 else {"q8": "q8", "q4": "q4", "f16": "f16"}.get(weights, "f32")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
import numpy as np  # noqa: E402
import magpie_amd as ma  # noqa: E402

C = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
os.makedirs(C, exist_ok=True)
files = {"f32": ("magpie_357m_f32_k32.gguf", "f32"), "q8": ("magpie_357m_q8_k32.gguf", "q8_0"),
         "q4": ("magpie_357m_q4_k32.gguf", "q4_0"), "f16": ("magpie_357m_f16_k32.gguf", "f16")}
fn, dt = files[kind]
path = ma.synth_gguf(os.path.join(C, fn), dtype=dt, lt_head_scale=ma.DECISIVE)
dev = ma.Device(path, weights=weights, xa=os.environ.get("MODE_XA", "auto"), kv=os.environ.get("MODE_KV", "f32"))
toks = [ma.synthetic_tokens(64, seed=1000 + b) for b in range(B)]
frames = 256
dev.synthesize(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=frames, ignore_eos=True)
ms = [dev.decode(B, frames).decode_ms for _ in range(3)]
fps = B * frames * 1e3 / float(np.median(ms))
dev.synthesize(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=frames // 2, ignore_eos=True)
names = dev.ops()
kev = dev.profile_ops_kev(iters=16)
ts = dev.profile_ops_ts(iters=16)
groups = {}
for i, n in enumerate(names):
    groups.setdefault(n, []).append(i)
print(f"== {weights} B={B} ({fn}): {fps:.1f} frames/s, {1e6 * B / fps:.1f} us/iteration (graph), "
      f"{len(names)} launches per iteration")
rows = []
for n, idx in groups.items():
    d = float(np.mean([kev[i] for i in idx]))
    sp = [ts[i] for i in idx if ts[i] > 0]
    rows.append((d * len(idx), n, len(idx), d, float(np.mean(sp)) if sp else -1.0))
for tot, n, k, d, sp in sorted(rows, reverse=True):
    print(f"  {n:14s} {k:3d} x {d:7.2f} us (wave span {sp:6.2f}) = {tot:7.1f} us/iter")
print(f"  dispatch-timed total {sum(r[0] for r in rows):.1f} us/iter")
dev.close()
