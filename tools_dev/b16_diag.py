"""bf16 mode: GPU vs oracle hidden-error per step (diagnostic, GPU box)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
sys.path.insert(0, REPO)
import magpie_amd as ma  # noqa: E402
from oracle import oracle as orc  # noqa: E402

cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
path = os.path.join(cache, "magpie_small_l2e1.gguf")
ma.synth_gguf(path, dec_layers=2, enc_layers=1)
tok = ma.synthetic_tokens(24, seed=1000)
H = {}
for w in ("f32", "bf16"):
    d = ma.Device(path, weights=w)
    r = d.synthesize([tok], speakers=[1], max_dec_steps=4, trace=True, ignore_eos=True)
    d.close()
    H["gpu_" + w] = r.hidden[0]
for mode in (0, 1):
    m = orc.Model(path)
    m.set_weight_mode(mode)
    o = m.synthesize(tok, speaker=1, max_steps=4, trace=True, ignore_eos=True)
    m.close()
    H["orc_" + ("f32" if mode == 0 else "bf16")] = o["hidden"]
keys = list(H)
for i in range(len(keys)):
    for j in range(i + 1, len(keys)):
        a, b = H[keys[i]], H[keys[j]]
        print(f"{keys[i]:9s} vs {keys[j]:9s}", [float(np.abs(a[s] - b[s]).max()) for s in range(3)])
