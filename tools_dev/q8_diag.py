"""Q8 mode GPU vs oracle weight mode 2: per-step hidden error and decision margins."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
sys.path.insert(0, REPO)
import magpie_amd as ma  # noqa: E402
from oracle import oracle as orc  # noqa: E402

cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
os.makedirs(cache, exist_ok=True)
path = ma.synth_gguf(os.path.join(cache, "magpie_small_q8.gguf"), dtype="q8_0", dec_layers=2, enc_layers=1)
tok = ma.synthetic_tokens(24, seed=1000)
for mode, wname in ((0, "f32"), (2, "q8")):
    dev = ma.Device(path, weights=wname)
    r = dev.synthesize([tok], speakers=[1], max_dec_steps=40, trace=True)
    dev.close()
    orc.set_mode(acc64=True, gelu_f16=False, threads=16)
    om = orc.Model(path)
    om.set_weight_mode(mode)
    o = om.synthesize(tok, speaker=1, max_steps=40, trace=True)
    om.close()
    g, oc = r.codes[0], o["codes"]
    n = min(len(g), len(oc))
    diff = np.argwhere(g[:n] != oc[:n])
    first = int(diff[0][0]) if len(diff) else n
    print(f"mode {wname}: frames gpu {len(g)} oracle {len(oc)} first diff frame {first}")
    for s in range(min(first + 2, 12)):
        e = np.abs(r.hidden[0, s] - o["hidden"][s]).max()
        print(f"  step {s}: hidden max err {e:.3e}  min margin {o['margins'][s].min():.3e}")
    if len(diff):
        f, cb = diff[0]
        print("  first diff", f, cb, g[f].tolist(), oc[f].tolist(), "margin", o["margins"][f, cb])
