"""Graph replay vs eager launches of the same decode (diagnostic): per-frame hidden diffs."""
import os, sys
import numpy as np
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
p = ma.synth_gguf(C + "/magpie_small_l2e1.gguf", dec_layers=2, enc_layers=1)
toks = [ma.synthetic_tokens(16 + 9 * b, seed=50 + b) for b in range(2)]
dev = ma.Device(p)
S = 24
kw = dict(speakers=[0, 0], max_dec_steps=S, ignore_eos=True, trace=True)
os.environ.pop("MAGPIE_EAGER", None)
ref = dev.synthesize(toks, **kw)
for label, eager in (("eager1", True), ("eager2", True), ("graph2", False)):
    if eager:
        os.environ["MAGPIE_EAGER"] = "1"
    else:
        os.environ.pop("MAGPIE_EAGER", None)
    r = dev.synthesize(toks, **kw)
    d = np.abs(r.hidden - ref.hidden).max(axis=(0, 2))
    print(label, "per-frame max diff", np.array2string(d[:8], precision=3), "codes equal",
          all(np.array_equal(r.codes[b], ref.codes[b]) for b in range(2)), flush=True)
