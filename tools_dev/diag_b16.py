"""bf16 batch of 16 vs the same utterance alone: first differing hidden frame and
code (diagnostic)."""
import os, sys
import numpy as np
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
path = ma.synth_gguf(C + "/magpie_small_l2e1.gguf", dec_layers=2, enc_layers=1)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
temp = float(sys.argv[2]) if len(sys.argv) > 2 else 0.7
toks = [ma.synthetic_tokens(9 + 7 * (b % 6), seed=3000 + b) for b in range(B)]
kw = dict(max_dec_steps=64, temperature=temp, top_k=80, seed=17, ignore_eos=True, trace=True)
dev = ma.Device(path, weights="bf16")
rb = dev.synthesize(toks, speakers=[b % 5 for b in range(B)], **kw)
for b in (0, 3, B - 1):
    rs = dev.synthesize([toks[b]], speakers=[b % 5], stream_base=b, **kw)
    d = np.abs(rb.hidden[b] - rs.hidden[0]).max(axis=-1)
    hf = np.nonzero(d)[0]
    cd = np.argwhere(rb.codes[b] != rs.codes[0])
    print(f"B={B} T={temp} slot {b}: hidden first diff frames {hf[:4]} max {d.max():.3g}; codes first diff {cd[:3].tolist()}",
          flush=True)
