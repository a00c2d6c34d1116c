"""Batched (B=2) vs one-sentence streams on the small model at temperature 0.7:
device codes, delivered frames and audio per utterance (diagnostic)."""
import os, sys
import numpy as np
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
p = ma.synth_gguf(C + "/magpie_small_l2e1.gguf", dec_layers=2, enc_layers=1)
cp = ma.synth_gguf(C + "/nano_codec.gguf", kind="codec")
tk = ma.Tokenizer(p)
toks = [tk(s) for s in ["Hello, world!", "The first voice, 21st of May."]]
kw = dict(max_dec_steps=500, temperature=0.7, top_k=80, seed=0, frames_per_chunk=4)
dev = ma.Device(p)
cdc = ma.Codec(cp)
ch_b = [[], []]
cb_, tot_b, _ = dev.synthesize_stream(cdc, toks, lambda u, a: ch_b[u].append(a), speakers=[0, 0], **kw)
for i in range(2):
    ch_s = []
    cs, tot_s, _ = dev.synthesize_stream(cdc, [toks[i]], lambda u, a: ch_s.append(a), speakers=[0], stream_base=i, **kw)
    ab, as_ = np.concatenate(ch_b[i]), np.concatenate(ch_s)
    n = min(len(cb_[i]), len(cs[0]))
    fd = np.nonzero((cb_[i][:n] != cs[0][:n]).any(axis=-1))[0]
    print(i, "frames batch/single", len(cb_[i]), len(cs[0]), "first code diff", fd[:3], "audio len", len(ab), len(as_),
          "chunks", len(ch_b[i]), len(ch_s), flush=True)
    for k in range(min(len(ch_b[i]), len(ch_s))):
        if not np.array_equal(ch_b[i][k], ch_s[k]):
            print("   first differing chunk", k, flush=True)
            break
