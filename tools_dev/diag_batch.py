"""Slot 0's local-transformer state after every frame, batched (B=2) vs single (diagnostic)."""
import os, sys
import numpy as np
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
p = ma.synth_gguf(C + "/magpie_small_l2e1.gguf", dec_layers=2, enc_layers=1)
tk = ma.Tokenizer(p)
toks = [tk(s) for s in ["Hello, world!", "The first voice, 21st of May."]]
kw = dict(max_dec_steps=3, temperature=0.7, top_k=80, seed=0, trace=True, ignore_eos=True)
dev = ma.Device(p)
for f in ("gpurun_out/lg_b.bin", "gpurun_out/lg_s.bin"):
    if os.path.exists(f): os.remove(f)
os.environ["MAGPIE_DUMP_LOGITS"] = "gpurun_out/lg_b.bin"
rb = dev.synthesize(toks, speakers=[0, 0], **kw)
os.environ["MAGPIE_DUMP_LOGITS"] = "gpurun_out/lg_s.bin"
r1 = dev.synthesize([toks[0]], speakers=[0], **kw)
names = [("hidden", 768), ("lt_s", 2304), ("ltX", 256), ("ltq", 256), ("ltk", 2048), ("ltv", 2048), ("ltY", 256),
         ("ltf", 1024), ("lty2", 256), ("logits", 2024)]
tot = sum(n for _, n in names)
lb = np.fromfile("gpurun_out/lg_b.bin", np.float32).reshape(3, tot)
ls = np.fromfile("gpurun_out/lg_s.bin", np.float32).reshape(3, tot)
for f in range(3):
    o = 0
    out = []
    for nm, n in names:
        d = np.abs(lb[f, o:o + n] - ls[f, o:o + n])
        out.append(f"{nm}:{d.max():.2e}")
        if nm in ("ltk", "ltv", "lt_s"):
            rows = d.reshape(-1, 256).max(axis=1)
            out.append("rows[" + " ".join(f"{r:.0e}" for r in rows) + "]")
        o += n
    print("frame", f, " ".join(out), flush=True)
