"""Decode beside a process that leaves NaN in LDS/VGPRs (tools_dev/garbage) (diagnostic)."""
import os, sys, subprocess, time
import numpy as np
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
p = ma.synth_gguf(C + "/magpie_small_l2e1.gguf", dec_layers=2, enc_layers=1)
toks = [ma.synthetic_tokens(16 + 9 * b, seed=50 + b) for b in range(2)]
dev = ma.Device(p)
kw = dict(speakers=[0, 0], max_dec_steps=96, ignore_eos=True, trace=True)
ref = dev.synthesize(toks, **kw)
child = subprocess.Popen(["tools_dev/garbage/garbage", sys.argv[1], "8"])
time.sleep(1.0)
for rep in range(4):
    r = dev.synthesize(toks, **kw)
    d = np.abs(r.hidden - ref.hidden).max(axis=(0, 2))
    bad = np.nonzero(~(d == 0))[0]
    print(sys.argv[1], "rep", rep, "max diff", np.nanmax(d) if np.isfinite(d).any() else d.max(), "nan frames",
          np.nonzero(np.isnan(d))[0][:5], "first bad", bad[:5], flush=True)
child.wait()
