"""Decode vs a codec loop running in ANOTHER process on the same GPU (diagnostic)."""
import os, sys, subprocess, time
import numpy as np
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
if len(sys.argv) > 1 and sys.argv[1] == "child":
    cdc = ma.Codec(ma.synth_gguf(C + "/nano_codec.gguf", kind="codec"))
    codes = np.random.default_rng(0).integers(0, 2016, (8, 4)).astype(np.int32)
    open("/tmp/codec_child_ready", "w").close()
    t0 = time.time()
    while time.time() - t0 < 20 and not os.path.exists("/tmp/codec_child_stop"):
        cdc.decode(codes)
    sys.exit(0)
p = ma.synth_gguf(C + "/magpie_small_l2e1.gguf", dec_layers=2, enc_layers=1)
ma.synth_gguf(C + "/nano_codec.gguf", kind="codec")
NBT = int(os.environ.get("DIAG_B", "2"))
toks = [ma.synthetic_tokens(16 + 9 * b, seed=50 + b) for b in range(NBT)]
dev = ma.Device(p, weights=os.environ.get("DIAG_W", "f32"))
kw = dict(speakers=[0] * NBT, max_dec_steps=96, ignore_eos=True, trace=True)
ref = dev.synthesize(toks, **kw)
for f in ("/tmp/codec_child_ready", "/tmp/codec_child_stop"):
    if os.path.exists(f): os.remove(f)
child = subprocess.Popen([sys.executable, __file__, "child"])
t0 = time.time()
while not os.path.exists("/tmp/codec_child_ready") and time.time() - t0 < 60:
    time.sleep(0.05)
for rep in range(4):
    r = dev.synthesize(toks, **kw)
    d = np.abs(r.hidden - ref.hidden).max(axis=(0, 2)); f = np.nonzero(d)[0]
    print("other-process codec, rep", rep, "first frames", f[:3], "diffs there", d[f[:3]], "codes", [np.nonzero((r.codes[b] != ref.codes[b]).any(-1))[0][:2] for b in range(NBT)], flush=True)
open("/tmp/codec_child_stop", "w").close()
child.wait()
