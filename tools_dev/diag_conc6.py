"""Which stage changes beside a codec loop in another process? Preamble buffers
(encoder output, XA K/V, SA cache of the 110 context frames) compared with the
run alone, then the BOS step. Diagnostic."""
import os, subprocess, sys, time
import numpy as np
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
p = ma.synth_gguf(C + "/magpie_small_l2e1.gguf", dec_layers=2, enc_layers=1)
cp = ma.synth_gguf(C + "/nano_codec.gguf", kind="codec")
toks = [ma.synthetic_tokens(16 + 9 * b, seed=50 + b) for b in range(2)]
dev = ma.Device(p)
kw = dict(speakers=[0, 0], max_dec_steps=4, ignore_eos=True, trace=True)
NAMES = ["enc_out", "xak", "xav", "kc", "vc"]


def snap():
    dev.begin(toks, **kw)
    d = {n: dev.debug_buffer(n) for n in NAMES}
    r = dev.decode(2, 4, True)
    d["hidden0"] = r.hidden[:, 0].ravel()
    return d


ref = snap()
again = snap()
print("alone twice:", {n: float(np.abs(again[n] - ref[n]).max()) for n in ref}, flush=True)
mode = sys.argv[1] if len(sys.argv) > 1 else "codec"
child = subprocess.Popen([sys.executable, "tools_dev/diag_conc5.py", "child", "25"] if mode == "codec"
                         else ["tools_dev/garbage/garbage", mode, "25"])
time.sleep(8.0)
for rep in range(4):
    s = snap()
    print(f"{mode} rep{rep}:", {n: float(np.abs(s[n] - ref[n]).max()) for n in ref}, flush=True)
child.wait()
