"""Decode with and without a concurrent workload on another stream of the same
GPU (codec chunks, or a torch matmul loop): codes and hidden must not change
(diagnostic)."""
import os, sys, threading
import numpy as np
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
p = ma.synth_gguf(C + "/magpie_small_l2e1.gguf", dec_layers=2, enc_layers=1)
cp = ma.synth_gguf(C + "/nano_codec.gguf", kind="codec")
toks = [ma.synthetic_tokens(16 + 9 * b, seed=50 + b) for b in range(2)]
dev = ma.Device(p)
kw = dict(max_dec_steps=96, temperature=0.0, ignore_eos=True, trace=True)
ref = dev.synthesize(toks, speakers=[0, 0], **kw)
cdc = ma.Codec(cp)
stop = False
def codec_loop():
    codes = np.random.default_rng(0).integers(0, 2016, (8, 4)).astype(np.int32)
    n = 0
    while not stop:
        cdc.decode(codes)
        n += 1
    print("codec calls", n, flush=True)
started = threading.Event()
def torch_loop():
    import torch
    a = torch.randn(2048, 2048, device="cuda")
    s = torch.cuda.Stream()
    n = 0
    with torch.cuda.stream(s):
        while not stop:
            a = torch.softmax(a @ a, dim=-1)
            s.synchronize()
            n += 1
            started.set()
    print("torch calls", n, flush=True)
mode = sys.argv[1]
if mode == "seq":  # the codec used before, not during, the decode
    cdc.decode(np.random.default_rng(0).integers(0, 2016, (8, 4)).astype(np.int32))
    th = threading.Thread(target=lambda: None)
elif mode == "noop":  # codec created only
    th = threading.Thread(target=lambda: None)
else:
    th = threading.Thread(target=codec_loop if mode == "codec" else torch_loop)
th.start()
if mode == "torch":
    started.wait(300)
for rep in range(5):
    r = dev.synthesize(toks, speakers=[0, 0], **kw)
    for b in range(2):
        d = np.abs(r.hidden[b] - ref.hidden[b]).max(axis=-1)
        bad = np.nonzero(d)[0]
        print(mode, "rep", rep, "utt", b, "codes equal", np.array_equal(r.codes[b], ref.codes[b]),
              "first hidden diff frame", bad[:3], "max", d.max(), flush=True)
stop = True
th.join()
