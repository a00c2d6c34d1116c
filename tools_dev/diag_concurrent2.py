"""Which phase does a concurrent codec corrupt: preamble (begin) or frame loop (decode)?"""
import os, sys, threading, time
import numpy as np
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
p = ma.synth_gguf(C + "/magpie_small_l2e1.gguf", dec_layers=2, enc_layers=1)
cp = ma.synth_gguf(C + "/nano_codec.gguf", kind="codec")
toks = [ma.synthetic_tokens(16 + 9 * b, seed=50 + b) for b in range(2)]
dev = ma.Device(p)
S = 96
ref = dev.synthesize(toks, speakers=[0, 0], max_dec_steps=S, ignore_eos=True, trace=True)
cdc = ma.Codec(cp)
busy = threading.Event()
stop = threading.Event()
def codec_loop():
    codes = np.random.default_rng(0).integers(0, 2016, (8, 4)).astype(np.int32)
    while not stop.is_set():
        if busy.is_set():
            cdc.decode(codes)
        else:
            time.sleep(0.0005)
th = threading.Thread(target=codec_loop)
th.start()
def run(pre_busy, dec_busy):
    (busy.set if pre_busy else busy.clear)()
    time.sleep(0.01)
    B = dev.begin(toks, [0, 0], S, 0.0, 80, True, 0, True, 0)
    (busy.set if dec_busy else busy.clear)()
    time.sleep(0.01)
    r = dev.decode(B, S, True)
    busy.clear()
    time.sleep(0.01)
    d = max(np.abs(r.hidden[b] - ref.hidden[b]).max() for b in range(2))
    print("codec during preamble", pre_busy, "during decode", dec_busy, "max hidden diff", d, flush=True)
for rep in range(2):
    run(False, False)
    run(True, False)
    run(False, True)
stop.set()
th.join()
