"""Decode beside a codec loop: in this process (thread, own stream) or in a child
process; then alone again (does anything persist?). Diagnostic."""
import os, subprocess, sys, threading, time
import numpy as np
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
p = ma.synth_gguf(C + "/magpie_small_l2e1.gguf", dec_layers=2, enc_layers=1)
cp = ma.synth_gguf(C + "/nano_codec.gguf", kind="codec")
if sys.argv[1] == "child":
    cdc = ma.Codec(cp)
    codes = np.random.default_rng(0).integers(0, 2016, (8, 8, 32)).astype(np.int32)
    t0 = time.time()
    n = 0
    while time.time() - t0 < float(sys.argv[2]):
        cdc.decode_chunks(codes)
        n += 1
    print("child codec calls", n, flush=True)
    sys.exit(0)
toks = [ma.synthetic_tokens(16 + 9 * b, seed=50 + b) for b in range(2)]
dev = ma.Device(p)
kw = dict(speakers=[0, 0], max_dec_steps=int(os.environ.get("STEPS", "96")), ignore_eos=True, trace=True)
ref = dev.synthesize(toks, **kw)


def report(tag, r):
    for b in range(2):
        d = np.abs(r.hidden[b] - ref.hidden[b]).max(axis=-1)
        bad = np.nonzero(d)[0]
        print(tag, "utt", b, "codes equal", np.array_equal(r.codes[b], ref.codes[b]), "first diff frames", bad[:4],
              "max", d.max(), flush=True)


mode = sys.argv[1]
stop = threading.Event()
if mode == "thread":
    cdc = ma.Codec(cp)
    def loop():
        codes = np.random.default_rng(0).integers(0, 2016, (8, 8, 32)).astype(np.int32)
        while not stop.is_set():
            cdc.decode_chunks(codes)
    th = threading.Thread(target=loop)
    th.start()
    time.sleep(0.5)
    for rep in range(3):
        report(f"thread rep{rep}", dev.synthesize(toks, **kw))
    stop.set()
    th.join()
elif mode == "proc":
    child = subprocess.Popen([sys.executable, __file__, "child", "20"])
    time.sleep(8.0)
    for rep in range(3):
        report(f"proc rep{rep}", dev.synthesize(toks, **kw))
    child.wait()
for rep in range(2):
    report(f"after rep{rep}", dev.synthesize(toks, **kw))
