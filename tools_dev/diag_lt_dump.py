"""bf16 batch of 8 vs slot 0 alone, LT state after every launch (MAGPIE_EAGER=1,
MAGPIE_DUMP_LT): the first LT launch whose slot-0 output differs (diagnostic)."""
import os, sys
import numpy as np
os.environ["MAGPIE_EAGER"] = "1"
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
path = ma.synth_gguf(C + "/magpie_small_l2e1.gguf", dec_layers=2, enc_layers=1)
B = 8
toks = [ma.synthetic_tokens(9 + 7 * (b % 6), seed=3000 + b) for b in range(B)]
kw = dict(max_dec_steps=int(os.environ.get("STEPS", "64")), temperature=0.7, top_k=80, seed=17, ignore_eos=True, trace=True)
dev = ma.Device(path, weights="bf16")
dev.synthesize(toks[:1], speakers=[0], **kw)
dev.synthesize(toks, speakers=[b % 5 for b in range(B)], **kw)  # records eager op lists
REC = 2024 + 8 + 4 * 256


def run(bt):
    f = f"gpurun_out/lt_{len(bt)}.bin"
    if os.path.exists(f):
        os.remove(f)
    os.environ["MAGPIE_DUMP_LT"] = f
    r = dev.synthesize(bt, speakers=[b % 5 for b in range(len(bt))], **kw)
    del os.environ["MAGPIE_DUMP_LT"]
    return r, np.fromfile(f, np.float32).reshape(-1, REC)


# per frame: single = lt_in0, lt_a, lt_b, 7 x lt_bg, 8 x (lt_c, lt_d, lt_e) interleaved
def names(batched):
    n = ["lt_in0", "lt_a", "lt_b", "lt_c0", "lt_d0", "lt_e0"]
    for cb in range(1, 8):
        n += ([f"lt_pick{cb}", f"lt_bo{cb}"] if batched else [f"lt_bg{cb}"]) + [f"lt_c{cb}", f"lt_d{cb}", f"lt_e{cb}"]
    return n


rs, ds = run(toks[:1])
rb, db = run(toks)
ns, nb = names(False), names(True)
print("records", ds.shape, db.shape, len(ns), len(nb), flush=True)
fs, fb = ds.reshape(-1, len(ns), REC), db.reshape(-1, len(nb), REC)
key = {n: i for i, n in enumerate(ns)}
done = False
for fr in range(min(len(fs), len(fb))):
    for j, n in enumerate(nb):
        m = n.replace("lt_bo", "lt_bg")
        if m not in key:
            continue
        a, b = fs[fr, key[m]], fb[fr, j]
        if not (np.array_equal(a[:2032], b[:2032]) and np.array_equal(a[2288:2800], b[2288:2800])):
            seg = {"logits": (0, 2024), "codes": (2024, 2032), "ltX": (2032, 2288), "ltY": (2288, 2544),
                   "lty2": (2544, 2800), "ltq": (2800, 3056)}
            diff = {k: float(np.abs(a[s:e] - b[s:e]).max()) for k, (s, e) in seg.items()}
            print("frame", fr, "first differing op", n, diff, flush=True)
            print(" codes single", a[2024:2032].view(np.int32), "batch", b[2024:2032].view(np.int32))
            done = True
            break
    if done:
        break
print("codes equal", np.array_equal(rs.codes[0], rb.codes[0]))
