"""Localise the first launch whose output changes while an MFMA neighbour runs
(MAGPIE_EAGER=1 MAGPIE_DUMP_OPS; needs tools_dev/dump_ops.patch applied and the library rebuilt): two decode frames dumped op by op, clean and
beside tools_dev/garbage/garbage mfma, compared record by record (diagnostic)."""
import os, sys, subprocess, time
import numpy as np
os.environ["MAGPIE_EAGER"] = "1"
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
p = ma.synth_gguf(C + "/magpie_small_l2e1.gguf", dec_layers=2, enc_layers=1)
toks = [ma.synthetic_tokens(16, seed=50)]
dev = ma.Device(p)
kw = dict(speakers=[0], max_dec_steps=2, ignore_eos=True, trace=True)
dev.synthesize(toks, **kw)  # records the eager op list
NAMES = [("x", 768), ("x2", 768), ("q", 768), ("h", 3072), ("logits", 2024), ("ltY", 256), ("sa_part", 3264),
         ("xa_part", 3088)]
REC = sum(n for _, n in NAMES)


def dumped(path):
    if os.path.exists(path):
        os.remove(path)
    os.environ["MAGPIE_DUMP_OPS"] = path
    dev.synthesize(toks, **kw)
    os.environ.pop("MAGPIE_DUMP_OPS")
    return np.fromfile(path, np.float32).reshape(-1, REC)


a = dumped("gpurun_out/ops_a.bin")
names = dev.ops()
child = subprocess.Popen(["tools_dev/garbage/garbage", "mfma", "6"])
time.sleep(1.0)
bs = [dumped(f"gpurun_out/ops_b{k}.bin") for k in range(3)]
child.wait()
print("records per run", a.shape[0], "ops per iteration", len(names), flush=True)
for k, b in enumerate(bs):
    diff = np.nonzero((a != b).any(axis=1))[0]
    if len(diff) == 0:
        print("run", k, "identical", flush=True)
        continue
    r = int(diff[0])
    o = 0
    which = []
    for nm, n in NAMES:
        d = np.abs(a[r, o:o + n] - b[r, o:o + n])
        if d.max() > 0:
            which.append(f"{nm}:{d.max():.2e}@{int(d.argmax())}")
        o += n
    print("run", k, "first differing record", r, "op", names[r % len(names)] if r < 2 * len(names) else "?",
          "(previous", names[(r - 1) % len(names)], ")", which, flush=True)
