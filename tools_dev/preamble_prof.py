"""Per-kernel time of ONE preamble (mp_hip_begin_batch: encoder, XA K/V, K'/V', 110-frame
prefill) at the bench's shape, for rocprofv3 --kernel-trace. Runs the preamble REPS times
after a warm-up, bracketed by profile marks; tools_dev/preamble_report.py cuts the trace.
usage: preamble_prof.py [weights=f32] [B=1] [T=64] [REPS=3]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
import magpie_amd as ma  # noqa: E402

weights = sys.argv[1] if len(sys.argv) > 1 else "f32"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
T = int(sys.argv[3]) if len(sys.argv) > 3 else 64
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
os.makedirs(cache, exist_ok=True)
path = ma.synth_gguf(os.path.join(cache, "magpie_357m_f32_k32.gguf"), lt_head_scale=ma.DECISIVE)
dev = ma.Device(path, weights=weights)
toks = [ma.synthetic_tokens(T, seed=1000 + b) for b in range(B)]
dev.begin(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=256, ignore_eos=True)  # warm-up (allocates)
ms = []
for r in range(reps):
    t0 = time.perf_counter()
    dev.begin(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=256, ignore_eos=True)
    ms.append((time.perf_counter() - t0) * 1e3)
print(f"preamble {weights} B={B} T={T}: wall ms per call {[round(x, 3) for x in ms]}")
dev.close()
