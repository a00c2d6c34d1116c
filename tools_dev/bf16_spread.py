"""The oracle's own bf16-mode (weight mode 1) arithmetic spread on configs[2]'s shape:
slot 0 of the bf16 B=16 test (Magpie-357M, T=64, 256 frames), f32 accumulation
teacher forced along the f64 run. Prints the largest top-1/top-2 margin shift and the
margins of the decisions that flip: the scale of a rounding-level difference, which
the bf16 near-tie bar (tests/test_long_range_gpu.py TIE_EPS) must cover.
usage: python tools_dev/bf16_spread.py [frames] [threads]"""
import os
import sys
import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
sys.path.insert(0, REPO)
import magpie_amd as ma  # noqa: E402
from oracle import oracle  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 256
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
os.makedirs(cache, exist_ok=True)
path = ma.synth_gguf(os.path.join(cache, "magpie_357m_f32_k32.gguf"), lt_head_scale=ma.DECISIVE)
tok = ma.synthetic_tokens(64, seed=1000)
m = oracle.Model(path)
m.set_weight_mode(1)
oracle.set_mode(acc64=True, gelu_f16=False, threads=threads)
a = m.synthesize(tok, speaker=0, max_steps=frames, ignore_eos=True)
oracle.set_mode(acc64=False, gelu_f16=False, threads=threads)
f = m.synthesize_forced(tok, a["codes"], speaker=0, ignore_eos=True)
m.close()
ma_, fa = np.asarray(a["margins"]), np.asarray(f["margins"])
shift = np.abs(fa - ma_)
diff = np.argwhere(np.asarray(f["codes"]) != np.asarray(a["codes"]))
print(f"{frames} frames: max margin shift {shift.max():.4f} (99.9th pct {np.percentile(shift, 99.9):.4f}); "
      f"{len(diff)} of {frames * 8} decisions flip, at f64 margins {sorted(float(ma_[i, j]) for i, j in diff)}")
