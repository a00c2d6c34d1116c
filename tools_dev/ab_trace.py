"""A/B numerics: one decode with the library MAGPIE_LIB names (or the default),
saved as gpurun_out/<tag>.npz (codes, hidden trace). Usage: ab_trace.py TAG WEIGHTS [B]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "magpie-tts.cpp_amd"))
import magpie_amd as ma  # noqa: E402

tag, weights = sys.argv[1], sys.argv[2]
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1
cache = "/tmp/magpie_amd_cache"
os.makedirs(cache, exist_ok=True)
path = ma.synth_gguf(os.path.join(cache, "magpie_357m_f32_k32.gguf"), lt_head_scale=ma.DECISIVE)
dev = ma.Device(path, weights=weights)
toks = [ma.synthetic_tokens(64, seed=1000 + b) for b in range(B)]
r = dev.synthesize(toks, speakers=[0] * B, max_dec_steps=24, ignore_eos=True, trace=True)
os.makedirs("gpurun_out", exist_ok=True)
np.savez(f"gpurun_out/{tag}.npz", codes=r.codes, hidden=r.hidden)
print(tag, "saved")
