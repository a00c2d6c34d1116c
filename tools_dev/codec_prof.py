"""Codec workload for rocprofv3: 8 chunks x 32 frames (the bench's shape), 4 decodes."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
import magpie_amd as ma  # noqa: E402

cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
os.makedirs(cache, exist_ok=True)
c = ma.Codec(ma.synth_gguf(os.path.join(cache, "nano_codec.gguf"), kind="codec"))
codes = np.random.default_rng(1).integers(0, 2016, (int(os.environ.get("NCHUNK", "8")), 8, 32)).astype(np.int32)
for _ in range(4):
    c.decode_chunks(codes)
print("codec ms", c.last_ms())
