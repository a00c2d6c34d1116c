"""Eager decode at a given batch / weight mode for rocprofv3 kernel traces:
trace_batch.py WEIGHTS B FRAMES (run with MAGPIE_EAGER=1 under rocprofv3)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
import magpie_amd as ma  # noqa: E402

cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
os.makedirs(cache, exist_ok=True)
weights, B, F = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
path = ma.synth_gguf(os.path.join(cache, "magpie_357m_q8.gguf" if weights == "q8" else "magpie_357m_f32.gguf"),
                     dtype="q8_0" if weights == "q8" else "f32")
dev = ma.Device(path, weights=weights)
toks = [ma.synthetic_tokens(64, seed=1000 + b) for b in range(B)]
r = dev.synthesize(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=F, ignore_eos=True)
print(weights, B, "decode_ms", r.decode_ms)
dev.close()
