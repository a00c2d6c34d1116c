"""Codec wall time per call at streaming chunk sizes (graph replay vs MAGPIE_EAGER)."""
import os, sys, time
import numpy as np
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
cdc = ma.Codec(ma.synth_gguf(C + "/nano_codec.gguf", kind="codec"))
for F, n in ((4, 1), (4, 8), (32, 8)):
    codes = np.random.default_rng(0).integers(0, 2016, (n, 8, F)).astype(np.int32)
    cdc.decode_chunks(codes)
    ts, ds = [], []
    for _ in range(20):
        t = time.perf_counter(); cdc.decode_chunks(codes); ts.append((time.perf_counter() - t) * 1e3)
        ds.append(cdc.last_ms())
    print(f"eager={os.environ.get('MAGPIE_EAGER', '0')} F={F} chunks={n}: wall {np.median(ts):.3f} ms, device {np.median(ds):.3f} ms"
          f" (min {min(ds):.3f})", flush=True)
