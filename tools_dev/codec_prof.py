"""Codec per-launch trace workload: 3 decodes of 8 x 32-frame chunks (run under
rocprofv3 --kernel-trace; tools_dev/codec_trace_report.py maps dispatches to stages)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "magpie-tts.cpp_amd"))
import magpie_amd as ma
C = "/tmp/magpie_amd_cache"
os.makedirs(C, exist_ok=True)
cdc = ma.Codec(ma.synth_gguf(C + "/nano_codec.gguf", kind="codec"))
codes = np.random.default_rng(0).integers(0, 2016, (8, 8, 32)).astype(np.int32)
for _ in range(3):
    cdc.decode_chunks(codes)
    print(f"device {cdc.last_ms():.3f} ms", flush=True)
