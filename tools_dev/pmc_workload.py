"""Workloads for the PMC passes (tools_dev/pmc_collect.sh), every kernel launched
eagerly (MAGPIE_EAGER=1 is set by the caller) so rocprofv3 attributes counters per
dispatch:
  decode WEIGHTS B : the bench's model (Magpie-357M, decisive LT heads; WEIGHTS q8:
                     its Q8_0 twin), T=64, EOS
                     masked, 64 frames; writes the op order of one iteration to
                     gpurun_out/pmc_ops_<WEIGHTS>_<B>.json
  codec            : the bench's codec shape, 8 chunks x 32 frames, 4 decodes"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
import magpie_amd as ma  # noqa: E402

cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
os.makedirs(cache, exist_ok=True)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
mode = sys.argv[1] if len(sys.argv) > 1 else "decode"
if mode == "codec":
    c = ma.Codec(ma.synth_gguf(os.path.join(cache, "nano_codec.gguf"), kind="codec"))
    codes = np.random.default_rng(1).integers(0, 2016, (8, 8, 32)).astype(np.int32)
    for _ in range(4):
        c.decode_chunks(codes)
    c.close()
    json.dump({"lib_sha16": ma.lib_sha16()}, open(os.path.join(REPO, "gpurun_out", "pmc_codec_build.json"), "w"))
    print("pmc codec workload done")
else:
    weights = sys.argv[2] if len(sys.argv) > 2 else "f32"
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    if weights == "q8":  # the reference converter's Q8_0 patterns (int8 MFMA decode projections)
        path = ma.synth_gguf(os.path.join(cache, "magpie_357m_q8_k32.gguf"), dtype="q8_0", lt_head_scale=ma.DECISIVE)
    else:
        path = ma.synth_gguf(os.path.join(cache, "magpie_357m_f32_k32.gguf"), lt_head_scale=ma.DECISIVE)
    dev = ma.Device(path, weights=weights)
    toks = [ma.synthetic_tokens(64, seed=1000 + b) for b in range(B)]
    r = dev.synthesize(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=int(os.environ.get("PMC_FRAMES", "64")),
                       ignore_eos=True)
    json.dump({"ops": dev.ops(), "frames": int(r.n_frames[0]), "lib_sha16": ma.lib_sha16()},
              open(os.path.join(REPO, "gpurun_out", f"pmc_ops_{weights}_{B}.json"), "w"))
    dev.close()
    print("pmc decode workload done", weights, B, r.n_frames[0], "frames")
