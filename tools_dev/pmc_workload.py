"""Workload for the PMC passes (tools_dev/pmc_traffic.sh): the bench's N=1
configuration (Magpie-357M f32, batch 1, T=64, EOS masked) decoded with every
kernel launched eagerly (MAGPIE_EAGER=1 is set by the caller) so rocprofv3 can
attribute counters per dispatch. Writes the op -> kernel symbol order of one
iteration to gpurun_out/pmc_ops.json."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))
import magpie_amd as ma  # noqa: E402

cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
os.makedirs(cache, exist_ok=True)
path = ma.synth_gguf(os.path.join(cache, "magpie_357m_f32.gguf"))
dev = ma.Device(path)
tok = [ma.synthetic_tokens(64, seed=1000)]
r = dev.synthesize(tok, speakers=[0], max_dec_steps=int(os.environ.get("PMC_FRAMES", "64")), ignore_eos=True)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump({"ops": dev.ops(), "frames": int(r.n_frames[0])}, open(os.path.join(REPO, "gpurun_out", "pmc_ops.json"), "w"))
dev.close()
print("pmc workload done", r.n_frames[0], "frames")
