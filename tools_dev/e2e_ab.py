"""configs[2] end to end (bench.py measure_configs2_e2e) under several codec background
CU shares, alternating: e2e_ab.py CUS[,CUS...] ROUNDS  (MAGPIE_CODEC_BG_CUS per setting)."""
import json
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402  (loads the library)

ma = bench.ma
cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
os.makedirs(cache, exist_ok=True)
model = ma.synth_gguf(os.path.join(cache, "magpie_357m_f32_k32.gguf"), lt_head_scale=ma.DECISIVE)
codec = ma.synth_gguf(os.path.join(cache, "nano_codec.gguf"), kind="codec")
# a setting: CUS or CUS/ASYNC (MAGPIE_CODEC_BG_CUS, MAGPIE_STREAM_ASYNC)
settings = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "64"]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
args = types.SimpleNamespace(frames=bench.FRAMES, tokens=bench.TEXT_TOKENS)
for r in range(rounds):
    for st in settings:
        cus, _, asy = st.partition("/")
        os.environ["MAGPIE_CODEC_BG_CUS"] = cus
        os.environ["MAGPIE_STREAM_ASYNC"] = asy or "1"
        res = bench.measure_configs2_e2e(model, codec, args)
        print(json.dumps({"bg_cus": int(cus), "async": int(asy or "1"), "fps": res["fps"], "decode_only_fps": res["decode_only_fps"],
                          "serial_fps": res["serial_fps"], "ratio": res["e2e_over_decode_only"]}), flush=True)
