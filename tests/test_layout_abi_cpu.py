"""CPU-only checks of the boundary: GGUF layout of the synthetic weights, the
C-ABI library's exports, error behaviour without a GPU, and the committed golden
fixtures."""
import json
import os
import re
import struct
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "include", "magpie_hip.h")


def read_gguf_index(path):
    """Independent minimal GGUF v3 index reader (header + tensor infos)."""
    with open(path, "rb") as f:
        assert f.read(4) == b"GGUF"
        ver, = struct.unpack("<I", f.read(4))
        nt, nkv = struct.unpack("<QQ", f.read(16))

        def rstr():
            n, = struct.unpack("<Q", f.read(8))
            return f.read(n).decode()
        sizes = {0: 1, 1: 1, 2: 2, 3: 2, 4: 4, 5: 4, 6: 4, 7: 1, 10: 8, 11: 8, 12: 8}
        kv = {}

        def rval(t):
            if t == 8:
                return rstr()
            if t == 9:
                et, = struct.unpack("<I", f.read(4))
                n, = struct.unpack("<Q", f.read(8))
                return [rval(et) for _ in range(n)]
            b = f.read(sizes[t])
            return struct.unpack({4: "<I", 5: "<i", 6: "<f"}.get(t, "<Q" if sizes[t] == 8 else "<B"), b)[0]
        for _ in range(nkv):
            k = rstr()
            t, = struct.unpack("<I", f.read(4))
            kv[k] = rval(t)
        tensors = {}
        for _ in range(nt):
            name = rstr()
            nd, = struct.unpack("<I", f.read(4))
            ne = struct.unpack("<" + "Q" * nd, f.read(8 * nd))
            typ, off = struct.unpack("<IQ", f.read(12))
            tensors[name] = (tuple(reversed(ne)), typ, off)
    return ver, kv, tensors


# Tensor names/shapes mapped by create_tensors (magpie.cpp:572-672), shapes per
# docs/MAGPIE_ARCHITECTURE.md:265-307 (PyTorch order).
def expected_magpie(dec_layers=12, enc_layers=6):
    e = {"text_embedding.weight": (2380, 768), "encoder.position_embeddings.weight": (4096, 768),
         "encoder.norm_out.weight": (768,), "decoder.norm_out.weight": (768,),
         "baked_context_embedding.weight": (5, 84480), "final_proj.weight": (16192, 768), "final_proj.bias": (16192,),
         "local_transformer_in_projection.weight": (256, 768), "local_transformer_in_projection.bias": (256,),
         "local_transformer.position_embeddings.weight": (10, 256),
         "local_transformer.layers.0.norm_self.weight": (256,),
         "local_transformer.layers.0.self_attention.qkv_net.weight": (768, 256),
         "local_transformer.layers.0.self_attention.o_net.weight": (256, 256),
         "local_transformer.layers.0.norm_pos_ff.weight": (256,),
         "local_transformer.layers.0.pos_ff.proj.conv.weight": (1024, 256, 1),
         "local_transformer.layers.0.pos_ff.o_net.conv.weight": (256, 1024, 1)}
    for l in range(enc_layers):
        p = f"encoder.layers.{l}."
        e.update({p + "norm_self.weight": (768,), p + "self_attention.qkv_net.weight": (2304, 768),
                  p + "self_attention.o_net.weight": (768, 768), p + "norm_pos_ff.weight": (768,),
                  p + "pos_ff.proj.conv.weight": (3072, 768, 3), p + "pos_ff.o_net.conv.weight": (768, 3072, 3)})
    for l in range(dec_layers):
        p = f"decoder.layers.{l}."
        e.update({p + "norm_self.weight": (768,), p + "self_attention.qkv_net.weight": (2304, 768),
                  p + "self_attention.o_net.weight": (768, 768), p + "norm_xattn_query.weight": (768,),
                  p + "cross_attention.q_net.weight": (128, 768), p + "cross_attention.kv_net.weight": (256, 768),
                  p + "cross_attention.o_net.weight": (768, 128), p + "norm_xattn_memory.weight": (768,),
                  p + "norm_pos_ff.weight": (768,), p + "pos_ff.proj.conv.weight": (3072, 768, 1),
                  p + "pos_ff.o_net.conv.weight": (768, 3072, 1)})
    for c in range(8):
        e[f"audio_embeddings.{c}.weight"] = (2024, 768)
        e[f"local_transformer_out_projections.{c}.weight"] = (2024, 256)
        e[f"local_transformer_out_projections.{c}.bias"] = (2024,)
    return e


def test_magpie_gguf_layout(small_model):
    ver, kv, t = read_gguf_index(small_model)
    assert ver == 3
    exp = expected_magpie(dec_layers=2, enc_layers=1)
    exp["decoder.position_embeddings.weight"] = t["decoder.position_embeddings.weight"][0]
    assert t["decoder.position_embeddings.weight"][0][0] >= 610  # max position 110 + 499
    assert {k: v[0] for k, v in t.items()} == exp
    assert all(v[1] == 0 for v in t.values())  # F32 file
    assert all(v[2] % 32 == 0 for v in t.values())  # 32-byte aligned data
    assert kv["magpie.d_model"] == 768 and kv["magpie.audio_eos_id"] == 2017
    assert kv["magpie.dec_layers"] == 2 and kv["magpie.enc_layers"] == 1


def test_q8_gguf_quantizes_reference_patterns(q8_model):
    """convert_magpie_to_gguf.py:155-176,311-320: attention/LT projections Q8_0;
    pos_ff conv weights stay F32 (inner dim 1 or 3 < 32)."""
    _, _, t = read_gguf_index(q8_model)
    q8 = {k for k, v in t.items() if v[1] == 8}
    assert "decoder.layers.0.self_attention.qkv_net.weight" in q8
    assert "decoder.layers.1.cross_attention.kv_net.weight" in q8
    assert "local_transformer_out_projections.7.weight" in q8
    assert "local_transformer_in_projection.weight" in q8
    assert "decoder.layers.0.pos_ff.proj.conv.weight" not in q8
    assert "encoder.layers.0.pos_ff.o_net.conv.weight" not in q8
    assert "audio_embeddings.0.weight" not in q8


def test_q8_block_semantics_match_converter(tmp_path):
    """Q8_0 = fp16 scale amax/127 + round-half-even int8 (convert_magpie_to_gguf.py:79-104),
    re-derived with numpy from the F32 twin of the same tensor."""
    import magpie_amd as ma
    f32 = ma.synth_gguf(str(tmp_path / "a.gguf"), dec_layers=1, enc_layers=1)
    q8 = ma.synth_gguf(str(tmp_path / "b.gguf"), dtype="q8_0", dec_layers=1, enc_layers=1)
    name = "decoder.layers.0.cross_attention.q_net.weight"
    _, _, t32 = read_gguf_index(f32)
    _, _, t8 = read_gguf_index(q8)

    def data_start(path):
        """(file bytes, offset of the 32-aligned data section)"""
        with open(path, "rb") as f:
            buf = f.read()
        p = 24
        def rstr(p):
            ln, = struct.unpack_from("<Q", buf, p)
            return p + 8 + ln
        nt, nkv = struct.unpack_from("<QQ", buf, 8)
        for _ in range(nkv):
            p = rstr(p)
            t, = struct.unpack_from("<I", buf, p); p += 4
            if t == 8:
                p = rstr(p)
            else:
                p += {4: 4, 5: 4, 6: 4}[t]
        for _ in range(nt):
            p = rstr(p)
            nd, = struct.unpack_from("<I", buf, p); p += 4 + 8 * nd + 12
        return buf, (p + 31) // 32 * 32
    shape, _, off32 = t32[name]
    n = int(np.prod(shape))
    b32, s32 = data_start(f32)
    b8, s8 = data_start(q8)
    x = np.frombuffer(b32, np.float32, n, s32 + off32).reshape(-1, 32)
    blk = np.frombuffer(b8, np.dtype([("d", "<f2"), ("q", "i1", 32)]), n // 32, s8 + t8[name][2])
    amax = np.abs(x).max(axis=1)
    d = (amax / 127.0).astype(np.float16)
    np.testing.assert_array_equal(blk["d"], d)
    q = np.round(x / d.astype(np.float32)[:, None]).astype(np.int8)
    np.testing.assert_array_equal(blk["q"], q)


def test_codec_gguf_layout(codec_model):
    """nano-codec.cpp:84-199 names (shortened by convert_codec_to_gguf.py:110-132)."""
    _, kv, t = read_gguf_index(codec_model)
    assert t["dec.pre.weight"][0] == (864, 32, 7)
    assert t["dec.post.weight"][0] == (1, 27, 3)
    assert t["dec.post_act.alpha"][0] == (1, 13, 1)
    assert t["dec.up.0.c.weight"][0] == (864, 1, 16)
    assert t["dec.up.4.c.weight"][0] == (54, 1, 4)
    assert t["dec.rl.2.rb.1.rb.0.in_conv.weight"][0] == (108, 108, 7)
    assert t["dec.rl.4.rb.2.rb.2.sk_act.alpha"][0] == (1, 13, 1)
    assert t["dec.act.0.activation.snake_act.alpha"][0] == (1, 432, 1)
    assert t["vq.fsqs.7.num_levels"][0] == (1, 4, 1)
    assert len(t) == 2 + 2 + 1 + 5 * (3 + 9 * 6) + 16
    assert kv["codec.hop_length"] == 1024


def test_generator_is_deterministic(tmp_path):
    import magpie_amd as ma
    a = ma.synth_gguf(str(tmp_path / "x.gguf"), kind="codec")
    b = ma.synth_gguf(str(tmp_path / "y.gguf"), kind="codec")
    assert open(a, "rb").read() == open(b, "rb").read()


def _declared_symbols():
    src = open(HDR).read()
    return sorted(set(re.findall(r"\b(mp_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import magpie_amd as ma
    lib = ma.load_library()
    declared = _declared_symbols()
    assert len(declared) >= 15
    for s in declared:
        assert hasattr(lib, s), s
    assert {s for s, _, _ in ma.SYMBOLS} == set(declared)
    # C++ drop-in API (include/magpie.h) is exported from the same library
    out = subprocess.run(["nm", "-DC", ma.LIB_PATH], capture_output=True, text=True).stdout
    for fn in ["magpie_init(char const*)", "magpie_free(magpie_context*)",
               "magpie_synthesize_codes_graph_reuse(magpie_context*, int const*, int)",
               "magpie_codec_decode(magpie_codec*, int const*, int)", "magpie_codec_init(char const*)",
               "magpie_local_transformer_sample_all(magpie_context*, float const*, float, int, bool)",
               "magpie_split_sentences[abi:cxx11](char const*)",
               "magpie_synthesize_streaming(magpie_context*, magpie_codec*, char const*, magpie_stream_params const&)",
               "magpie_synthesize_sentence_streaming(magpie_context*, magpie_codec*, int const*, int, "
               "magpie_stream_params const&)",
               "magpie_tokenize(magpie_tokenizer const*, std::__cxx11::basic_string<char, std::char_traits<char>, "
               "std::allocator<char> > const&)"]:
        assert fn in out, fn


def test_no_device_fails_loudly():
    """No GPU in this container: the product path must refuse, not fall back."""
    import magpie_amd as ma
    if ma.device_count() > 0:
        pytest.skip("a HIP device is visible")
    with pytest.raises(ma.MagpieError):
        ma.Device("/nonexistent.gguf")
    import ctypes
    h = ctypes.c_void_p()
    assert ma.load_library().mp_hip_init(0, ctypes.byref(h)) != 0


def test_golden_small_model_matches_oracle(oracle, small_model):
    """The committed oracle fixture still reproduces (oracle regression pin)."""
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "small_model_codes.json")))
    case = g["cases"][1]
    m = oracle.Model(small_model)
    r = m.synthesize(np.array(case["tokens"], np.int32), speaker=case["speaker"], max_steps=case["max_steps"])
    m.close()
    assert r["n_frames"] == case["n_frames"]
    np.testing.assert_array_equal(r["codes"], np.array(case["codes"]))
    np.testing.assert_allclose(np.abs(r["hidden"][:r["n_frames"] + 1]).sum(axis=1), case["hidden_l1"], rtol=1e-6)


def test_bench_bytes_per_frame_matches_survey():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    # ~388.4 MB/frame at B=1, L=238.5, T=64 (f32)
    assert abs(bench.decoder_bytes_per_frame(1, 238.5, 64) / 1e6 - 388.4) < 0.5


def _gfx950_code_objects(so_path, tmp_path):
    """Every gfx950 code object in a HIP shared library: the .hip_fatbin section is a
    run of clang offload bundles (one per translation unit), each '__CLANG_OFFLOAD_
    BUNDLE__' + entry count + (offset, size, triple) records, offsets from its start."""
    sec = tmp_path / "fatbin.bin"
    subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objcopy", f"--dump-section=.hip_fatbin={sec}", so_path,
                    str(tmp_path / "discard.so")], check=True)
    data = sec.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out, pos = [], data.find(magic)
    while pos >= 0:
        n, = struct.unpack_from("<Q", data, pos + 24)
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and size:
                co = tmp_path / f"co{len(out)}.elf"
                co.write_bytes(data[pos + off:pos + off + size])
                out.append(co)
        pos = data.find(magic, pos + 1)
    return out


def test_library_has_no_packed_fp32_instructions(tmp_path):
    """v_pk_fma/mul/add_f32 returned wrong values on gfx950 while
    MFMA work ran on the GPU; the library is built with -packed-fp32-ops
    (magpie-tts.cpp_amd/Makefile, NOPK, appended in the rules). A rebuild that loses
    the flag must fail here, not corrupt a decode beside the codec."""
    import magpie_amd as ma
    cos = _gfx950_code_objects(ma.LIB_PATH, tmp_path)
    assert len(cos) >= 6, f"expected one gfx950 code object per HIP source, found {len(cos)}"
    n_mfma = 0
    for co in cos:
        dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--mcpu=gfx950", str(co)],
                             capture_output=True, text=True, check=True).stdout
        bad = re.findall(r"\bv_pk_(?:fma|mul|add)_f32\b", dis)
        assert not bad, f"{co.name}: {len(bad)} packed-FP32 instructions ({bad[0]})"
        # no mixed-precision FMA: an f32 multiply folded into its f16 / bf16 conversion
        # rounds once where the same value computed elsewhere rounds twice (batch ==
        # single, round 4); the library is built with -fma-mix-insts (Makefile)
        mix = re.findall(r"\bv_(?:fma|mad)_mix\w*", dis)
        assert not mix, f"{co.name}: {len(mix)} mixed-precision FMA instructions ({mix[0]})"
        # no kernel keeps registers in scratch memory (round 4: arrays of HIP's float4 /
        # uint4 structs assigned under a condition, and arrays passed to a __noinline__
        # function, went to scratch: a dependent memory round trip per element)
        spill = re.findall(r"\bscratch_(?:load|store)_\w+", dis)
        assert not spill, f"{co.name}: {len(spill)} scratch instructions ({spill[0]})"
        n_mfma += len(re.findall(r"\bv_mfma_", dis))
    assert n_mfma > 1000  # the disassembly is real: the MFMA kernels are in it


CALLER = r'''
// a caller written against the reference header (src/magpie.h:107,265-307,604-648)
#include "magpie.h"
static bool on_audio(const float *, int, void *) { return true; }
static void on_progress(int, int, int, void *) {}
int use(magpie_context *ctx, magpie_codec *codec) {
    ctx->temperature = 0.0f; ctx->top_k = 80; ctx->speaker_id = 1; ctx->n_threads = 8; ctx->codec = codec;
    ctx->model.hparams.max_dec_steps = 500;
    ctx->state.reset();
    size_t n = ctx->state.generated_codes.size() + ctx->state.encoder_output.size();
    n += (size_t)ctx->state.n_generated_frames + (size_t)ctx->state.enc_seq_len;
    magpie_tokenizer tok;
    struct gguf_context *g = magpie_gguf_open("x.gguf");
    bool ok = magpie_tokenizer_init(&tok, g) && tok.loaded;
    magpie_gguf_close(g);
    magpie_stream_params p{0.7f, 80, 0, 4, true, on_audio, on_progress, nullptr};  // the reference's 8 fields, in order
    p.temperature = 0.5f; p.top_k = 40; p.speaker_id = 2; p.frames_per_chunk = 8; p.sentence_chunking = false;
    p.on_audio = on_audio; p.on_progress = on_progress; p.user_data = nullptr;
    int s = magpie_synthesize_streaming(ctx, codec, "Hello, world!", p);
    std::vector<int32_t> ids = magpie_tokenize(&ctx->model.tokenizer, "Hello");
    std::vector<int32_t> codes = magpie_synthesize_codes_graph_reuse(ctx, ids.data(), (int)ids.size());
    magpie_sample_result r = magpie_local_transformer_sample_all(ctx, nullptr, 0.7f, 80, false);
    // src/magpie.h:332, 555-558, 753
    bool enc = magpie_encode_text(ctx, ids.data(), (int)ids.size()) && ctx->state.enc_seq_len > 0;
    magpie_model m;
    bool ld = magpie_model_load(std::string("model.gguf"), m) && magpie_model_load("model.gguf", m, MAGPIE_BACKEND_CPU);
    magpie_codec c;
    bool cl = magpie_codec_load(std::string("codec.gguf"), c, MAGPIE_BACKEND_AUTO);
    return (int)n + s + (ok ? 1 : 0) + (int)codes.size() + (int)r.argmax_codes.size() + enc + ld + cl;
}
'''


def test_reference_caller_compiles_and_links(tmp_path):
    """include/magpie.h keeps the reference's field names (magpie_context incl. state,
    magpie_stream_params' exact 8 fields, magpie_tokenizer_init): a reference-side
    caller compiles unchanged and links against libmagpie_hip.so."""
    import magpie_amd as ma
    src = tmp_path / "caller.cpp"
    src.write_text(CALLER + "int main() { return 0; }\n")
    exe = tmp_path / "caller"
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"),
                        "-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", str(src), "-o", str(exe),
                        ma.LIB_PATH, f"-Wl,-rpath,{os.path.dirname(ma.LIB_PATH)}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
