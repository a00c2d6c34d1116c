"""ctypes binding of the CPU oracle (liboracle.so).

*** TEST INFRASTRUCTURE. *** Importable only from tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg — as the checker or the timed CPU baseline, never
as the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import time

import numpy as np

ORACLE_DIR = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(ORACLE_DIR, "liboracle.so")
_lib = None


def build() -> None:
    subprocess.run(["make", "-C", ORACLE_DIR], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P, I = ctypes.c_void_p, ctypes.c_int
        L.orc_set_mode.argtypes = [I, I, I]
        L.orc_load.restype = P
        L.orc_load.argtypes = [ctypes.c_char_p]
        L.orc_free.argtypes = [P]
        L.orc_dec_layers.argtypes = [P]
        L.orc_synthesize.argtypes = [P, P, I, I, I, I, P, P, P, P]
        L.orc_synthesize_ex.argtypes = [P, P, I, I, I, I, ctypes.c_float, I, ctypes.c_uint64, I, I, P, P, P, P]
        L.orc_encode.argtypes = [P, P, I, P]
        L.orc_synthesize_forced.argtypes = [P, P, I, I, I, I, ctypes.c_float, I, ctypes.c_uint64, I, P, P, P, P]
        L.orc_set_weight_mode.argtypes = [P, I]
        L.orc_set_kv_bf16.argtypes = [I]
        L.orc_lt_sample.argtypes = [P, P, ctypes.c_float, I, I, ctypes.c_uint64, I, I, P, P, P]
        L.orc_draw_u.restype = ctypes.c_float
        L.orc_draw_u.argtypes = [ctypes.c_uint64, I, I, I]
        L.orc_sample_top_k.argtypes = [P, I, ctypes.c_float, I, ctypes.c_float, P]
        L.orc_codec_load.restype = P
        L.orc_codec_load.argtypes = [ctypes.c_char_p]
        L.orc_codec_free.argtypes = [P]
        L.orc_codec_decode.argtypes = [P, P, I, P, I]
        L.orc_codec_set_resinit.argtypes = [P, I]
        L.orc_fsq.argtypes = [P, I, P]
        L.orc_q8_matvec.argtypes = [P, I, I, P, P]
        L.orc_q8_quantize_row.argtypes = [P, I, P, P]
        L.orc_qblock_dots.argtypes = [P, I, I, I, P, P]
        _lib = L
    return _lib


def set_mode(acc64: bool = True, gelu_f16: bool = False, threads: int = 0) -> None:
    lib().orc_set_mode(int(acc64), int(gelu_f16), int(threads))


def set_kv_bf16(on: bool) -> None:
    """SA cache rows rounded to bf16 on append (the GPU's MP_KV_BF16 mode)."""
    lib().orc_set_kv_bf16(int(on))


def draw_u(seed: int, stream: int, step: int, cb: int) -> float:
    return float(lib().orc_draw_u(int(seed) & (2**64 - 1), stream, step, cb))


def sample_top_k(logits, temperature: float, top_k: int, u: float):
    """(index, margin) of sample_top_k (magpie.cpp:1072-1109) for one logits row."""
    lg = np.ascontiguousarray(logits, np.float32)
    mg = ctypes.c_float()
    i = lib().orc_sample_top_k(lg.ctypes.data, len(lg), float(temperature), int(top_k), float(u), ctypes.byref(mg))
    return i, mg.value


class Model:
    def __init__(self, path: str):
        self.h = lib().orc_load(path.encode())
        if not self.h:
            raise RuntimeError(f"oracle: cannot load {path}")

    def set_weight_mode(self, mode: int) -> None:
        """0 = f32 (dequantised), 1 = bf16 decode projections, 2 = ggml Q8_0 mul_mat
        for the file's Q8_0 / Q4_0 tensors, 3 = ggml F16 mul_mat for the file's F16
        tensors (see magpie_oracle.h)."""
        if lib().orc_set_weight_mode(self.h, int(mode)) != 0:
            raise RuntimeError("oracle: bad weight mode")

    def close(self):
        if self.h:
            lib().orc_free(self.h)
            self.h = None

    def synthesize(self, tokens, speaker=0, max_steps=32, ignore_eos=False, trace=True,
                   temperature=0.0, top_k=80, seed=0, stream=0, emit_eos=False):
        """magpie_synthesize_codes_graph_reuse restated (magpie.cpp:4063-4432).
        temperature >= 0.01 samples with sample_top_k's arithmetic (1072-1109) from
        the counter-based stream u(seed, stream, step, cb); stream = batch slot."""
        tok = np.ascontiguousarray(tokens, np.int32)
        codes = np.zeros((max_steps, 8), np.int32)
        marg = np.zeros((max_steps, 8), np.float32)
        hid = np.zeros((max_steps + 1, 768), np.float32) if trace else None
        tim = np.zeros(2, np.float64)
        n = lib().orc_synthesize_ex(self.h, tok.ctypes.data, len(tok), speaker, max_steps, int(ignore_eos),
                                    float(temperature), int(top_k), int(seed) & (2**64 - 1), int(stream),
                                    int(emit_eos), codes.ctypes.data, marg.ctypes.data,
                                    hid.ctypes.data if trace else None, tim.ctypes.data)
        if n < 0:
            raise RuntimeError(f"oracle synthesize failed ({n})")
        return {"n_frames": n, "codes": codes[:n], "margins": marg[:max(n + 1, 0)],
                "hidden": hid, "preamble_ms": tim[0], "decode_ms": tim[1]}

    def synthesize_forced(self, tokens, forced, speaker=0, ignore_eos=True, temperature=0.0, top_k=80, seed=0,
                          stream=0):
        """Teacher-forced oracle run along `forced` ([n][8], the codes under test):
        the oracle's own decision and margin at every codebook of every frame, and the
        hidden state along the forced trajectory ([n+1][768], BOS first)."""
        tok = np.ascontiguousarray(tokens, np.int32)
        fc = np.ascontiguousarray(forced, np.int32).reshape(-1, 8)
        n = len(fc)
        codes = np.zeros((n, 8), np.int32)
        marg = np.zeros((n, 8), np.float32)
        hid = np.zeros((n + 1, 768), np.float32)
        r = lib().orc_synthesize_forced(self.h, tok.ctypes.data, len(tok), speaker, n, int(ignore_eos),
                                        float(temperature), int(top_k), int(seed) & (2**64 - 1), int(stream),
                                        fc.ctypes.data, codes.ctypes.data, marg.ctypes.data, hid.ctypes.data)
        if r != n:
            raise RuntimeError(f"oracle forced synthesize failed ({r})")
        return {"codes": codes, "margins": marg, "hidden": hid}

    def lt_sample(self, hidden, temperature=0.0, top_k=80, forbid_eos=False, seed=0, stream=-1, step=4):
        """magpie_local_transformer_sample_all restated: (sampled[8], argmax[8], margins[8])."""
        h = np.ascontiguousarray(hidden, np.float32)
        smp, amx, mg = np.zeros(8, np.int32), np.zeros(8, np.int32), np.zeros(8, np.float32)
        if lib().orc_lt_sample(self.h, h.ctypes.data, float(temperature), int(top_k), int(forbid_eos),
                               int(seed) & (2**64 - 1), int(stream), int(step), smp.ctypes.data, amx.ctypes.data,
                               mg.ctypes.data) != 0:
            raise RuntimeError("oracle lt_sample failed")
        return smp, amx, mg

    def encode(self, tokens):
        tok = np.ascontiguousarray(tokens, np.int32)
        out = np.zeros((len(tok), 768), np.float32)
        if lib().orc_encode(self.h, tok.ctypes.data, len(tok), out.ctypes.data) != 0:
            raise RuntimeError("oracle encode failed")
        return out


class Codec:
    def __init__(self, path: str):
        self.h = lib().orc_codec_load(path.encode())
        if not self.h:
            raise RuntimeError(f"oracle: cannot load codec {path}")

    def decode(self, codes_cb_major, f16_operands=True, resinit=False):
        """resinit: residual convs rounded as (x + sum) + b (this build's kernels) instead of
        the reference's (sum + b) + x."""
        lib().orc_codec_set_resinit(self.h, int(resinit))
        c = np.ascontiguousarray(codes_cb_major, np.int32)
        F = c.shape[1]
        out = np.zeros(F * 1024, np.float32)
        if lib().orc_codec_decode(self.h, c.ctypes.data, F, out.ctypes.data, int(f16_operands)) < 0:
            raise RuntimeError("oracle codec decode failed")
        return out

    def close(self):
        if self.h:
            lib().orc_codec_free(self.h)
            self.h = None


def q8_matvec(blocks: bytes, N: int, K: int, x) -> np.ndarray:
    """ggml Q8_0 mul_mat (activation quantised to Q8_0) of raw GGUF blocks with x[K]."""
    buf = np.frombuffer(blocks, np.uint8)
    assert buf.size == N * K // 32 * 34
    xv = np.ascontiguousarray(x, np.float32)
    y = np.zeros(N, np.float32)
    if lib().orc_q8_matvec(buf.ctypes.data, N, K, xv.ctypes.data, y.ctypes.data) != 0:
        raise RuntimeError("oracle q8_matvec failed")
    return y


def q8_quantize_row(x):
    """ggml quantize_row_q8_0 of x[K] (the oracle's restatement): (int8 q[K], f32 d[K/32])."""
    xv = np.ascontiguousarray(x, np.float32)
    K = xv.size
    q = np.zeros(K, np.int8)
    d = np.zeros(K // 32, np.float32)
    if lib().orc_q8_quantize_row(xv.ctypes.data, K, q.ctypes.data, d.ctypes.data) != 0:
        raise RuntimeError("oracle q8_quantize_row failed")
    return q, d


def qblock_dots(blocks: bytes, gguf_type: int, N: int, K: int, aq) -> np.ndarray:
    """Exact integer block dots [N][K/32] of raw GGUF Q8_0 (8) / Q4_0 (2) blocks with aq[K]."""
    buf = np.frombuffer(blocks, np.uint8)
    a = np.ascontiguousarray(aq, np.int8)
    out = np.zeros((N, K // 32), np.int32)
    if lib().orc_qblock_dots(buf.ctypes.data, gguf_type, N, K, a.ctypes.data, out.ctypes.data) != 0:
        raise RuntimeError("oracle qblock_dots failed")
    return out


def fsq(codes_cb_major):
    c = np.ascontiguousarray(codes_cb_major, np.int32)
    F = c.shape[1]
    out = np.zeros((32, F), np.float32)
    lib().orc_fsq(c.ctypes.data, F, out.ctypes.data)
    return out


def time_decode_fps(model_path: str, tokens, n_frames: int, threads: int, acc64: bool = False):
    """CPU baseline: frames/s of the oracle's decode loop (BOS + AR steps), f32 accumulation."""
    set_mode(acc64=acc64, gelu_f16=False, threads=threads)
    m = Model(model_path)
    t0 = time.time()
    r = m.synthesize(tokens, max_steps=n_frames, ignore_eos=True, trace=False)
    wall = time.time() - t0
    m.close()
    set_mode(acc64=True, gelu_f16=False, threads=threads)
    return {"frames": r["n_frames"], "decode_s": r["decode_ms"] / 1e3, "preamble_s": r["preamble_ms"] / 1e3,
            "wall_s": wall}
