"""magpie_amd — Python binding of the MI355X-native Magpie decode path.

The product is the C-ABI shared library ``lib/libmagpie_hip.so`` (hand-written
gfx950 HIP kernels + runtime, boundary declared in ``include/magpie_hip.h``).
This module only binds it with ctypes: no torch types, no fallback. If the
library or a GPU is missing, every entry point raises — there is deliberately
no CPU path here (the CPU oracle under ``oracle/`` is test infrastructure).

Reference interface mirrored (m1el/magpie-tts.cpp, src/magpie.h):
  magpie_init / magpie_free              -> Device(model_path) / Device.close()
  magpie_synthesize_codes_graph_reuse    -> Device.synthesize(tokens, ...)   (magpie.h:592-595)
  magpie_codec_init / magpie_codec_decode -> Codec(path).decode(codes)       (magpie.h:746-759)
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.environ.get("MAGPIE_LIB") or os.path.join(PKG_DIR, "lib", "libmagpie_hip.so")  # MAGPIE_LIB: A/B builds
SYNTH_BIN = os.path.join(PKG_DIR, "bin", "mp_synth_gguf")

MP_OK = 0
_ERRS = {-1: "MP_ERR_ARG", -2: "MP_ERR_HIP", -3: "MP_ERR_IO", -4: "MP_ERR_FORMAT", -5: "MP_ERR_STATE",
         -6: "MP_ERR_UNSUPPORTED"}

# magpie.h:70-73 token constants
TEXT_BOS, TEXT_EOS, AUDIO_BOS, AUDIO_EOS = 2378, 2379, 2016, 2017
NUM_CODEBOOKS, VOCAB_PER_CB, CONTEXT_FRAMES = 8, 2024, 110
FRAMES_PER_SECOND = 22050.0 / 1024.0  # 21.533 codec frames per audio second


class MagpieError(RuntimeError):
    pass


class mp_params(ctypes.Structure):
    _fields_ = [("temperature", ctypes.c_float), ("top_k", ctypes.c_int), ("max_dec_steps", ctypes.c_int),
                ("ignore_eos", ctypes.c_int), ("seed", ctypes.c_uint64), ("trace_hidden", ctypes.c_int),
                ("stream_base", ctypes.c_int), ("emit_eos_frame", ctypes.c_int)]


class mp_timing(ctypes.Structure):
    _fields_ = [("preamble_ms", ctypes.c_double), ("decode_ms", ctypes.c_double), ("frames_total", ctypes.c_int),
                ("iterations", ctypes.c_int), ("first_audio_ms", ctypes.c_double)]


# int (*mp_audio_cb)(int utterance, const float *samples, int n_samples, void *user)
AUDIO_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.c_void_p)


# (name, restype, argtypes) of every symbol include/magpie_hip.h declares
_P = ctypes.c_void_p
_I = ctypes.c_int
SYMBOLS = [
    ("mp_hip_device_count", _I, [ctypes.POINTER(_I)]),
    ("mp_hip_runtime_path", ctypes.c_char_p, []),
    ("mp_hip_init", _I, [_I, ctypes.POINTER(_P)]),
    ("mp_hip_load_model", _I, [_P, ctypes.c_char_p]),
    ("mp_hip_load_model_ex", _I, [_P, ctypes.c_char_p, _I]),
    ("mp_hip_weight_mode", _I, [_P]),
    ("mp_hip_max_batch", _I, [_P]),
    ("mp_hip_set_kv_mode", _I, [_P, _I]),
    ("mp_hip_set_xa_mode", _I, [_P, _I]),
    ("mp_hip_model_info", _I, [_P, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(ctypes.c_size_t)]),
    ("mp_hip_free", None, [_P]),
    ("mp_hip_error", ctypes.c_char_p, [_P]),
    ("mp_hip_begin_batch", _I, [_P, _P, _P, _P, _I, _I, ctypes.POINTER(mp_params)]),
    ("mp_hip_decode", _I, [_P, _P, _P]),
    ("mp_hip_get_trace", _I, [_P, _P]),
    ("mp_hip_debug_buffer", ctypes.c_int64, [_P, ctypes.c_char_p, _P, ctypes.c_int64]),
    ("mp_hip_encode_text", _I, [_P, _P, _I, _P]),
    ("mp_hip_get_timing", _I, [_P, ctypes.POINTER(mp_timing)]),
    ("mp_hip_decode_stream", _I, [_P, _P, _I, AUDIO_CB, _P, _P, _P, ctypes.POINTER(ctypes.c_int64)]),
    ("mp_hip_lt_sample", _I, [_P, _P, ctypes.c_float, _I, _I, ctypes.c_uint64, _P, _P]),
    ("mp_hip_num_ops", _I, [_P]),
    ("mp_hip_op_name", ctypes.c_char_p, [_P, _I]),
    ("mp_hip_op_bytes", ctypes.c_double, [_P, _I]),
    ("mp_hip_time_op", _I, [_P, _I, _I, ctypes.POINTER(ctypes.c_float)]),
    ("mp_hip_profile_ops", _I, [_P, _I, _P]),
    ("mp_hip_profile_ops_ex", _I, [_P, _I, _P, _P]),
    ("mp_hip_profile_ops_ts", _I, [_P, _I, _P]),
    ("mp_hip_profile_ops_kev", _I, [_P, _I, _P]),
    ("mp_tokenizer_load", _I, [ctypes.c_char_p, ctypes.POINTER(_P)]),
    ("mp_tokenize", _I, [_P, ctypes.c_char_p, _P, _I]),
    ("mp_tokenizer_free", None, [_P]),
    ("mp_split_sentences", _I, [ctypes.c_char_p, _P, _P, _I]),
    ("mp_hip_codec_init", _I, [_I, ctypes.c_char_p, ctypes.POINTER(_P)]),
    ("mp_hip_codec_decode", _I, [_P, _P, _I, _P]),
    ("mp_hip_codec_decode_chunks", _I, [_P, _P, _I, _I, _P]),
    ("mp_hip_codec_last_ms", _I, [_P, ctypes.POINTER(ctypes.c_float)]),
    ("mp_hip_codec_free", None, [_P]),
    ("mp_hip_codec_error", ctypes.c_char_p, [_P]),
]

# entry points added after round 4: absent from the A/B baseline libraries
OPTIONAL = {"mp_hip_encode_text"}

_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libmagpie_hip.so (RTLD_GLOBAL so its HIP runtime is the process's)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise MagpieError(f"{path} is missing: build it with `make -C {PKG_DIR}` (or __graft_entry__.build())")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, res, args in SYMBOLS:
        if name in OPTIONAL and not hasattr(lib, name):
            continue  # an older library (A/B runs against a previous round's build)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def lib_sha16(path: str = LIB_PATH) -> str:
    """sha256[:16] of the library file: ties a committed profile to the build it measured."""
    import hashlib
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def device_count() -> int:
    n = ctypes.c_int(0)
    load_library().mp_hip_device_count(ctypes.byref(n))
    return n.value


def build(jobs: int = 8) -> None:
    subprocess.run(["make", "-C", PKG_DIR, f"-j{jobs}"], check=True)


# LT output-head scale of the parity/bench models: logits wide enough that >= 98 % of
# greedy decisions have a top-1/top-2 gap above 1e-2 (1.0 leaves 58 % below it)
DECISIVE = 32.0


def synth_gguf(path: str, kind: str = "magpie", seed: int = 0x4D414750, dtype: str = "f32",
               dec_layers: int = 12, enc_layers: int = 6, lt_head_scale: float = 1.0,
               audio_bos: Optional[int] = None, eos_bias: Optional[float] = None) -> str:
    """Write (or reuse) a deterministic synthetic GGUF with the reference's layout.
    lt_head_scale multiplies the std of the LT output heads (weights and bias);
    audio_bos moves the 8 special audio ids (EOS = audio_bos + 1), eos_bias raises
    codebook 3's EOS logit (test models)."""
    if os.path.exists(path):
        return path
    tmp = f"{path}.tmp{os.getpid()}"  # written aside, then renamed: never a partial file at `path`
    cmd = [SYNTH_BIN, kind, tmp, "--seed", str(seed)]
    if kind == "magpie":
        cmd += ["--dtype", dtype, "--dec-layers", str(dec_layers), "--enc-layers", str(enc_layers),
                "--lt-head-scale", repr(float(lt_head_scale))]
        if audio_bos is not None:
            cmd += ["--audio-bos", str(int(audio_bos))]
        if eos_bias is not None:
            cmd += ["--eos-bias", repr(float(eos_bias))]
    try:
        subprocess.run(cmd, check=True)
        os.replace(tmp, path)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)
    return path


def synthetic_tokens(T: int, seed: int) -> np.ndarray:
    """BOS + (T-2) ids ~ U[0,96) + EOS, seeded per utterance."""
    rng = np.random.default_rng(seed)
    body = rng.integers(0, 96, max(T - 2, 0))
    return np.concatenate([[TEXT_BOS], body, [TEXT_EOS]]).astype(np.int32)[:T]


@dataclass
class SynthResult:
    codes: List[np.ndarray]          # per utterance [n_frames][8]
    n_frames: np.ndarray
    preamble_ms: float
    decode_ms: float
    iterations: int
    hidden: Optional[np.ndarray] = None  # [B][max_steps+1][768] when traced


class Device:
    """One GPU with resident Magpie weights (magpie_init_with_backend, magpie.cpp:781)."""

    WEIGHT_MODES = {"f32": 0, "as_stored": 0, "bf16": 1, "q8": 2, "q4": 2, "f16": 3}

    KV_MODES = {"f32": 0, "bf16": 1}
    XA_MODES = {"auto": 0, "reassoc": 1, "direct": 2}

    def __init__(self, model_path: str, device: int = 0, weights: str = "f32", kv: str = "f32", xa: str = "auto"):
        """weights: "f32" (as stored, widened to f32), "bf16" (decode projections
        on bf16 MFMA, activations rounded to bf16; batches up to 16) or "q8" / "q4"
        (the file's Q8_0 / Q4_0 tensors kept as int8 (Q4_0: q - 8, losslessly),
        multiplied with ggml's semantics: activations quantised to Q8_0 per
        32-block, integer dots scaled by d_w * d_a; batches up to 16 when every
        decode projection is quantised, else 8, Device.max_batch()) or "f16" (an
        F16 file with ggml's F16 mul_mat semantics: activations rounded to f16,
        decode projections on f16 MFMA; batches up to 16).
        kv: SA cache element type, "f32" (the reference's) or "bf16" (rows rounded
        to bf16 on append, mp_hip_set_kv_mode).
        xa: cross-attention form (mp_hip_set_xa_mode): "auto" (direct above 160 text
        tokens), "reassoc" (K'/V' precomputed, fused in the O-projection launch) or
        "direct" (q_net, attention, o_net)."""
        if xa not in self.XA_MODES:
            raise ValueError(f"xa must be one of {sorted(self.XA_MODES)}")
        if kv not in self.KV_MODES:
            raise ValueError(f"kv must be one of {sorted(self.KV_MODES)}")
        if weights not in self.WEIGHT_MODES:
            raise ValueError(f"weights must be one of {sorted(self.WEIGHT_MODES)}")
        self.lib = load_library()
        h = ctypes.c_void_p()
        rc = self.lib.mp_hip_init(device, ctypes.byref(h))
        if rc != MP_OK or not h.value:
            raise MagpieError(f"mp_hip_init(device={device}) failed ({_ERRS.get(rc, rc)}): no usable HIP device")
        self.h = h
        self.weights = weights
        self._check(self.lib.mp_hip_load_model_ex(self.h, model_path.encode(), self.WEIGHT_MODES[weights]))
        self.kv = kv
        self._check(self.lib.mp_hip_set_kv_mode(self.h, self.KV_MODES[kv]))
        self.xa = xa
        self._check(self.lib.mp_hip_set_xa_mode(self.h, self.XA_MODES[xa]))

    def _check(self, rc: int) -> None:
        if rc != MP_OK:
            msg = self.lib.mp_hip_error(self.h).decode(errors="replace")
            raise MagpieError(f"{_ERRS.get(rc, rc)}: {msg}")

    def close(self) -> None:
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.mp_hip_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def model_info(self):
        dl, el, wb = ctypes.c_int(), ctypes.c_int(), ctypes.c_size_t()
        self._check(self.lib.mp_hip_model_info(self.h, ctypes.byref(dl), ctypes.byref(el), ctypes.byref(wb)))
        return {"dec_layers": dl.value, "enc_layers": el.value, "weight_bytes": wb.value}

    def max_batch(self) -> int:
        n = self.lib.mp_hip_max_batch(self.h)
        self._check(min(n, 0))
        return n

    def begin(self, tokens: Sequence[Sequence[int]], speakers: Optional[Sequence[int]] = None,
              max_dec_steps: int = 500, temperature: float = 0.0, top_k: int = 80, ignore_eos: bool = False,
              seed: int = 0, trace: bool = False, stream_base: int = 0, emit_eos_frame: bool = False) -> int:
        """mp_hip_begin_batch: preamble of B independent utterances; returns B."""
        B = len(tokens)
        tmax = max(len(t) for t in tokens)
        tok = np.zeros((B, tmax), np.int32)
        for b, t in enumerate(tokens):
            tok[b, :len(t)] = np.asarray(t, np.int32)
        nt = np.array([len(t) for t in tokens], np.int32)
        spk = np.zeros(B, np.int32) if speakers is None else np.asarray(speakers, np.int32)
        p = mp_params(temperature, top_k, max_dec_steps, int(ignore_eos), seed, int(trace), int(stream_base),
                      int(emit_eos_frame))
        self._check(self.lib.mp_hip_begin_batch(self.h, tok.ctypes.data, nt.ctypes.data, spk.ctypes.data, B, tmax,
                                                ctypes.byref(p)))
        return B

    def synthesize(self, tokens: Sequence[Sequence[int]], speakers: Optional[Sequence[int]] = None,
                   max_dec_steps: int = 500, temperature: float = 0.0, top_k: int = 80, ignore_eos: bool = False,
                   seed: int = 0, trace: bool = False, stream_base: int = 0) -> SynthResult:
        """Batched magpie_synthesize_codes_graph_reuse over independent utterances."""
        B = self.begin(tokens, speakers, max_dec_steps, temperature, top_k, ignore_eos, seed, trace, stream_base)
        return self.decode(B, max_dec_steps, trace)

    def synthesize_stream(self, codec: "Codec", tokens: Sequence[Sequence[int]], on_audio,
                          speakers: Optional[Sequence[int]] = None, max_dec_steps: int = 500,
                          temperature: float = 0.0, top_k: int = 80, seed: int = 0, frames_per_chunk: int = 4,
                          stream_base: int = 0, ignore_eos: bool = False):
        """magpie_synthesize_sentence_streaming over a batch: on_audio(utt, np.ndarray) -> bool
        (False stops that utterance). The EOS frame is emitted, as the reference's streaming
        loop does. Returns (codes per utterance, total samples, timing)."""
        B = self.begin(tokens, speakers, max_dec_steps, temperature, top_k, ignore_eos, seed, False, stream_base, True)
        return self.decode_stream_only(codec, on_audio, B, max_dec_steps, frames_per_chunk)

    def decode_stream_only(self, codec: "Codec", on_audio, B: int, max_dec_steps: int, frames_per_chunk: int = 4):
        """mp_hip_decode_stream on the batch the last begin() prepared (the preamble is not
        re-run): the decode on this device's stream, each chunk through the codec on the
        codec's stream as it completes. Returns (codes per utterance, total samples, timing)."""
        def _cb(utt, ptr, n, _user):
            if n == 0:  # end-of-utterance notice
                return 1
            return 1 if on_audio(utt, np.ctypeslib.as_array(ptr, shape=(n,)).copy()) is not False else 0

        cb = AUDIO_CB(_cb)
        codes = np.zeros((B, max_dec_steps, 8), np.int32)
        nf = np.zeros(B, np.int32)
        total = ctypes.c_int64()
        self._check(self.lib.mp_hip_decode_stream(self.h, codec.h, frames_per_chunk, cb, None, codes.ctypes.data,
                                                  nf.ctypes.data, ctypes.byref(total)))
        tm = mp_timing()
        self._check(self.lib.mp_hip_get_timing(self.h, ctypes.byref(tm)))
        return [codes[b, :nf[b]].copy() for b in range(B)], int(total.value), tm

    def lt_sample(self, hidden, temperature: float = 0.0, top_k: int = 80, forbid_eos: bool = False, seed: int = 0):
        """magpie_local_transformer_sample_all: (sampled[8], argmax[8]) for one hidden[768]."""
        h = np.ascontiguousarray(hidden, np.float32)
        assert h.shape == (768,)
        smp, amx = np.zeros(8, np.int32), np.zeros(8, np.int32)
        self._check(self.lib.mp_hip_lt_sample(self.h, h.ctypes.data, temperature, top_k, int(forbid_eos), seed,
                                              smp.ctypes.data, amx.ctypes.data))
        return smp, amx

    def decode(self, B: int, max_dec_steps: int, trace: bool = False) -> SynthResult:
        codes = np.zeros((B, max_dec_steps, 8), np.int32)
        nf = np.zeros(B, np.int32)
        self._check(self.lib.mp_hip_decode(self.h, codes.ctypes.data, nf.ctypes.data))
        tm = mp_timing()
        self._check(self.lib.mp_hip_get_timing(self.h, ctypes.byref(tm)))
        hidden = None
        if trace:
            hidden = np.zeros((B, max_dec_steps + 1, 768), np.float32)
            self._check(self.lib.mp_hip_get_trace(self.h, hidden.ctypes.data))
        return SynthResult([codes[b, :nf[b]].copy() for b in range(B)], nf, tm.preamble_ms, tm.decode_ms,
                           tm.iterations, hidden)

    def encode_text(self, tokens) -> np.ndarray:
        """mp_hip_encode_text (magpie_encode_text, magpie.cpp:2284-2374): the text encoder
        alone for one utterance, [T][768]; a batch in progress is not touched."""
        tok = np.ascontiguousarray(tokens, np.int32)
        out = np.zeros((len(tok), 768), np.float32)
        self._check(self.lib.mp_hip_encode_text(self.h, tok.ctypes.data, len(tok), out.ctypes.data))
        return out

    def debug_buffer(self, name: str) -> np.ndarray:
        """mp_hip_debug_buffer: a per-batch device buffer (flat f32) for diagnostics."""
        n = self.lib.mp_hip_debug_buffer(self.h, name.encode(), None, 0)
        if n < 0:
            self._check(int(n))
        out = np.zeros(n // 4, np.float32)
        self._check(0 if self.lib.mp_hip_debug_buffer(self.h, name.encode(), out.ctypes.data, n) == n else -5)
        return out

    def debug_bytes(self, name: str) -> bytes:
        """mp_hip_debug_buffer as raw bytes (e.g. "q8dump", "q8dump_index" with MAGPIE_Q8DUMP=1)."""
        n = self.lib.mp_hip_debug_buffer(self.h, name.encode(), None, 0)
        if n < 0:
            self._check(int(n))
        out = ctypes.create_string_buffer(max(int(n), 1))
        self._check(0 if self.lib.mp_hip_debug_buffer(self.h, name.encode(), out, n) == n else -5)
        return out.raw[:n]

    # ---- measurement
    def ops(self) -> List[str]:
        return [self.lib.mp_hip_op_name(self.h, i).decode() for i in range(self.lib.mp_hip_num_ops(self.h))]

    def op_bytes(self, op: int) -> float:
        return float(self.lib.mp_hip_op_bytes(self.h, op))

    def profile_ops(self, iters: int = 32) -> np.ndarray:
        """In-situ mean launch time (us) of every op of the decode iteration."""
        n = self.lib.mp_hip_num_ops(self.h)
        out = np.zeros(max(n, 1), np.float32)
        self._check(self.lib.mp_hip_profile_ops(self.h, iters, out.ctypes.data))
        return out[:n]

    def profile_ops_ex(self, iters: int = 32):
        """(event-pair time per op, empty-pair time right after it), us"""
        n = self.lib.mp_hip_num_ops(self.h)
        out = np.zeros(max(n, 1), np.float32)
        pair = np.zeros(max(n, 1), np.float32)
        self._check(self.lib.mp_hip_profile_ops_ex(self.h, iters, out.ctypes.data, pair.ctypes.data))
        return out[:n], pair[:n]

    def profile_ops_ts(self, iters: int = 32) -> np.ndarray:
        """per-op launch duration from in-kernel timestamps (us; -1: not instrumented)"""
        n = self.lib.mp_hip_num_ops(self.h)
        out = np.zeros(max(n, 1), np.float32)
        self._check(self.lib.mp_hip_profile_ops_ts(self.h, iters, out.ctypes.data))
        return out[:n]

    def profile_ops_kev(self, iters: int = 32) -> np.ndarray:
        """per-op launch duration from the dispatch's begin/end timestamps (us), the
        interval rocprofv3's kernel trace reports"""
        n = self.lib.mp_hip_num_ops(self.h)
        out = np.zeros(max(n, 1), np.float32)
        self._check(self.lib.mp_hip_profile_ops_kev(self.h, iters, out.ctypes.data))
        return out[:n]

    def time_op(self, op: int, reps: int = 50) -> float:
        us = ctypes.c_float()
        self._check(self.lib.mp_hip_time_op(self.h, op, reps, ctypes.byref(us)))
        return us.value


class Tokenizer:
    """Text front end of the reference (magpie_tokenizer_init / magpie_tokenize,
    magpie.cpp:124-495), host C++ in libmagpie_hip.so."""

    def __init__(self, gguf_path: str):
        self.lib = load_library()
        h = ctypes.c_void_p()
        rc = self.lib.mp_tokenizer_load(gguf_path.encode(), ctypes.byref(h))
        if rc != MP_OK or not h.value:
            raise MagpieError(f"{gguf_path}: no tokenizer ({_ERRS.get(rc, rc)})")
        self.h = h

    def __call__(self, text: str) -> List[int]:
        raw = text.encode("utf-8")
        n = self.lib.mp_tokenize(self.h, raw, None, 0)
        if n < 0:
            raise MagpieError(f"mp_tokenize failed ({n})")
        out = (ctypes.c_int32 * max(n, 1))()
        self.lib.mp_tokenize(self.h, raw, out, n)
        return list(out[:n])

    def close(self) -> None:
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.mp_tokenizer_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def split_sentences(text: str) -> List[str]:
    """magpie_split_sentences (magpie.cpp:4439-4480) via the C-ABI."""
    lib = load_library()
    raw = text.encode("utf-8")
    n = lib.mp_split_sentences(raw, None, None, 0)
    off, ln = (ctypes.c_int32 * max(n, 1))(), (ctypes.c_int32 * max(n, 1))()
    lib.mp_split_sentences(raw, off, ln, n)
    return [raw[off[i]:off[i] + ln[i]].decode("utf-8") for i in range(n)]


class Codec:
    """Nano-codec on the GPU (magpie_codec_init / magpie_codec_decode, nano-codec.cpp:339-845)."""

    def __init__(self, path: str, device: int = 0):
        self.lib = load_library()
        h = ctypes.c_void_p()
        rc = self.lib.mp_hip_codec_init(device, path.encode(), ctypes.byref(h))
        if rc != MP_OK or not h.value:
            raise MagpieError(f"mp_hip_codec_init failed ({_ERRS.get(rc, rc)})")
        self.h = h

    def decode(self, codes_cb_major: np.ndarray) -> np.ndarray:
        codes = np.ascontiguousarray(codes_cb_major, np.int32)
        assert codes.ndim == 2 and codes.shape[0] == 8
        F = codes.shape[1]
        out = np.zeros(F * 1024, np.float32)
        rc = self.lib.mp_hip_codec_decode(self.h, codes.ctypes.data, F, out.ctypes.data)
        if rc != MP_OK:
            raise MagpieError(f"{_ERRS.get(rc, rc)}: {self.lib.mp_hip_codec_error(self.h).decode(errors='replace')}")
        return out

    def decode_chunks(self, codes: np.ndarray) -> np.ndarray:
        """codes [n_chunks][8][F] -> audio [n_chunks][F*1024], chunks independent."""
        codes = np.ascontiguousarray(codes, np.int32)
        n, eight, F = codes.shape
        assert eight == 8
        out = np.zeros((n, F * 1024), np.float32)
        rc = self.lib.mp_hip_codec_decode_chunks(self.h, codes.ctypes.data, n, F, out.ctypes.data)
        if rc != MP_OK:
            raise MagpieError(f"{_ERRS.get(rc, rc)}: {self.lib.mp_hip_codec_error(self.h).decode(errors='replace')}")
        return out

    def last_ms(self) -> float:
        ms = ctypes.c_float()
        self.lib.mp_hip_codec_last_ms(self.h, ctypes.byref(ms))
        return ms.value

    def close(self) -> None:
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.mp_hip_codec_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
