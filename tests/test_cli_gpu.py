"""magpie-tts CLI and the C++ drop-in API end to end on the device.

Reference behaviour: src/magpie-tts.cpp:138-226 (tokenize -> graph-reuse decode
-> 32-frame stateless codec chunks -> 16-bit WAV at 22050 Hz, clamp + truncation),
and magpie_synthesize_streaming (magpie.cpp:4843-4863) for --stream: sentences
split at . ! ?, each streamed in 4-frame chunks with its EOS frame.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TEXT = "Hello, world! The first voice, 21st of May."


@pytest.fixture(scope="module")
def ma():
    import magpie_amd
    if magpie_amd.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return magpie_amd


def _read_wav(path):
    raw = open(path, "rb").read()
    assert raw[:4] == b"RIFF" and raw[8:16] == b"WAVEfmt "
    fmt, ch, rate, brate, align, bits = struct.unpack("<HHIIHH", raw[20:36])
    assert (fmt, ch, rate, brate, align, bits) == (1, 1, 22050, 44100, 2, 16)
    assert raw[36:40] == b"data"
    (n,) = struct.unpack("<I", raw[40:44])
    assert struct.unpack("<I", raw[4:8])[0] == 36 + n and len(raw) == 44 + n
    return np.frombuffer(raw[44:], np.int16)


def _pcm(audio):
    return (np.clip(audio, -1.0, 1.0) * np.float32(32767.0)).astype(np.int16)  # truncation toward zero


def _cli(ma, *args):
    exe = os.path.join(os.path.dirname(ma.LIB_PATH), "..", "bin", "magpie-tts")
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return r


def test_cli_greedy_matches_library(ma, small_model, codec_model, tmp_path):
    out = str(tmp_path / "a.wav")
    _cli(ma, "-m", small_model, "-c", codec_model, "-t", TEXT, "-o", out, "--temp", "0", "-q")
    wav = _read_wav(out)
    tok = ma.Tokenizer(small_model)(TEXT)
    dev = ma.Device(small_model)
    codes = dev.synthesize([tok], max_dec_steps=500).codes[0]
    dev.close()
    cdc = ma.Codec(codec_model)
    audio = np.concatenate([cdc.decode(codes[c:c + 32].T) for c in range(0, len(codes), 32)])
    cdc.close()
    assert len(wav) == len(codes) * 1024
    assert np.array_equal(wav, _pcm(audio))


def test_cli_stream_matches_sentence_streams(ma, small_model, codec_model, tmp_path):
    out = str(tmp_path / "s.wav")
    _cli(ma, "-m", small_model, "-c", codec_model, "-t", TEXT, "-o", out, "--stream", "--temp", "0.7", "-q")
    wav = _read_wav(out)
    sents = ma.split_sentences(TEXT)
    assert sents == ["Hello, world!", "The first voice, 21st of May."]
    tk = ma.Tokenizer(small_model)
    dev = ma.Device(small_model)
    cdc = ma.Codec(codec_model)
    parts = []
    for i, s in enumerate(sents):
        chunks = []
        dev.synthesize_stream(cdc, [tk(s)], lambda u, a: chunks.append(a), speakers=[0], max_dec_steps=500,
                              temperature=0.7, top_k=80, seed=0, frames_per_chunk=4, stream_base=i)
        parts.extend(chunks)
    dev.close()
    cdc.close()
    assert np.array_equal(wav, _pcm(np.concatenate(parts)))


def test_model_load_encode_text_codec_load(ma, oracle, small_model, codec_model, tmp_path):
    """magpie_model_load, magpie_encode_text and magpie_codec_load (src/magpie.h:332,
    555-558, 753) through bin/magpie-api-probe: the model loads, the encoder output that
    magpie_encode_text leaves in ctx->state equals the oracle's encoder within 1e-4, and
    the codec loads and decodes."""
    import json
    exe = os.path.join(os.path.dirname(ma.LIB_PATH), "..", "bin", "magpie-api-probe")
    out = tmp_path / "enc.bin"
    r = subprocess.run([exe, small_model, codec_model, str(out), "Hello, world!"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    info = json.loads(r.stdout.strip().splitlines()[-1])
    assert info["model_load"] and info["encode_text"] and info["codec_load"], info
    assert info["dec_layers"] == 2 and info["enc_seq_len"] == info["n_tokens"] > 2, info
    assert info["codec_samples"] == 4 * 1024
    assert info["cpu_backend_refused"], info
    enc = np.fromfile(out, np.float32).reshape(info["n_tokens"], 768)
    om = oracle.Model(small_model)
    ref = om.encode(np.asarray(info["tokens"], np.int32))
    om.close()
    err = float(np.abs(enc - ref).max())
    print(f"encoder output (T = {info['n_tokens']}): max abs err {err:.3g}")
    assert err < 1e-4, err
