"""Streaming synthesis and magpie_local_transformer_sample_all on the device.

Reference behaviour: magpie_synthesize_sentence_streaming (magpie.cpp:4479-4863):
frames are decoded by the codec in stateless chunks of frames_per_chunk (default
4) as they are produced, the EOS frame is emitted too (4800-4806), the last chunk
may be shorter, and the audio callback can stop generation (4820-4824).
magpie_local_transformer_sample_all (1113-1317): sampled + argmax codes of one
normalised hidden vector.
"""
import numpy as np
import pytest

from parity import compare_codes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ma():
    import magpie_amd
    if magpie_amd.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return magpie_amd


@pytest.fixture(scope="module")
def codec(ma, codec_model):
    c = ma.Codec(codec_model)
    yield c
    c.close()


def _collect(B):
    chunks = {b: [] for b in range(B)}

    def on_audio(utt, samples):
        chunks[utt].append(samples)
        return True
    return chunks, on_audio


def test_stream_emits_eos_frame_in_chunks(ma, oracle, eos_model, codec):
    toks = [ma.synthetic_tokens(16, seed=7), ma.synthetic_tokens(9, seed=8)]
    dev = ma.Device(eos_model)
    chunks, cb = _collect(2)
    codes, total, tm = dev.synthesize_stream(codec, toks, cb, max_dec_steps=64, frames_per_chunk=4)
    dev.close()
    om = oracle.Model(eos_model)
    for b in range(2):
        o = om.synthesize(toks[b], max_steps=64, trace=False, emit_eos=True)
        # EOS at step 4 (forbidden before), and the EOS frame itself is part of the stream
        assert o["n_frames"] == 5 and len(codes[b]) == 5 and codes[b][4].tolist().count(2017) >= 1
        compare_codes(codes[b], o["codes"], o["margins"])
        assert [len(c) for c in chunks[b]] == [4 * 1024, 1 * 1024]
        # each chunk is the codec's stateless decode of those frames (decode_frames_to_audio)
        ref = [codec.decode(codes[b][0:4].T), codec.decode(codes[b][4:5].T)]
        for got, want in zip(chunks[b], ref):
            assert np.array_equal(got, want)
    om.close()
    assert total == 2 * 5 * 1024
    assert tm.first_audio_ms > 0


def test_stream_max_steps_partial_last_chunk_and_stop(ma, small_model, codec):
    toks = [ma.synthetic_tokens(12, seed=3)]
    dev = ma.Device(small_model)
    chunks, cb = _collect(1)
    codes, total, _ = dev.synthesize_stream(codec, toks, cb, max_dec_steps=10, frames_per_chunk=4)
    assert [len(c) for c in chunks[0]] == [4096, 4096, 2048] and total == 10 * 1024
    ref = dev.synthesize(toks, max_dec_steps=10)
    assert np.array_equal(codes[0], ref.codes[0])
    # the callback stops generation after the first chunk
    seen = []

    def stop_after_first(utt, audio):
        seen.append(len(audio))
        return False

    codes2, total2, _ = dev.synthesize_stream(codec, toks, stop_after_first, max_dec_steps=10, frames_per_chunk=4)
    dev.close()
    assert seen == [4096] and total2 == 4096 and len(codes2[0]) == 4


def test_batched_longform_equals_sequential(ma, small_model, codec):
    """Sentences of one text batched on the device reproduce the sentence-by-sentence
    stream exactly (sampling included: utterance b draws from stream b)."""
    sents = [ma.synthetic_tokens(6 + 4 * i, seed=300 + i) for i in range(3)]
    kw = dict(max_dec_steps=12, frames_per_chunk=4, temperature=0.7, top_k=80, seed=42)
    dev = ma.Device(small_model)
    chunks_b, cb = _collect(3)
    codes_b, _, _ = dev.synthesize_stream(codec, sents, cb, speakers=[2, 2, 2], **kw)
    for i, t in enumerate(sents):
        chunks_s, cbs = _collect(1)
        codes_s, _, _ = dev.synthesize_stream(codec, [t], cbs, speakers=[2], stream_base=i, **kw)
        assert np.array_equal(codes_s[0], codes_b[i])
        assert all(np.array_equal(x, y) for x, y in zip(chunks_s[0], chunks_b[i]))
    dev.close()


def test_batched_stream_stop_one_utterance(ma, small_model, codec):
    """A callback stopping one utterance of a batch ends that utterance only (its
    chunks already decoded this round are dropped); the others stream on unchanged."""
    sents = [ma.synthetic_tokens(8 + 3 * i, seed=500 + i) for i in range(3)]
    kw = dict(max_dec_steps=16, frames_per_chunk=4, ignore_eos=True)
    dev = ma.Device(small_model)
    got = {0: [], 1: [], 2: []}

    def cb(utt, audio):
        got[utt].append(audio)
        return utt != 1

    codes_b, total, _ = dev.synthesize_stream(codec, sents, cb, speakers=[0, 1, 2], **kw)
    assert len(got[1]) == 1 and len(codes_b[1]) == 4
    assert total == (16 + 4 + 16) * 1024
    for i in (0, 2):
        chunks_s, cbs = _collect(1)
        codes_s, _, _ = dev.synthesize_stream(codec, [sents[i]], cbs, speakers=[i], stream_base=i, **kw)
        assert np.array_equal(codes_s[0], codes_b[i])
        assert len(chunks_s[0]) == len(got[i]) == 4
        assert all(np.array_equal(x, y) for x, y in zip(chunks_s[0], got[i]))
    dev.close()


def test_lt_sample_matches_oracle(ma, oracle, small_model):
    rng = np.random.default_rng(5)
    dev = ma.Device(small_model)
    om = oracle.Model(small_model)
    for call in range(6):
        h = rng.normal(0, 1, 768).astype(np.float32)
        forbid = call % 2 == 1
        temp = 0.0 if call < 3 else 0.8
        smp, amx = dev.lt_sample(h, temperature=temp, top_k=50, forbid_eos=forbid, seed=11)
        o_smp, o_amx, o_mg = om.lt_sample(h, temperature=temp, top_k=50, forbid_eos=forbid, seed=11, stream=-1,
                                          step=4 + call)
        compare_codes(smp[None], o_smp[None], o_mg[None])
        if np.array_equal(smp, o_smp):
            assert np.array_equal(amx, o_amx)
        if temp == 0.0:
            assert np.array_equal(smp, amx)
    dev.close()
    om.close()


def test_lt_sample_q8_matches_oracle(ma, oracle, q8_model):
    """magpie_local_transformer_sample_all with the Q8_0 LT projections (weight mode q8)."""
    rng = np.random.default_rng(6)
    dev = ma.Device(q8_model, weights="q8")
    om = oracle.Model(q8_model)
    om.set_weight_mode(2)
    for call in range(4):
        h = rng.normal(0, 1, 768).astype(np.float32)
        temp = 0.0 if call < 2 else 0.8
        smp, amx = dev.lt_sample(h, temperature=temp, top_k=50, seed=12)
        o_smp, o_amx, o_mg = om.lt_sample(h, temperature=temp, top_k=50, seed=12, stream=-1, step=4 + call)
        compare_codes(smp[None], o_smp[None], o_mg[None], tie_eps=1e-2)
    dev.close()
    om.close()


def test_configs2_overlapped_codec_equals_serial(ma, small_model, codec):
    """configs[2]'s end-to-end form (bench.py measure_configs2_e2e): bf16, 16 slots, each
    slot's 32-frame chunks decoded by the codec on its stream while the decode continues
    (mp_hip_decode_stream, frames_per_chunk = 32). The waveform equals the serial form
    bit for bit: the decode alone, then the codec over the same chunks."""
    B, F, C = 16, 64, 32
    toks = [ma.synthetic_tokens(12 + (b % 5), seed=1900 + b) for b in range(B)]
    spk = [b % 5 for b in range(B)]
    dev = ma.Device(small_model, weights="bf16")
    ser = dev.synthesize(toks, speakers=spk, max_dec_steps=F, ignore_eos=True)
    chunks, cb = _collect(B)
    codes, total, tm = dev.synthesize_stream(codec, toks, cb, speakers=spk, max_dec_steps=F, frames_per_chunk=C,
                                             ignore_eos=True)
    dev.close()
    assert total == B * F * 1024
    serial = codec.decode_chunks(np.stack([ser.codes[b][s0:s0 + C].T for b in range(B) for s0 in range(0, F, C)]))
    for b in range(B):
        assert np.array_equal(codes[b], ser.codes[b]), b
        assert [len(c) for c in chunks[b]] == [C * 1024] * (F // C)
        for k, got in enumerate(chunks[b]):
            assert np.array_equal(got, serial[b * (F // C) + k]), (b, k)
