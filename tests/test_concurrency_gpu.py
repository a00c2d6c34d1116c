"""The decode beside concurrent MFMA work on the same GPU.

Round 1 saw decoded hidden states change while the codec's MFMA convolutions ran
on another stream (or in another process). Root cause, found with
tools_dev/garbage/victim3.hip (the decode's own kernels on constant inputs, each
launch compared bitwise with the first, beside `garbage mfma`): on gfx950 the
packed-FP32 instructions (v_pk_fma_f32 / v_pk_mul_f32 with op_sel broadcasts) the
compiler emits for float4 arithmetic returned wrong values while MFMA work ran on
the GPU; the same kernels built with `-packed-fp32-ops` are bit-exact beside it.
The library is built that way (magpie-tts.cpp_amd/Makefile). This test pins it: a
decode running while a second thread keeps the codec busy on its own stream must be
bit-identical (codes and every hidden state) to the same decode run alone.
"""
import threading

import numpy as np
import pytest

import magpie_amd as ma

pytestmark = pytest.mark.gpu


def _run_beside_codec(model, codec_model, tokens, reps, **kw):
    dev = ma.Device(model)
    ref = dev.synthesize(tokens, **kw)
    cdc = ma.Codec(codec_model)
    stop = threading.Event()
    calls = [0]

    def codec_loop():
        codes = np.random.default_rng(0).integers(0, 2016, (8, 8, 32)).astype(np.int32)
        while not stop.is_set():
            cdc.decode_chunks(codes)  # 8 x 32-frame chunks: ~3 ms of MFMA convolutions per call
            calls[0] += 1

    th = threading.Thread(target=codec_loop)
    th.start()
    try:
        runs = [dev.synthesize(tokens, **kw) for _ in range(reps)]
    finally:
        stop.set()
        th.join()
    cdc.close()
    dev.close()
    assert calls[0] >= reps, f"the codec ran only {calls[0]} times beside {reps} decodes"
    for rep, r in enumerate(runs):
        for b in range(len(tokens)):
            d = np.abs(r.hidden[b] - ref.hidden[b]).max(axis=-1)
            bad = np.nonzero(d)[0]
            assert len(bad) == 0, (f"rep {rep} utt {b}: hidden differs from the run alone at frames {bad[:5]} "
                                   f"(max {d.max():.3g}) with the codec running beside it")
            assert np.array_equal(r.codes[b], ref.codes[b]), f"rep {rep} utt {b}: codes differ"
    print(f"{reps} decodes x {len(tokens)} utterances bit-identical beside {calls[0]} codec calls")


def test_small_model_beside_codec_bit_identical(small_model, codec_model):
    toks = [ma.synthetic_tokens(16 + 9 * b, seed=50 + b) for b in range(2)]
    _run_beside_codec(small_model, codec_model, toks, reps=6, speakers=[0, 0], max_dec_steps=96,
                      ignore_eos=True, trace=True)


def test_batch1_full_model_beside_codec_bit_identical(full_model, codec_model):
    toks = [ma.synthetic_tokens(64, seed=1000)]
    _run_beside_codec(full_model, codec_model, toks, reps=4, speakers=[0], max_dec_steps=128, ignore_eos=True,
                      trace=True)
