"""BASELINE.json configs[2]-[4] at full size (Magpie-357M shapes, 12 decoder
layers), the batched shapes the bench reports:

- configs[2]: bf16, batch 16 on one GPU;
- configs[3]: bf16, 8 utterances per GPU (the per-GPU share of batch 64);
- configs[4]: Q8_0 weights, 60 s long-form streaming (6 sentences x 216 frames as
  one device batch, 4-frame codec chunks).

The reference is batch 1 only: a batch's parity criterion is that
every utterance equals the same utterance run alone, bit for bit; one slot is
also checked decision by decision against the oracle (teacher forced).
"""
import numpy as np
import pytest

from parity import compare_forced

pytestmark = pytest.mark.gpu

TIE_EPS = 3e-2          # bf16 near-tie bar (test_decode_gpu.py: the oracle's own f32/f64 spread)
Q8_TIE_EPS = 1e-1       # Q8_0 near-tie bar (test_decode_gpu.py: the oracle's own f32/f64 spread)
HIDDEN_TOL, HIDDEN_REL = 3e-2, 5e-3


@pytest.fixture(scope="module")
def ma():
    import magpie_amd
    if magpie_amd.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return magpie_amd


def _hidden_ok(h_gpu, h_orc):
    err = np.abs(h_gpu - h_orc).max()
    nrm = np.linalg.norm(h_orc, axis=-1)
    rel = (np.linalg.norm(h_gpu - h_orc, axis=-1)[nrm > 0] / nrm[nrm > 0]).max()
    print(f"hidden vs oracle: max abs err {err:.3g}, max relative L2 {rel:.3g} over {len(h_gpu)} steps")
    assert err < HIDDEN_TOL and rel < HIDDEN_REL, (err, rel)


@pytest.mark.parametrize("B", [8, 16])
def test_bf16_full_model_batch_equals_single(ma, oracle, full_model, B):
    steps = 32
    toks = [ma.synthetic_tokens(40 + 3 * b, seed=7000 + b) for b in range(B)]
    spk = [b % 5 for b in range(B)]
    dev = ma.Device(full_model, weights="bf16")
    rb = dev.synthesize(toks, speakers=spk, max_dec_steps=steps, ignore_eos=True, trace=True)
    assert (rb.n_frames == steps).all()
    for b in (0, B // 2, B - 1):
        rs = dev.synthesize([toks[b]], speakers=[spk[b]], max_dec_steps=steps, ignore_eos=True, trace=True)
        assert np.array_equal(rb.codes[b], rs.codes[0]), f"slot {b} codes"
        assert np.array_equal(rb.hidden[b], rs.hidden[0]), f"slot {b} hidden"
    dev.close()
    om = oracle.Model(full_model)
    om.set_weight_mode(1)
    o = om.synthesize_forced(toks[0], rb.codes[0], speaker=spk[0], ignore_eos=True)
    om.close()
    res = compare_forced(rb.codes[0], o, tie_eps=TIE_EPS, max_ties=6)
    assert res["decisions"] == steps * 8
    _hidden_ok(rb.hidden[0, :steps + 1], o["hidden"])


@pytest.mark.parametrize("B,env", [(8, "MAGPIE_MERGE8=0"), (8, "MAGPIE_MERGE8=1"), (8, "MAGPIE_MERGE8=2"),
                                   (16, "MAGPIE_SA16=0")])
def test_bf16_batched_forms_equal(ma, full_model, B, env):
    """The batched bf16 layer's alternative forms compute the default's bits: at 8 slots which
    split states the split workgroups merge themselves (MAGPIE_MERGE8, default 3 = SA and XA),
    at 16 slots the SA in the QKV launch (the default) or as its own launch (MAGPIE_SA16=0)."""
    import os
    steps = 16
    toks = [ma.synthetic_tokens(40 + 3 * b, seed=7400 + b) for b in range(B)]
    spk = [b % 5 for b in range(B)]
    k, v = env.split("=")
    runs = []
    for setting in (None, v):
        if setting is not None:
            os.environ[k] = setting
        try:
            dev = ma.Device(full_model, weights="bf16")
            runs.append(dev.synthesize(toks, speakers=spk, max_dec_steps=steps, ignore_eos=True, trace=True))
            dev.close()
        finally:
            os.environ.pop(k, None)
    a, b = runs
    np.testing.assert_array_equal(a.codes, b.codes)
    assert np.array_equal(a.hidden, b.hidden)


def test_bf16_full_model_sampled_batch8_equals_single(ma, full_model):
    """configs[3]'s per-GPU batch with top-k sampling: slot b draws from stream b, so
    it reproduces its single run with stream_base=b bit for bit."""
    B, steps = 8, 48
    toks = [ma.synthetic_tokens(30 + 5 * b, seed=7100 + b) for b in range(B)]
    kw = dict(max_dec_steps=steps, temperature=0.7, top_k=80, seed=31, ignore_eos=True, trace=True)
    dev = ma.Device(full_model, weights="bf16")
    rb = dev.synthesize(toks, speakers=[b % 5 for b in range(B)], **kw)
    for b in (0, 5, 7):
        rs = dev.synthesize([toks[b]], speakers=[b % 5], stream_base=b, **kw)
        assert np.array_equal(rb.codes[b], rs.codes[0]), f"slot {b} codes"
        assert np.array_equal(rb.hidden[b], rs.hidden[0]), f"slot {b} hidden"
    dev.close()


def test_q8_full_model_batch16_equals_single(ma, oracle, q8_full_model):
    """Q8_0 Magpie-357M at 16 utterances (int8 MFMA projections, F32 FFN convs on the
    f32 GEMV family in two 8-slot halves): each slot equals its single run bit for
    bit, and slot 0's decisions match the oracle's Q8_0 mode teacher forced."""
    B, steps = 16, 24
    toks = [ma.synthetic_tokens(40 + 3 * b, seed=7300 + b) for b in range(B)]
    spk = [b % 5 for b in range(B)]
    dev = ma.Device(q8_full_model, weights="q8")
    assert dev.max_batch() == 16
    rb = dev.synthesize(toks, speakers=spk, max_dec_steps=steps, ignore_eos=True, trace=True)
    assert (rb.n_frames == steps).all()
    for b in (0, 9, 15):
        rs = dev.synthesize([toks[b]], speakers=[spk[b]], max_dec_steps=steps, ignore_eos=True, trace=True)
        assert np.array_equal(rb.codes[b], rs.codes[0]), f"slot {b} codes"
        assert np.array_equal(rb.hidden[b], rs.hidden[0]), f"slot {b} hidden"
    dev.close()
    om = oracle.Model(q8_full_model)
    om.set_weight_mode(2)
    o = om.synthesize_forced(toks[0], rb.codes[0], speaker=spk[0], ignore_eos=True)
    om.close()
    res = compare_forced(rb.codes[0], o, tie_eps=Q8_TIE_EPS, max_ties=10)  # 5 % of 192
    assert res["decisions"] == steps * 8
    _hidden_ok(rb.hidden[0, :steps + 1], o["hidden"])


def test_q8_longform_60s_batched_equals_sentence_by_sentence(ma, oracle, q8_full_model, codec_model):
    """configs[4] as the bench runs it: 6 sentences x 216 frames (60.2 s of audio)
    streamed as one device batch with 4-frame codec chunks; every sentence's codes and
    audio chunks equal the same sentence streamed alone (stream_base = its index), and
    the first sentence's decisions match the oracle's Q8_0 mode (weight mode 2)."""
    n_s, frames = 6, 216
    sents = [ma.synthetic_tokens(40, seed=5000 + i) for i in range(n_s)]
    dev = ma.Device(q8_full_model, weights="q8")
    cdc = ma.Codec(codec_model)
    got = {i: [] for i in range(n_s)}
    codes_b, total, _ = dev.synthesize_stream(cdc, sents, lambda u, a: got[u].append(a) or True,
                                              max_dec_steps=frames, ignore_eos=True)
    assert total == n_s * frames * 1024
    for i in (0, 3, 5):
        one = []
        codes_s, _, _ = dev.synthesize_stream(cdc, [sents[i]], lambda u, a: one.append(a) or True,
                                              max_dec_steps=frames, ignore_eos=True, stream_base=i)
        assert np.array_equal(codes_s[0], codes_b[i]), f"sentence {i} codes"
        assert len(one) == len(got[i]) == frames // 4
        assert all(np.array_equal(x, y) for x, y in zip(one, got[i])), f"sentence {i} audio"
    cdc.close()
    # the whole first sentence (216 frames, 1,728 decisions) against the oracle's Q8_0
    # mode, teacher forced
    r = dev.synthesize([sents[0]], speakers=[0], max_dec_steps=frames, ignore_eos=True, trace=True)
    assert np.array_equal(r.codes[0], codes_b[0])
    dev.close()
    om = oracle.Model(q8_full_model)
    om.set_weight_mode(2)
    o = om.synthesize_forced(sents[0], r.codes[0], speaker=0, ignore_eos=True)
    om.close()
    res = compare_forced(r.codes[0], o, tie_eps=Q8_TIE_EPS, max_ties=86)  # <= 5 % of 1,728
    assert res["decisions"] == frames * 8
    _hidden_ok(r.hidden[0, :frames + 1], o["hidden"])
