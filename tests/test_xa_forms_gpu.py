"""Cross-attention forms of the decode step (mp_hip_set_xa_mode).

The reassociated form (K' = W_q^T K, V' = W_o V precomputed per utterance, fused in
the O-projection launch) reads 6 KB per text token and layer; the direct form
(q_net GEMV, attention over K, V, o_net: magpie.cpp:1713-1767, the order the oracle
restates) reads 1 KB per token + 0.79 MB of q_net / o_net, so AUTO switches to it
above MP_XA_DIRECT_T = 160 tokens. Both are checked against the oracle at the f32
bar, and batches against single runs of the same form.
"""
import numpy as np
import pytest

from parity import compare_codes, compare_forced

pytestmark = pytest.mark.gpu

HIDDEN_TOL = 2e-5  # f32 vs the acc64 oracle (tests/test_decode_gpu.py)
BF16_TIE_EPS, BF16_HIDDEN_TOL = 3e-2, 3e-2  # test_decode_gpu.py


@pytest.fixture(scope="module")
def ma():
    import magpie_amd
    if magpie_amd.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return magpie_amd


def _gpu(ma, path, toks, steps, xa, weights="f32", spk=None):
    dev = ma.Device(path, weights=weights, xa=xa)
    r = dev.synthesize(toks, speakers=spk or [b % 5 for b in range(len(toks))], max_dec_steps=steps,
                       ignore_eos=True, trace=True)
    dev.close()
    return r


def test_direct_f32_small_model_matches_oracle(ma, oracle, small_model):
    tok = ma.synthetic_tokens(24, seed=1000)
    r = _gpu(ma, small_model, [tok], 40, "direct", spk=[1])
    om = oracle.Model(small_model)
    o = om.synthesize(tok, speaker=1, max_steps=40, ignore_eos=True, trace=True)
    om.close()
    res = compare_codes(r.codes[0], o["codes"], o["margins"])
    n = res["frames"]
    err = np.abs(r.hidden[0, :n + 1] - o["hidden"][:n + 1]).max()
    assert err < HIDDEN_TOL, f"hidden max abs err {err}"


def test_auto_switches_to_direct_on_long_texts(ma, small_model):
    """T = 200 > 160: AUTO runs the direct form (bit-identical to forcing it) and the
    reassociated form differs from it only by rounding."""
    tok = [ma.synthetic_tokens(200, seed=77)]
    auto = _gpu(ma, small_model, tok, 12, "auto")
    direct = _gpu(ma, small_model, tok, 12, "direct")
    reassoc = _gpu(ma, small_model, tok, 12, "reassoc")
    assert np.array_equal(auto.hidden, direct.hidden) and np.array_equal(auto.codes, direct.codes)
    d = np.abs(reassoc.hidden - direct.hidden).max()
    assert 0 < d < HIDDEN_TOL, d
    short = [ma.synthetic_tokens(100, seed=78)]  # below the threshold AUTO keeps the reassociated form
    assert np.array_equal(_gpu(ma, small_model, short, 8, "auto").hidden,
                          _gpu(ma, small_model, short, 8, "reassoc").hidden)


@pytest.mark.parametrize("weights,B", [("f32", 4), ("f32", 8), ("bf16", 16)])
def test_direct_batch_equals_single(ma, small_model, weights, B):
    toks = [ma.synthetic_tokens(10 + 9 * b, seed=4000 + b) for b in range(B)]
    rb = _gpu(ma, small_model, toks, 20, "direct", weights=weights)
    for b in (0, B // 2, B - 1):
        rs = _gpu(ma, small_model, [toks[b]], 20, "direct", weights=weights, spk=[b % 5])
        assert np.array_equal(rb.codes[b], rs.codes[0]), f"slot {b} codes"
        assert np.array_equal(rb.hidden[b], rs.hidden[0]), f"slot {b} hidden"


def test_long_text_full_model_matches_oracle(ma, oracle, full_model):
    """Magpie-357M with a 300-token text (AUTO -> direct): every frame's codes
    against the oracle at the f32 bar."""
    tok = ma.synthetic_tokens(300, seed=1300)
    r = _gpu(ma, full_model, [tok], 24, "auto", spk=[0])
    om = oracle.Model(full_model)
    o = om.synthesize(tok, speaker=0, max_steps=24, ignore_eos=True, trace=True)
    om.close()
    res = compare_codes(r.codes[0], o["codes"], o["margins"])
    n = res["frames"]
    err = np.abs(r.hidden[0, :n + 1] - o["hidden"][:n + 1]).max()
    assert err < HIDDEN_TOL, f"hidden max abs err {err}"


def test_direct_bf16_teacher_forced(ma, oracle, small_model):
    """bf16 weight mode keeps XA f32 (oracle weight mode 1): direct form, every
    decision teacher forced."""
    tok = ma.synthetic_tokens(24, seed=1000)
    r = _gpu(ma, small_model, [tok], 40, "direct", weights="bf16", spk=[1])
    om = oracle.Model(small_model)
    om.set_weight_mode(1)
    o = om.synthesize_forced(tok, r.codes[0], speaker=1, ignore_eos=True)
    om.close()
    assert compare_forced(r.codes[0], o, tie_eps=BF16_TIE_EPS, max_ties=8)["decisions"] == 40 * 8
    assert np.abs(r.hidden[0, :41] - o["hidden"]).max() < BF16_HIDDEN_TOL
