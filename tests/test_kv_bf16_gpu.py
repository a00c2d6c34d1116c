"""bf16 SA cache (MP_KV_BF16, mp_hip_set_kv_mode) against the oracle's kv_bf16 mode.

No reference counterpart: the reference's graph-reuse cache is f32
(magpie.cpp:3313-3376). In this mode every K and V row is rounded to bf16 (round
to nearest even) when it is appended, in the 110-frame prefill and every decode
step, and every attention reads the rounded rows (include/magpie_hip.h). The
oracle restates exactly that (orc_set_kv_bf16), so:

- the prefill rows of the cache are the f32 mode's rows rounded, bit for bit;
- every decision is checked teacher forced against the oracle in the same mode
  (f32 weights: the f32 bars; bf16 weights at batch 16: the bf16 bars);
- a batch equals its utterances run alone, bit for bit.
"""
import numpy as np
import pytest

from parity import compare_forced

pytestmark = pytest.mark.gpu

CTX = 110
TIE_EPS_F32 = 2e-4
BF16_TIE_EPS = 3e-2  # the oracle's own bf16 f32/f64 spread (test_decode_gpu.py)
# bf16 weights AND bf16 cache: two bf16 roundings whose flips (GPU f32 vs oracle f64
# arithmetic rounding a value to the other side of a bf16 half-ulp) both reach the
# logits. The near-tie bar sits just above the first flip measured on this case
# (margin 0.015) and below BF16_TIE_EPS, the bf16 mode's bar from the oracle's own
# f32/f64 spread over 256 frames (this case runs 16 frames teacher forced)
KV_BF16_TIE_EPS = 2e-2
HIDDEN_TOL, HIDDEN_REL = 3e-2, 5e-3


@pytest.fixture(scope="module")
def ma():
    import magpie_amd
    if magpie_amd.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return magpie_amd


@pytest.fixture
def oracle_kv(oracle):
    oracle.set_kv_bf16(True)
    try:
        yield oracle
    finally:
        oracle.set_kv_bf16(False)


def _bf16_rne(x):
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def _cache(dev, name, nb, layers, bf16):
    import ctypes
    n = dev.lib.mp_hip_debug_buffer(dev.h, name.encode(), None, 0)
    assert n > 0
    buf = np.zeros(n // (2 if bf16 else 4), np.uint16 if bf16 else np.float32)
    assert dev.lib.mp_hip_debug_buffer(dev.h, name.encode(), buf.ctypes.data_as(ctypes.c_void_p), n) == n
    return buf.reshape(nb, layers, -1, 768)


def test_prefill_rows_are_rounded_f32_rows(ma, small_model):
    """Layer 0's 110 prefill rows come from the same prefill GEMM in both modes (later
    layers see attention over rounded rows): the bf16 cache holds exactly the f32
    cache's values rounded to nearest even, and layer 1 differs."""
    tok = ma.synthetic_tokens(20, seed=1000)
    got = {}
    for kv in ("f32", "bf16"):
        dev = ma.Device(small_model, kv=kv)
        dev.synthesize([tok], speakers=[2], max_dec_steps=4, ignore_eos=True)
        got[kv] = (_cache(dev, "kc", 1, 2, kv == "bf16"), _cache(dev, "vc", 1, 2, kv == "bf16"))
        dev.close()
    for i in range(2):
        ref = _bf16_rne(got["f32"][i][:, 0, :CTX])
        np.testing.assert_array_equal(got["bf16"][i][:, 0, :CTX], ref)
        assert not np.array_equal(got["bf16"][i][:, 1, :CTX], _bf16_rne(got["f32"][i][:, 1, :CTX]))
    print(f"layer-0 prefill K/V rows: {ref.size} values each, bf16 == RNE(f32) bit for bit")


def test_f32_weights_bf16_kv_every_decision(ma, oracle_kv, small_model):
    """f32 weights, bf16 cache: all 40 x 8 decisions against the oracle's kv_bf16
    mode conditioned on the GPU's own codes; both round the same K/V rows, so the
    f32 bars apply (hidden 2e-3, near-tie 2e-4)."""
    tok = ma.synthetic_tokens(24, seed=1000)
    dev = ma.Device(small_model, kv="bf16")
    r = dev.synthesize([tok], speakers=[1], max_dec_steps=40, ignore_eos=True, trace=True)
    dev.close()
    om = oracle_kv.Model(small_model)
    o = om.synthesize_forced(tok, r.codes[0], speaker=1, ignore_eos=True)
    om.close()
    res = compare_forced(r.codes[0], o, tie_eps=TIE_EPS_F32, max_ties=2)
    assert res["decisions"] == 320
    err = np.abs(r.hidden[0, :41] - o["hidden"][:41]).max()
    print(f"bf16 KV, f32 weights: hidden max abs err {err:.3g}")
    assert err < 2e-3


def test_bf16_kv_changes_the_cache_not_the_path(ma, small_model):
    """The mode is per batch: f32 -> bf16 -> f32 on one device reproduces the
    first f32 run bit for bit, and the bf16 run differs from it (the rounding is live)."""
    tok = ma.synthetic_tokens(20, seed=1001)
    dev = ma.Device(small_model)
    a = dev.synthesize([tok], speakers=[0], max_dec_steps=16, ignore_eos=True, trace=True)
    dev._check(dev.lib.mp_hip_set_kv_mode(dev.h, 1))
    b = dev.synthesize([tok], speakers=[0], max_dec_steps=16, ignore_eos=True, trace=True)
    dev._check(dev.lib.mp_hip_set_kv_mode(dev.h, 0))
    c = dev.synthesize([tok], speakers=[0], max_dec_steps=16, ignore_eos=True, trace=True)
    dev.close()
    assert np.array_equal(a.hidden, c.hidden) and np.array_equal(a.codes[0], c.codes[0])
    assert not np.array_equal(a.hidden, b.hidden)
    assert dev.lib.mp_hip_set_kv_mode(None, 1) != 0


def test_bf16_weights_bf16_kv_batch16_full_model(ma, oracle_kv, full_model):
    """configs[2] shape (bf16 weights, 16 utterances, 12 layers) with the bf16 cache:
    batch == single bit for bit, slot 0 teacher forced against oracle mode 1 + kv_bf16."""
    B, steps = 16, 24
    toks = [ma.synthetic_tokens(40 + 3 * b, seed=7100 + b) for b in range(B)]
    spk = [b % 5 for b in range(B)]
    dev = ma.Device(full_model, weights="bf16", kv="bf16")
    rb = dev.synthesize(toks, speakers=spk, max_dec_steps=steps, ignore_eos=True, trace=True)
    for b in (0, B - 1):
        rs = dev.synthesize([toks[b]], speakers=[spk[b]], max_dec_steps=steps, ignore_eos=True, trace=True)
        assert np.array_equal(rb.codes[b], rs.codes[0]), f"slot {b} codes"
        assert np.array_equal(rb.hidden[b], rs.hidden[0]), f"slot {b} hidden"
    dev.close()
    om = oracle_kv.Model(full_model)
    om.set_weight_mode(1)
    o = om.synthesize_forced(toks[0], rb.codes[0], speaker=spk[0], ignore_eos=True)
    om.close()
    h, ho = rb.hidden[0, :steps + 1], o["hidden"]
    err = np.abs(h - ho).max()
    nrm = np.linalg.norm(ho, axis=-1)
    rel = (np.linalg.norm(h - ho, axis=-1)[nrm > 0] / nrm[nrm > 0]).max()
    print(f"bf16 weights + bf16 KV, B=16: hidden max abs {err:.3g}, rel L2 {rel:.3g}")
    assert err < HIDDEN_TOL and rel < HIDDEN_REL
    res = compare_forced(rb.codes[0], o, tie_eps=KV_BF16_TIE_EPS, max_ties=6)
    assert res["decisions"] == steps * 8
