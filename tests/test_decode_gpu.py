"""GPU parity of the decode path (C-ABI -> HIP kernels) against the CPU oracle.

Reference behaviour: magpie_synthesize_codes_graph_reuse (magpie.cpp:4063-4432)
at temperature 0. Bar: bit-identical codec-token indices (up to a reported
genuine near-tie, tests/parity.py) and decoder hidden states within 2e-5 abs of
the acc64 oracle in the f32 mode (measured ~2e-6; the reference's own
full-decoder tolerance vs ggml is 2.66e-3, docs/STATUS.md:108-116, so this bar
is ~100x tighter than the reference's and ~10x above what f32 rounding gives).
"""
import numpy as np
import pytest

from parity import compare_codes, compare_forced

pytestmark = pytest.mark.gpu

HIDDEN_TOL = 2e-5


@pytest.fixture(scope="module")
def ma():
    import magpie_amd
    if magpie_amd.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return magpie_amd


def _run_both(ma, oracle, model_path, tokens, steps, speaker=0, ignore_eos=False):
    dev = ma.Device(model_path)
    r = dev.synthesize([tokens], speakers=[speaker], max_dec_steps=steps, ignore_eos=ignore_eos, trace=True)
    dev.close()
    om = oracle.Model(model_path)
    o = om.synthesize(tokens, speaker=speaker, max_steps=steps, ignore_eos=ignore_eos, trace=True)
    om.close()
    return r, o


def test_small_model_codes_and_hidden(ma, oracle, small_model):
    tok = ma.synthetic_tokens(24, seed=1000)
    r, o = _run_both(ma, oracle, small_model, tok, steps=40, speaker=1)
    res = compare_codes(r.codes[0], o["codes"], o["margins"])
    n = res["frames"]
    # hidden after BOS and after every step that both sides computed identically
    h_gpu, h_orc = r.hidden[0, :n + 1], o["hidden"][:n + 1]
    err = np.abs(h_gpu - h_orc).max()
    assert err < HIDDEN_TOL, f"hidden max abs err {err}"


def test_full_model_codes_and_hidden(ma, oracle, full_model):
    tok = ma.synthetic_tokens(64, seed=1000)
    r, o = _run_both(ma, oracle, full_model, tok, steps=24, speaker=0, ignore_eos=True)
    res = compare_codes(r.codes[0], o["codes"], o["margins"])
    n = res["frames"]
    err = np.abs(r.hidden[0, :n + 1] - o["hidden"][:n + 1]).max()
    assert err < HIDDEN_TOL, f"hidden max abs err {err}"
    assert r.n_frames[0] == 24


def test_small_model_matches_committed_golden(ma, small_model):
    """GPU codes vs the committed oracle fixture (tests/golden/small_model_codes.json,
    tests/golden/make_golden.py), independent of a live oracle run: every frame
    identical, hidden states (first 8 elements, L1 norm) within the f32 bar."""
    import json
    import os
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "small_model_codes.json")))
    dev = ma.Device(small_model)
    for case in gold["cases"]:
        r = dev.synthesize([case["tokens"]], speakers=[case["speaker"]], max_dec_steps=case["max_steps"],
                           trace=True)
        n = case["n_frames"]
        assert r.n_frames[0] == n
        np.testing.assert_array_equal(r.codes[0], np.asarray(case["codes"], np.int32).reshape(-1, 8))
        h = r.hidden[0, :n + 1]
        assert np.abs(h[:, :8] - np.asarray(case["hidden_first8"])).max() < HIDDEN_TOL
        l1 = np.abs(h).sum(axis=1)
        assert np.abs(l1 - np.asarray(case["hidden_l1"])).max() < HIDDEN_TOL * 768
        print(f"golden case (T={len(case['tokens'])}, speaker {case['speaker']}): {n} frames identical")
    dev.close()


def test_eos_stops_like_reference(ma, oracle, eos_model):
    """EOS is forbidden for the first 4 frames (magpie.cpp:4267,4325); the EOS
    frame itself is not emitted (4349-4352)."""
    tok = ma.synthetic_tokens(16, seed=7)
    r, o = _run_both(ma, oracle, eos_model, tok, steps=64)
    assert o["n_frames"] == 4
    assert r.n_frames[0] == o["n_frames"]
    compare_codes(r.codes[0], o["codes"], o["margins"])


def test_max_steps_boundary(ma, oracle, small_model):
    tok = ma.synthetic_tokens(8, seed=3)
    r, o = _run_both(ma, oracle, small_model, tok, steps=5, ignore_eos=True)
    assert r.n_frames[0] == 5 == o["n_frames"]
    compare_codes(r.codes[0], o["codes"], o["margins"])


@pytest.mark.parametrize("B", [2, 4, 8])
def test_batch_equals_single(ma, small_model, B):
    """Batched decode is new (the reference is batch=1); its parity
    criterion: each utterance in a batch equals the same utterance run alone."""
    toks = [ma.synthetic_tokens(8 + 5 * b, seed=1000 + b) for b in range(B)]
    spk = [b % 5 for b in range(B)]
    dev = ma.Device(small_model)
    rb = dev.synthesize(toks, speakers=spk, max_dec_steps=20, trace=True)
    for b in range(B):
        r1 = dev.synthesize([toks[b]], speakers=[spk[b]], max_dec_steps=20, trace=True)
        np.testing.assert_array_equal(rb.codes[b], r1.codes[0])
        np.testing.assert_allclose(rb.hidden[b, :rb.n_frames[b] + 1], r1.hidden[0, :r1.n_frames[0] + 1], atol=1e-5)
    dev.close()


@pytest.mark.parametrize("weights,B", [("f32", 4), ("bf16", 4), ("q8", 4), ("f32", 8), ("bf16", 16), ("q8", 8),
                                       ("q8", 16)])
def test_sampled_batch_equals_single(ma, small_model, q8_model, weights, B):
    """Sampling is what exposes ulp-level batch variance (a near-tie in the top-k
    order flips a draw), so a sampled batch over many frames must reproduce each
    utterance run alone bit for bit: codes, decoder hidden, every codebook draw.
    B >= 8 runs the LT pick as its own per-slot launch (lt_pick_kernel)."""
    path = q8_model if weights == "q8" else small_model
    toks = [ma.synthetic_tokens(9 + 7 * (b % 6), seed=3000 + b) for b in range(B)]
    kw = dict(max_dec_steps=64, temperature=0.7, top_k=80, seed=17, ignore_eos=True, trace=True)
    dev = ma.Device(path, weights=weights)
    rb = dev.synthesize(toks, speakers=[b % 5 for b in range(B)], **kw)
    for b in (range(B) if B <= 4 else (0, 3, B - 1)):
        rs = dev.synthesize([toks[b]], speakers=[b % 5], stream_base=b, **kw)
        assert np.array_equal(rb.codes[b], rs.codes[0]), f"slot {b}"
        assert np.array_equal(rb.hidden[b], rs.hidden[0]), f"slot {b} hidden"
    dev.close()


def test_q8_model_loads_and_matches_oracle(ma, oracle, q8_model):
    """Q8_0 attention/LT projections (convert_magpie_to_gguf.py:155-176) are
    dequantised on load; the oracle dequantises the same blocks."""
    tok = ma.synthetic_tokens(12, seed=11)
    r, o = _run_both(ma, oracle, q8_model, tok, steps=16, ignore_eos=True)
    compare_codes(r.codes[0], o["codes"], o["margins"])


def test_repeat_runs_are_deterministic(ma, small_model):
    tok = ma.synthetic_tokens(20, seed=5)
    dev = ma.Device(small_model)
    a = dev.synthesize([tok], max_dec_steps=16, ignore_eos=True)
    b = dev.synthesize([tok], max_dec_steps=16, ignore_eos=True)
    np.testing.assert_array_equal(a.codes[0], b.codes[0])
    dev.close()


def test_invalid_arguments_fail_loudly(ma, small_model):
    dev = ma.Device(small_model)
    with pytest.raises(ma.MagpieError):
        dev.synthesize([[99999]], max_dec_steps=4)
    with pytest.raises(ma.MagpieError):
        dev.synthesize([[1, 2, 3]], speakers=[7], max_dec_steps=4)
    dev.close()


# ---------------------------------------------------------------- sampling
# sample_top_k (magpie.cpp:1072-1109) on the device. The reference draws from an
# unseeded mt19937 (1129), so its sampled codes are not reproducible run to run;
# parity here is GPU == oracle on the same counter-based stream u(seed, slot,
# step, cb), bit-identical up to a reported near-boundary draw (margin < TIE_EPS).

def _sample_both(ma, oracle, model_path, toks, steps, temperature, top_k, seed, ignore_eos=False):
    dev = ma.Device(model_path)
    r = dev.synthesize(toks, speakers=[b % 5 for b in range(len(toks))], max_dec_steps=steps,
                       temperature=temperature, top_k=top_k, seed=seed, ignore_eos=ignore_eos)
    dev.close()
    om = oracle.Model(model_path)
    outs = [om.synthesize(t, speaker=b % 5, max_steps=steps, ignore_eos=ignore_eos, trace=False,
                          temperature=temperature, top_k=top_k, seed=seed, stream=b) for b, t in enumerate(toks)]
    om.close()
    return r, outs


@pytest.mark.parametrize("B", [1, 3])
def test_topk_sampling_matches_oracle(ma, oracle, small_model, B):
    toks = [ma.synthetic_tokens(12 + 3 * b, seed=500 + b) for b in range(B)]
    r, outs = _sample_both(ma, oracle, small_model, toks, steps=32, temperature=0.7, top_k=80, seed=1234)
    for b in range(B):
        compare_codes(r.codes[b], outs[b]["codes"], outs[b]["margins"])
    # sampling actually departs from greedy
    g = ma.Device(small_model)
    rg = g.synthesize(toks[:1], speakers=[0], max_dec_steps=32)
    g.close()
    assert not np.array_equal(rg.codes[0], r.codes[0])


def test_topk_full_vocab_sampling(ma, oracle, small_model):
    """top_k = 2024: plain temperature sampling over every unmasked token."""
    toks = [ma.synthetic_tokens(10, seed=77)]
    r, outs = _sample_both(ma, oracle, small_model, toks, steps=6, temperature=1.0, top_k=2024, seed=9)
    compare_codes(r.codes[0], outs[0]["codes"], outs[0]["margins"])


def test_top1_sampling_is_greedy(ma, small_model):
    toks = [ma.synthetic_tokens(16, seed=3)]
    d = ma.Device(small_model)
    s = d.synthesize(toks, max_dec_steps=20, temperature=0.9, top_k=1, seed=5)
    g = d.synthesize(toks, max_dec_steps=20)
    d.close()
    assert np.array_equal(s.codes[0], g.codes[0])


def test_sampling_eos_from_argmax(ma, oracle, eos_model):
    """EOS stops the utterance when any codebook's sampled code OR argmax is EOS
    (magpie.cpp:4340-4348); EOS is forbidden for the first 4 frames."""
    toks = [ma.synthetic_tokens(16, seed=7), ma.synthetic_tokens(9, seed=8)]
    r, outs = _sample_both(ma, oracle, eos_model, toks, steps=64, temperature=0.7, top_k=80, seed=99)
    for b in range(2):
        assert outs[b]["n_frames"] == 4
        assert r.n_frames[b] == 4
        compare_codes(r.codes[b], outs[b]["codes"], outs[b]["margins"])


# ---------------------------------------------------------------- bf16 weight mode
# Decode projections on bf16 MFMA (mp_decode_b16.hip) vs the oracle's weight
# mode 1 (bf16-rounded weights and input activations, magpie_oracle.h). Rounding
# activations to bf16 is discontinuous: an f32-level difference (GPU f32 vs
# oracle f64 accumulation, ~1e-7 relative) flips an element across a bf16
# rounding boundary a few times per step, a 2^-8 relative step in that input.
# On the synthetic weights the residual stream is small (std ~0.03) and every
# LayerNorm amplifies such a flip ~30x, so hidden states drift apart by ~1e-2
# over 24 frames (a mis-indexed fragment gives O(1)). The bar is therefore wider
# than f32's: identical codes up to a decision whose oracle margin is < 1e-2
# (logits / draw probability), hidden within 3e-2 max abs and 5e-3 relative L2.
# bf16 near-tie bar: the oracle's own bf16 mode with f32 instead of f64 accumulation
# shifts margins by up to 0.026 and flips a decision of margin 0.0119
# (test_oracle_cpu.py::test_bf16_mode_accumulation_spread)
BF16_TIE_EPS = 3e-2
BF16_HIDDEN_TOL = 3e-2
BF16_HIDDEN_REL = 5e-3


def _rel_l2(h_gpu, h_orc):
    """per-step relative L2 error over the steps the oracle computed (a run that ends
    at max_dec_steps leaves the last trace row unwritten on both sides)"""
    nrm = np.linalg.norm(h_orc, axis=-1)
    live = nrm > 0
    return np.linalg.norm(h_gpu - h_orc, axis=-1)[live] / nrm[live]


def _check_hidden_b16(h_gpu, h_orc):
    err = np.abs(h_gpu - h_orc).max()
    rel = _rel_l2(h_gpu, h_orc)
    print(f"hidden vs oracle: max abs err {err:.3g}, max relative L2 {rel.max():.3g} over {len(h_gpu)} steps")
    assert err < BF16_HIDDEN_TOL, f"hidden max abs err {err}"
    assert rel.max() < BF16_HIDDEN_REL, f"hidden rel L2 err {rel.max()}"

def _run_both_b16(ma, oracle, model_path, tokens, steps, speaker=0, ignore_eos=False):
    dev = ma.Device(model_path, weights="bf16")
    r = dev.synthesize([tokens], speakers=[speaker], max_dec_steps=steps, ignore_eos=ignore_eos, trace=True)
    dev.close()
    om = oracle.Model(model_path)
    om.set_weight_mode(1)
    o = om.synthesize(tokens, speaker=speaker, max_steps=steps, ignore_eos=ignore_eos, trace=True)
    om.close()
    return r, o


def test_bf16_small_model_matches_oracle(ma, oracle, small_model):
    tok = ma.synthetic_tokens(24, seed=1000)
    r, o = _run_both_b16(ma, oracle, small_model, tok, steps=40, speaker=1)
    # bf16 activation rounding flips amplify into ~1e-2 logit differences: a genuine
    # near-tie (oracle margin < 1e-2) may end the free-running comparison early
    res = compare_codes(r.codes[0], o["codes"], o["margins"], tie_eps=BF16_TIE_EPS, min_frames=8)
    n = res["frames"]
    _check_hidden_b16(r.hidden[0, :n + 1], o["hidden"][:n + 1])


@pytest.mark.parametrize("weights", ["bf16"])
def test_every_decision_teacher_forced(ma, oracle, small_model, q8_model, weights):
    """All 40 x 8 decisions of a bf16 GPU run (Q8: test_q8_small_model_matches_oracle),
    each checked against the oracle (weight mode 1) conditioned on the GPU's own
    earlier codes: a decision may
    differ only at a genuine near-tie, and the hidden state stays within the bar
    along the whole trajectory (no early stop at the first near-tie)."""
    path = q8_model if weights == "q8" else small_model
    tok = ma.synthetic_tokens(24, seed=1000)
    dev = ma.Device(path, weights=weights)
    r = dev.synthesize([tok], speakers=[1], max_dec_steps=40, ignore_eos=True, trace=True)
    dev.close()
    om = oracle.Model(path)
    om.set_weight_mode(1 if weights == "bf16" else 2)
    o = om.synthesize_forced(tok, r.codes[0], speaker=1, ignore_eos=True)
    om.close()
    res = compare_forced(r.codes[0], o, tie_eps=BF16_TIE_EPS if weights == "bf16" else Q8_TIE_EPS,
                         max_ties=8 if weights == "bf16" else 16)  # 16 = 5 % of 320
    assert res["decisions"] == 320
    _check_hidden_b16(r.hidden[0, :41], o["hidden"][:41])


def test_bf16_full_model_matches_oracle(ma, oracle, full_model):
    """Free running until the first genuine near-tie (this case has one of margin
    5.5e-3 at frame 9 that an ulp-level change anywhere can flip), then every one of
    the 192 decisions teacher forced along the GPU's own codes."""
    tok = ma.synthetic_tokens(64, seed=1000)
    r, o = _run_both_b16(ma, oracle, full_model, tok, steps=24, ignore_eos=True)
    res = compare_codes(r.codes[0], o["codes"], o["margins"], tie_eps=BF16_TIE_EPS, min_frames=8)
    n = res["frames"]
    _check_hidden_b16(r.hidden[0, :n + 1], o["hidden"][:n + 1])
    assert r.n_frames[0] == 24
    om = oracle.Model(full_model)
    om.set_weight_mode(1)
    of = om.synthesize_forced(tok, r.codes[0], speaker=0, ignore_eos=True)
    om.close()
    assert compare_forced(r.codes[0], of, tie_eps=BF16_TIE_EPS, max_ties=6)["decisions"] == 24 * 8
    _check_hidden_b16(r.hidden[0, :25], of["hidden"])


@pytest.mark.parametrize("B", [3, 16])
def test_bf16_batch_equals_single(ma, small_model, B):
    """bf16 batches reach 16 slots; each output's MFMA arithmetic is independent of
    the batch size, so a batch reproduces its utterances run alone exactly."""
    toks = [ma.synthetic_tokens(8 + 3 * b, seed=2000 + b) for b in range(B)]
    spk = [b % 5 for b in range(B)]
    dev = ma.Device(small_model, weights="bf16")
    rb = dev.synthesize(toks, speakers=spk, max_dec_steps=24, ignore_eos=True, trace=True)
    for b in (0, B // 2, B - 1):
        rs = dev.synthesize([toks[b]], speakers=[spk[b]], max_dec_steps=24, ignore_eos=True, trace=True)
        assert np.array_equal(rb.codes[b], rs.codes[0]), f"slot {b}"
        assert np.array_equal(rb.hidden[b], rs.hidden[0]), f"slot {b} hidden"
    dev.close()


# ---------------------------------------------------------------- F16 weight mode
# An F16 GGUF (the converter's --outtype f16) with ggml's F16 mul_mat semantics
# (MP_WEIGHTS_F16) vs the oracle's weight mode 3. Every decision teacher forced;
# f16 rounding is 8x finer than bf16, the bars are the bf16 ones (the fused XA
# applies o_net to the unrounded attention output, a documented deviation).
def test_f16_small_model_matches_oracle(ma, oracle, f16_model):
    tok = ma.synthetic_tokens(24, seed=1000)
    dev = ma.Device(f16_model, weights="f16")
    r = dev.synthesize([tok], speakers=[1], max_dec_steps=40, ignore_eos=True, trace=True)
    dev.close()
    om = oracle.Model(f16_model)
    om.set_weight_mode(3)
    o = om.synthesize_forced(tok, r.codes[0], speaker=1, ignore_eos=True)
    om.close()
    res = compare_forced(r.codes[0], o, tie_eps=BF16_TIE_EPS, max_ties=8)
    assert res["decisions"] == 320
    _check_hidden_b16(r.hidden[0, :41], o["hidden"][:41])
    err = np.abs(r.hidden[0, :41] - o["hidden"][:41]).max()
    print(f"f16 vs oracle mode 3: hidden max abs err {err:.3g}")


def test_f16_mode_rounds_like_ggml(ma, f16_model):
    """The F16 mode is not the widened-f32 mode (activations really are rounded)."""
    tok = ma.synthetic_tokens(16, seed=3)
    d16 = ma.Device(f16_model, weights="f16")
    a = d16.synthesize([tok], max_dec_steps=4, ignore_eos=True, trace=True)
    d16.close()
    d32 = ma.Device(f16_model)
    b = d32.synthesize([tok], max_dec_steps=4, ignore_eos=True, trace=True)
    d32.close()
    d = np.abs(a.hidden[0, 0] - b.hidden[0, 0]).max()
    assert 1e-6 < d < 2e-2, d


@pytest.mark.parametrize("B", [3, 16])
def test_f16_batch_equals_single(ma, f16_model, B):
    toks = [ma.synthetic_tokens(8 + 3 * b, seed=2500 + b) for b in range(B)]
    spk = [b % 5 for b in range(B)]
    dev = ma.Device(f16_model, weights="f16")
    rb = dev.synthesize(toks, speakers=spk, max_dec_steps=16, ignore_eos=True, trace=True)
    for b in (0, B - 1):
        rs = dev.synthesize([toks[b]], speakers=[spk[b]], max_dec_steps=16, ignore_eos=True, trace=True)
        assert np.array_equal(rb.codes[b], rs.codes[0]) and np.array_equal(rb.hidden[b], rs.hidden[0]), f"slot {b}"
    dev.close()


def test_f16_mode_needs_f16_file(ma, small_model):
    with pytest.raises(ma.MagpieError):
        ma.Device(small_model, weights="f16")


def test_f32_mode_rejects_batch_16(ma, small_model):
    dev = ma.Device(small_model)
    with pytest.raises(ma.MagpieError):
        dev.synthesize([ma.synthetic_tokens(8, seed=b) for b in range(9)], max_dec_steps=4)
    dev.close()


# ---------------------------------------------------------------- Q8_0 weight mode
# The reference's Q8 GGUF (convert_magpie_to_gguf.py:155-176) run the way ggml
# runs it: Q8_0 tensors stay int8 and every activation row they multiply is
# quantised to Q8_0 (mp_decode_q8.hip, gemm_q8_kernel), vs the oracle's weight
# mode 2. Quantising activations is discontinuous like bf16 rounding (an
# f32-level difference moves an element across a rounding boundary now and
# then, a 1/127-of-amax step; the oracle's own f64 vs f32 accumulation differ
# by ~3e-3 in the hidden state for that reason): same bar as the bf16 mode.
# Q8 decisions are inherently more sensitive: the oracle's OWN f32-accumulating mode,
# teacher forced along its f64 run of the full Q8 model (48 frames), differs at 10 of
# 384 decisions, with oracle margins up to 0.034 (activation-quantisation flips move
# the hidden state by up to 2e-2, and the decisive heads turn that into ~1e-1 of
# logit). Any f32 implementation is held to that spread: a differing decision needs
# an oracle margin < 0.1, and at most 5 % of decisions may differ (the hidden-state
# bar below is the precise check of the arithmetic).
Q8_TIE_EPS = 1e-1
# Hidden-state bars per case, ~2-4x the error each case measures (printed by every test;
# gpurun_out/r05f_tests.log): small Q8 2.3e-3 / 6.7e-4, Q4 8.1e-3 / 2.2e-3, sampled
# 5.5e-3 / 1.6e-3, full Q8 1.7e-2 / 4.5e-3 (max abs / max relative L2 over the steps).
# What the error is: every integer part of the Q8_0 arithmetic is bit-exact given the
# same f32 input row (tests/test_q8_exact_gpu.py: activation blocks, fp16 scales and int32
# block dots of every int8 GEMM launch). What remains is the f32 rows themselves (sums in
# another order, ~1e-7 relative), and where such a difference crosses a rounding boundary
# of an activation block the quantised operand moves by a whole 1/127-of-amax step. On the
# 2-layer model that is a few isolated flips (median step 9.5e-7); on the 12-layer model an
# early flip lands in a layer's KV cache row and every later step attends over it, so the
# error persists at ~1.4e-2 (median step) without growing (max 1.7e-2 over 25 steps): a
# shifted trajectory, not accumulating drift. Bars: ~2x the measured maximum.
Q8_BARS = {"small": (1e-2, 3e-3), "q4": (2e-2, 5e-3), "sampled": (1.5e-2, 4e-3), "full": (3e-2, 5e-3)}


def _check_hidden_q8(h_gpu, h_orc, case):
    tol, rtol = Q8_BARS[case]
    per_step = np.abs(h_gpu - h_orc).max(axis=-1)
    err = per_step.max()
    rel = _rel_l2(h_gpu, h_orc)
    print(f"Q8 hidden vs oracle mode 2 ({case}): max abs err {err:.3g} (median step {np.median(per_step):.3g}), "
          f"max relative L2 {rel.max():.3g} over {len(h_gpu)} steps; bars {tol:g} / {rtol:g}")
    assert err < tol, f"hidden max abs err {err}"
    assert rel.max() < rtol, f"hidden rel L2 err {rel.max()}"
    return err


def _q8_forced(ma, oracle, model_path, tok, steps, speaker=0, tie_frac=0.05, **smp):
    dev = ma.Device(model_path, weights="q8")
    r = dev.synthesize([tok], speakers=[speaker], max_dec_steps=steps, ignore_eos=True, trace=True, **smp)
    dev.close()
    om = oracle.Model(model_path)
    om.set_weight_mode(2)
    o = om.synthesize_forced(tok, r.codes[0], speaker=speaker, ignore_eos=True, **smp)
    om.close()
    res = compare_forced(r.codes[0], o, tie_eps=Q8_TIE_EPS, max_ties=int(tie_frac * steps * 8))
    assert res["decisions"] == steps * 8
    return r, o


def test_q8_small_model_matches_oracle(ma, oracle, q8_model):
    """Q8 decisions are checked teacher forced (every decision, see Q8_TIE_EPS): a
    free-running comparison ends at the first quantisation-sensitive decision."""
    tok = ma.synthetic_tokens(24, seed=1000)
    r, o = _q8_forced(ma, oracle, q8_model, tok, steps=40, speaker=1)
    _check_hidden_q8(r.hidden[0, :41], o["hidden"], "small")


def test_q8_full_model_matches_oracle(ma, oracle, q8_full_model):
    tok = ma.synthetic_tokens(64, seed=1000)
    r, o = _q8_forced(ma, oracle, q8_full_model, tok, steps=24)
    _check_hidden_q8(r.hidden[0, :25], o["hidden"], "full")
    assert r.n_frames[0] == 24


def test_q8_mode_differs_from_dequantised(ma, q8_model):
    """Activation quantisation really happens (q8 != dequantised-f32 mode)."""
    tok = ma.synthetic_tokens(16, seed=3)
    d8 = ma.Device(q8_model, weights="q8")
    a = d8.synthesize([tok], max_dec_steps=4, ignore_eos=True, trace=True)
    d8.close()
    d32 = ma.Device(q8_model)
    b = d32.synthesize([tok], max_dec_steps=4, ignore_eos=True, trace=True)
    d32.close()
    d = np.abs(a.hidden[0, 0] - b.hidden[0, 0]).max()
    assert 1e-5 < d < 0.2, d


@pytest.mark.parametrize("B", [3, 8, 16])
def test_q8_batch_equals_single(ma, q8_model, B):
    """The int8 MFMA projections serve every batch size (one 16-column tile, fixed
    K split and merge order), so slot b of a batch is its single run bit for bit."""
    toks = [ma.synthetic_tokens(8 + 3 * b, seed=3000 + b) for b in range(B)]
    spk = [b % 5 for b in range(B)]
    dev = ma.Device(q8_model, weights="q8")
    assert dev.max_batch() == 16
    rb = dev.synthesize(toks, speakers=spk, max_dec_steps=16, ignore_eos=True, trace=True)
    for b in ((0, B - 1) if B < 16 else (0, 7, 8, 15)):
        rs = dev.synthesize([toks[b]], speakers=[spk[b]], max_dec_steps=16, ignore_eos=True, trace=True)
        assert np.array_equal(rb.codes[b], rs.codes[0]), f"slot {b}"
        assert np.array_equal(rb.hidden[b], rs.hidden[0]), f"slot {b} hidden"
    dev.close()


def test_q8_sampling_matches_oracle(ma, oracle, q8_model):
    """Sampled Q8 decisions against the oracle's Q8_0 mode, teacher forced. They are
    the most fragile of all: the oracle's own f32-accumulating mode, teacher forced
    along its f64 run of this case, differs at 69 of 192 sampled decisions (a draw
    lands within ~4e-3 of an interval boundary at the median, and the activation
    quantiser's flips move the logits by ~1e-2). So here every differing decision
    needs an oracle margin < Q8_TIE_EPS and the count is only a sanity bound (50 %);
    the arithmetic under the draws is held to the Q8 hidden-state bars at every forced
    step, and the draws themselves exactly by test_q8_sampling_draws_exact."""
    tok = ma.synthetic_tokens(12, seed=41)
    r, o = _q8_forced(ma, oracle, q8_model, tok, steps=24, tie_frac=0.5, temperature=0.7, top_k=80, seed=77)
    _check_hidden_q8(r.hidden[0, :25], o["hidden"], "sampled")


def test_q8_sampling_draws_exact(ma, oracle, q8_model, tmp_path):
    """Every sampled Q8 decision recomputed from the logits the GPU's Q8_0 heads
    produced (MAGPIE_DUMP_LT, eager): the oracle's sample_top_k (magpie.cpp:1072-1109,
    after the 1133-1145 mask) on those logits with the same counter-stream draw
    u(seed, slot, step, cb) picks the GPU's code, decision for decision. This checks the
    device's top-k (radix select, compaction, rank, sequential sum / cumsum) exactly,
    apart from the logits' own numeric spread (test_q8_sampling_matches_oracle)."""
    import os
    steps, T, K, seed = 12, 0.7, 80, 77
    dump = str(tmp_path / "lt_q8_sampled.bin")
    env = {"MAGPIE_EAGER": "1", "MAGPIE_DUMP_LT": dump}
    os.environ.update(env)
    try:
        dev = ma.Device(q8_model, weights="q8")
        r = dev.synthesize([ma.synthetic_tokens(12, seed=41)], max_dec_steps=steps, ignore_eos=True,
                           temperature=T, top_k=K, seed=seed)
        dev.close()
    finally:
        for k in env:
            os.environ.pop(k, None)
    rec = np.fromfile(dump, dtype=np.float32).reshape(-1, 2024 + 8 + 4 * 256)
    # per iteration: the in_proj, position 0's q|k|v, then (LT step, head) for codebooks
    # 0..7 (the loop may run an iteration past the last frame)
    per = 18
    assert rec.shape[0] % per == 0 and rec.shape[0] >= per * steps, rec.shape
    codes = np.asarray(r.codes[0]).reshape(-1, 8)
    assert codes.shape[0] == steps
    cur = rec[:, 2024:2032].view(np.int32)
    # the iteration of frame st: LT step cb + 1 holds codebook cb's pick (codes_cur)
    nit = rec.shape[0] // per
    picks = np.stack([[cur[per * i + 2 + 2 * (cb + 1), cb] for cb in range(7)] for i in range(nit)])
    its = []
    for st in range(steps):
        cand = [i for i in range(its[-1] + 1 if its else 0, nit) if np.array_equal(picks[i], codes[st, :7])]
        assert cand, f"no LT record block holds frame {st}'s codes {codes[st]} (picks {picks[:3]})"
        its.append(cand[0])
    bos, eos = 2016, 2017
    close = []
    for st in range(steps):
        for cb in range(8):
            lg = rec[per * its[st] + 3 + 2 * cb, :2024].astype(np.float32).copy()
            lg[bos:bos + 8] = -np.inf  # ignore_eos: EOS masked too
            u = oracle.draw_u(seed, 0, st, cb)
            pick, mg = oracle.sample_top_k(lg, T, K, u)
            if pick != codes[st, cb]:
                assert mg < 1e-5, f"frame {st} cb {cb}: gpu {codes[st, cb]} oracle {pick} (margin {mg:.3g})"
                close.append(mg)
    print(f"Q8 sampled draws: {steps * 8} decisions recomputed from the GPU's logits, "
          f"{len(close)} differ (all within 1e-5 of an interval boundary)")
    assert len(close) <= 1


def test_q4_small_model_matches_oracle(ma, oracle, q4_model):
    """Q4_0 file (convert_magpie_to_gguf.py:107-138): its blocks run on the Q8_0
    kernels as int8 (q - 8) = ggml's vec_dot_q4_0_q8_0; teacher forced against the
    oracle's weight mode 2 on the same file, with the Q8 bars."""
    tok = ma.synthetic_tokens(24, seed=1000)
    r, o = _q8_forced(ma, oracle, q4_model, tok, steps=40, speaker=1)
    _check_hidden_q8(r.hidden[0, :41], o["hidden"], "q4")


@pytest.mark.parametrize("B", [3, 16])
def test_q4_batch_equals_single(ma, q4_model, B):
    toks = [ma.synthetic_tokens(8 + 3 * b, seed=3100 + b) for b in range(B)]
    dev = ma.Device(q4_model, weights="q4")
    rb = dev.synthesize(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=16, ignore_eos=True, trace=True)
    for b in (0, B - 1):
        rs = dev.synthesize([toks[b]], speakers=[b % 5], max_dec_steps=16, ignore_eos=True, trace=True)
        assert np.array_equal(rb.codes[b], rs.codes[0]) and np.array_equal(rb.hidden[b], rs.hidden[0]), f"slot {b}"
    dev.close()


def test_q8_mode_needs_q8_file(ma, small_model):
    with pytest.raises(ma.MagpieError):
        ma.Device(small_model, weights="q8")


def test_encode_text_alone_leaves_batch_untouched(ma, oracle, small_model):
    """mp_hip_encode_text (magpie_encode_text, magpie.cpp:2284-2374): the encoder output
    equals the oracle's encoder, and calling it between a batch's preamble and its decode
    changes nothing in that decode (own workspace)."""
    tok_a, tok_b = ma.synthetic_tokens(24, seed=1000), ma.synthetic_tokens(40, seed=11)
    dev = ma.Device(small_model)
    try:
        r1 = dev.synthesize([tok_a], speakers=[1], max_dec_steps=16, ignore_eos=True, trace=True)
        enc = dev.encode_text(tok_b)
        r2 = dev.decode(1, 16, trace=True)  # the same batch again (preamble state reused)
    finally:
        dev.close()
    np.testing.assert_array_equal(r1.codes[0], r2.codes[0])
    np.testing.assert_array_equal(r1.hidden, r2.hidden)
    om = oracle.Model(small_model)
    ref = om.encode(tok_b)
    om.close()
    err = float(np.abs(enc - ref).max())
    print(f"encoder alone (T = {len(tok_b)}): max abs err {err:.3g} vs the oracle")
    assert err < 2e-5


@pytest.mark.parametrize("weights", ["f32", "f16"])
def test_preamble_mfma_equals_valu(ma, small_model, f16_model, weights, monkeypatch):
    """The preamble GEMMs on the exact-f32 matrix cores (v_mfma_f32_16x16x4_f32: a
    k-ordered fmaf chain) compute the same bits as the f32 VALU kernel they replace
    (MAGPIE_PRE_VALU=1): encoder output, codes and every hidden state."""
    path = f16_model if weights == "f16" else small_model
    tok = ma.synthetic_tokens(40, seed=11)
    dev = ma.Device(path, weights=weights)
    try:
        a = dev.synthesize([tok], speakers=[3], max_dec_steps=12, ignore_eos=True, trace=True)
        ea = dev.encode_text(tok)
        monkeypatch.setenv("MAGPIE_PRE_VALU", "1")
        b = dev.synthesize([tok], speakers=[3], max_dec_steps=12, ignore_eos=True, trace=True)
        eb = dev.encode_text(tok)
    finally:
        dev.close()
    assert np.array_equal(ea, eb)
    assert np.array_equal(a.codes[0], b.codes[0]) and np.array_equal(a.hidden, b.hidden)
    print(f"preamble MFMA == VALU ({weights}): encoder, {len(a.codes[0])} frames, hidden bitwise; "
          f"preamble {a.preamble_ms:.2f} ms (MFMA) vs {b.preamble_ms:.2f} ms (VALU)")


# ---------------------------------------------------------------- moved special ids
# A GGUF may put the 8 special audio ids anywhere (magpie.audio_bos_id, EOS = bos + 1):
# the pick then takes its general per-row mask (wave_pick_v / wave_pick_rows) instead
# of the last-row fast path of the reference's ids (2016..2023).
MOVED_BOS = 1000


@pytest.fixture(scope="module")
def moved_ids_model():
    import os
    import magpie_amd as ma
    cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
    os.makedirs(cache, exist_ok=True)
    return ma.synth_gguf(os.path.join(cache, f"magpie_small_bos{MOVED_BOS}_k32.gguf"), dec_layers=2, enc_layers=1,
                         lt_head_scale=ma.DECISIVE, audio_bos=MOVED_BOS)


@pytest.fixture(scope="module")
def moved_ids_eos_model():
    import os
    import magpie_amd as ma
    cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
    os.makedirs(cache, exist_ok=True)
    return ma.synth_gguf(os.path.join(cache, f"magpie_small_bos{MOVED_BOS}_eos.gguf"), dec_layers=2, enc_layers=1,
                         audio_bos=MOVED_BOS, eos_bias=8.0)


def _no_special(codes, eos_ok=False):
    c = np.asarray(codes).reshape(-1)
    bad = [(MOVED_BOS <= v < MOVED_BOS + 8) and not (eos_ok and v == MOVED_BOS + 1) for v in c]
    assert not any(bad), f"special id emitted: {c[np.array(bad)]}"


def test_moved_special_ids_greedy(ma, oracle, moved_ids_model):
    """Greedy f32 at batch 1 (the pick split over 4 waves) and at batch 3 (one wave per
    slot) with the special ids at 1000..1007: codes equal the oracle's, no special id
    emitted, the batch equals its single runs."""
    tok = ma.synthetic_tokens(20, seed=1300)
    r, o = _run_both(ma, oracle, moved_ids_model, tok, steps=32, ignore_eos=True)
    compare_codes(r.codes[0], o["codes"], o["margins"])
    _no_special(r.codes[0])
    toks = [ma.synthetic_tokens(12 + 4 * b, seed=1310 + b) for b in range(3)]
    dev = ma.Device(moved_ids_model)
    rb = dev.synthesize(toks, speakers=[0, 1, 2], max_dec_steps=16, ignore_eos=True)
    for b in range(3):
        rs = dev.synthesize([toks[b]], speakers=[b], max_dec_steps=16, ignore_eos=True)
        assert np.array_equal(rb.codes[b], rs.codes[0]), b
        _no_special(rb.codes[b])
    dev.close()
    # bf16 mode: the split pick of lt_slot_kernel at 1 and 2 slots
    d16 = ma.Device(moved_ids_model, weights="bf16")
    r2 = d16.synthesize(toks[:2], speakers=[0, 1], max_dec_steps=16, ignore_eos=True)
    r1 = d16.synthesize(toks[:1], speakers=[0], max_dec_steps=16, ignore_eos=True)
    d16.close()
    assert np.array_equal(r2.codes[0], r1.codes[0])
    _no_special(r2.codes[0]); _no_special(r2.codes[1])


def test_moved_special_ids_sampled_and_eos(ma, oracle, moved_ids_model, moved_ids_eos_model):
    """Top-k draws with the moved ids equal the oracle's; with codebook 3's EOS logit
    raised, both stop at frame 4 (EOS forbidden before, magpie.cpp:4340-4348)."""
    toks = [ma.synthetic_tokens(14, seed=1320)]
    r, outs = _sample_both(ma, oracle, moved_ids_model, toks, steps=20, temperature=0.7, top_k=80, seed=31,
                           ignore_eos=True)
    compare_codes(r.codes[0], outs[0]["codes"], outs[0]["margins"])
    _no_special(r.codes[0])
    for temp in (0.0, 0.7):
        dev = ma.Device(moved_ids_eos_model)
        re_ = dev.synthesize(toks, max_dec_steps=64, temperature=temp, top_k=80, seed=5)
        dev.close()
        om = oracle.Model(moved_ids_eos_model)
        oe = om.synthesize(toks[0], max_steps=64, trace=False, temperature=temp, top_k=80, seed=5, stream=0)
        om.close()
        assert oe["n_frames"] == 4 and re_.n_frames[0] == 4, (temp, oe["n_frames"], re_.n_frames[0])
        # default (near-flat) heads here: a genuine near-tie may end the comparison early
        compare_codes(re_.codes[0], oe["codes"], oe["margins"], min_frames=0)


@pytest.mark.parametrize("which", ["decisive", "default_heads", "moved_ids", "moved_ids_eos", "eos"])
def test_lt_all_equals_launch_sequence(ma, oracle, request, which):
    """f32 batch 1, greedy: the whole local transformer of a frame in one launch (lt_all_kernel,
    MAGPIE_LT_ALL=1, opt-in: measured slower; FFN merges, heads and picks through in-launch
    granules, the pick from the 64 workgroups' masked first-max keys with EOS in its own slot)
    computes the same codes and hidden states bit for bit as the launch sequence (MAGPIE_LT_ALL=0,
    the default: the front, then 7 x {lt_ffn2, lt_e} and lt_e), and they equal the oracle's: the reference's special ids,
    moved ids (the general mask), near-flat heads (near-ties) and EOS live."""
    import os
    path = {"decisive": "small_model", "default_heads": "full_model_default_heads", "moved_ids": "moved_ids_model",
            "moved_ids_eos": "moved_ids_eos_model", "eos": "eos_model"}[which]
    path = request.getfixturevalue(path)
    ignore = which in ("decisive", "default_heads", "moved_ids")
    steps = 24 if which == "default_heads" else 40
    tok = ma.synthetic_tokens(20, seed=2400)
    runs = {}
    for mode in ("0", "1"):
        os.environ["MAGPIE_LT_ALL"] = mode
        try:
            dev = ma.Device(path)
            runs[mode] = dev.synthesize([tok], speakers=[2], max_dec_steps=steps, ignore_eos=ignore, trace=True)
            dev.close()
        finally:
            os.environ.pop("MAGPIE_LT_ALL", None)
    a, b = runs["0"], runs["1"]
    assert int(a.n_frames[0]) == int(b.n_frames[0])
    np.testing.assert_array_equal(a.codes[0], b.codes[0])
    n = int(b.n_frames[0])
    assert np.array_equal(a.hidden[0, :n + 1], b.hidden[0, :n + 1])
    om = oracle.Model(path)
    o = om.synthesize(tok, speaker=2, max_steps=steps, ignore_eos=ignore, trace=True)
    om.close()
    compare_codes(b.codes[0], o["codes"], o["margins"], min_frames=min(len(o["codes"]), 4))
    print(f"{which}: {n} frames, one-launch LT == launch sequence bit for bit")


@pytest.mark.parametrize("which", ["decisive", "default_heads", "moved_ids", "moved_ids_eos", "eos"])
def test_lt_head_candidates_equal_logit_scan(ma, oracle, request, which):
    """f32 batch 1, greedy: the LT step picks codebook c-1's code from the head's ~253
    workgroup candidates (each head workgroup's masked first-max as an ordered key, EOS in
    its own slot, dropped while step < 4 or ignore_eos; MAGPIE_LT_CAND=1, opt-in: measured
    slower) instead of scanning the 2024 logits (MAGPIE_LT_CAND=0, the default). Same codes and hidden states
    bit for bit, and equal to the oracle, with the reference's special ids, with the ids
    moved (the general mask), near-flat heads (many near-ties) and EOS live."""
    import os
    path = {"decisive": "small_model", "default_heads": "full_model_default_heads", "moved_ids": "moved_ids_model",
            "moved_ids_eos": "moved_ids_eos_model", "eos": "eos_model"}[which]
    path = request.getfixturevalue(path)
    ignore = which in ("decisive", "default_heads", "moved_ids")
    steps = 24 if which == "default_heads" else 40
    tok = ma.synthetic_tokens(20, seed=2300)
    runs = {}
    for mode in ("0", "1"):
        os.environ["MAGPIE_LT_CAND"] = mode
        try:
            dev = ma.Device(path)
            runs[mode] = dev.synthesize([tok], speakers=[1], max_dec_steps=steps, ignore_eos=ignore, trace=True)
            dev.close()
        finally:
            os.environ.pop("MAGPIE_LT_CAND", None)
    a, b = runs["0"], runs["1"]
    assert int(a.n_frames[0]) == int(b.n_frames[0])
    np.testing.assert_array_equal(a.codes[0], b.codes[0])
    n = int(b.n_frames[0])
    assert np.array_equal(a.hidden[0, :n + 1], b.hidden[0, :n + 1])
    om = oracle.Model(path)
    o = om.synthesize(tok, speaker=1, max_steps=steps, ignore_eos=ignore, trace=True)
    om.close()
    compare_codes(b.codes[0], o["codes"], o["margins"], min_frames=min(len(o["codes"]), 4))
    print(f"{which}: {n} frames, candidate pick == logit scan bit for bit")
