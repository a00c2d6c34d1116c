"""f32 parity over the reference's whole decode range on Magpie-357M shapes.

The reference decodes up to max_dec_steps = 500 frames (src/magpie.h:76) into a
cache of max_seq = context_frames + max_dec_steps + 16 rows
(src/magpie.cpp:4077), so keys run up to L = 610 and decoder position row 609 is
read (magpie.cpp:4321-4358). These tests run the 12-layer model to the bench's
length (256 frames, L to 366) and to that limit (500 frames, L to 610) and check
every frame against the oracle (acc64): codes bit-identical over every frame
(parity.compare_codes with min_frames = all) and the decoder's final hidden state
within 2e-5 at every step. Also here: configs[0]'s own prompt "Hello, world!"
through the 12-layer model with the EOS rules live, bf16 batch 16 teacher forced
over 256 frames, and the two batch-state cases of round 2's review (a device
reused across cross-attention forms; an EOS-stopped slot's hidden trace).
"""
import numpy as np
import pytest

from parity import compare_codes, compare_forced

pytestmark = pytest.mark.gpu

HIDDEN_TOL = 2e-5  # f32 path vs the acc64 oracle: measured 1.9e-6 .. 2.3e-6 over 256 / 500 frames
# (the reference's own full-decoder tolerance vs ggml is 2.66e-3, docs/STATUS.md:108-116: this bar is
# ~100x tighter, so an f32 arithmetic regression cannot hide under it)
TIE_EPS = 3e-2     # bf16 near-tie bar (tests/test_decode_gpu.py, the oracle's own f32/f64 spread)
# over configs[2]'s whole 256-frame utterance on 12 layers the oracle's own bf16-mode f32/f64
# spread is ~0.09 (margins shift up to 0.0915, a decision of margin 0.060 flips:
# tests/test_oracle_cpu.py::test_bf16_mode_spread_full_model_256, tools_dev/bf16_spread.py)
BF16_LONG_TIE_EPS = 0.1
HIDDEN_TOL16, HIDDEN_REL16 = 3e-2, 5e-3


@pytest.fixture(scope="module")
def ma():
    import magpie_amd
    if magpie_amd.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return magpie_amd


def _f32_vs_oracle(ma, oracle, path, tok, steps, ignore_eos=True, speaker=0):
    dev = ma.Device(path)
    r = dev.synthesize([tok], speakers=[speaker], max_dec_steps=steps, ignore_eos=ignore_eos, trace=True)
    dev.close()
    om = oracle.Model(path)
    o = om.synthesize(tok, speaker=speaker, max_steps=steps, ignore_eos=ignore_eos, trace=True)
    om.close()
    return r, o


def _check_every_step(r, o):
    res = compare_codes(r.codes[0], o["codes"], o["margins"])  # min_frames: every frame the oracle produced
    n = int(r.n_frames[0])
    assert n == o["n_frames"], (n, o["n_frames"])
    err_step = np.abs(r.hidden[0, :n + 1] - o["hidden"][:n + 1]).max(axis=1)
    worst = int(err_step.argmax())
    print(f"hidden max abs err {err_step.max():.3g} (step {worst}), mean over steps {err_step.mean():.3g}")
    assert err_step.max() < HIDDEN_TOL, f"hidden err {err_step.max()} at step {worst}"
    return res


@pytest.mark.timeout(600)
@pytest.mark.parametrize("steps", [256, 500])
def test_f32_full_range_matches_oracle(ma, oracle, full_model, steps):
    """256 = the bench's utterance (L = 111..366); 500 = max_dec_steps (L to 610)."""
    tok = ma.synthetic_tokens(64, seed=1000)
    r, o = _f32_vs_oracle(ma, oracle, full_model, tok, steps)
    assert r.n_frames[0] == steps
    res = _check_every_step(r, o)
    assert res["identical"] and res["frames"] == steps
    print(f"identical over {steps} frames, keys up to L = {110 + steps}")


@pytest.mark.timeout(600)
def test_hello_world_full_model_with_eos(ma, oracle, full_model):
    """configs[0]'s prompt, tokenized by the C++ front end, through the 12-layer
    model with the reference's EOS rules (forbidden for 4 frames, stop on EOS in any
    codebook's sample or argmax, magpie.cpp:4320-4358), up to max_dec_steps = 500."""
    tok = np.asarray(ma.Tokenizer(full_model)("Hello, world!"), np.int32)
    assert 8 <= len(tok) <= 24, len(tok)
    r, o = _f32_vs_oracle(ma, oracle, full_model, tok, 500, ignore_eos=False)
    _check_every_step(r, o)
    print(f"T = {len(tok)} tokens, {int(r.n_frames[0])} frames")


@pytest.mark.timeout(600)
def test_bf16_batch16_teacher_forced_256(ma, oracle, full_model):
    """configs[2]'s shape over the bench's whole utterance: slot 0 of a bf16 batch of
    16, every one of its 256 x 8 decisions against the oracle's bf16 mode conditioned
    on the GPU's codes, and a middle and the last slot equal to their single runs."""
    B, steps = 16, 256
    toks = [ma.synthetic_tokens(64, seed=1000 + b) for b in range(B)]
    spk = [b % 5 for b in range(B)]
    dev = ma.Device(full_model, weights="bf16")
    rb = dev.synthesize(toks, speakers=spk, max_dec_steps=steps, ignore_eos=True, trace=True)
    assert (rb.n_frames == steps).all()
    for b in (7, B - 1):
        rs = dev.synthesize([toks[b]], speakers=[spk[b]], max_dec_steps=steps, ignore_eos=True, trace=True)
        assert np.array_equal(rb.codes[b], rs.codes[0]), f"slot {b} codes"
        assert np.array_equal(rb.hidden[b], rs.hidden[0]), f"slot {b} hidden"
    dev.close()
    om = oracle.Model(full_model)
    om.set_weight_mode(1)
    o = om.synthesize_forced(toks[0], rb.codes[0], speaker=spk[0], ignore_eos=True)
    om.close()
    res = compare_forced(rb.codes[0], o, tie_eps=BF16_LONG_TIE_EPS, max_ties=steps * 8 // 40)
    print(f"bf16 slot 0: {res}")
    assert res["decisions"] == steps * 8
    h, ho = rb.hidden[0, :steps + 1], o["hidden"]
    live = np.linalg.norm(ho, axis=-1) > 0  # rows the forced run computed (BOS .. last input frame)
    assert live.sum() >= steps, live.sum()
    h, ho = h[live], ho[live]
    err = np.abs(h - ho).max()
    rel = (np.linalg.norm(h - ho, axis=-1) / np.linalg.norm(ho, axis=-1)).max()
    print(f"bf16 slot 0 hidden: max abs {err:.3g}, max rel L2 {rel:.3g}")
    assert err < HIDDEN_TOL16 and rel < HIDDEN_REL16, (err, rel)


@pytest.mark.timeout(600)
def test_f32_default_heads_every_decision_teacher_forced(ma, oracle, full_model_default_heads):
    """The 12-layer model with the survey's default LT head scale (1.0, no decisive
    heads): the logits are near-flat, so a free-running comparison would end at the
    first close call. Every one of the 256 x 8 decisions is checked against the oracle
    (acc64) teacher forced along the GPU's own codes: a decision may differ only where
    the oracle's top-1/top-2 margin is below the f32 tie bar (2e-4; the GPU's f32
    logit error is ~1e-6), and the hidden state stays within 2e-5 at every step."""
    steps = 256
    tok = ma.synthetic_tokens(64, seed=1000)
    dev = ma.Device(full_model_default_heads)
    r = dev.synthesize([tok], speakers=[0], max_dec_steps=steps, ignore_eos=True, trace=True)
    dev.close()
    assert r.n_frames[0] == steps
    om = oracle.Model(full_model_default_heads)
    o = om.synthesize_forced(tok, r.codes[0], speaker=0, ignore_eos=True)
    om.close()
    res = compare_forced(r.codes[0], o)  # parity.TIE_EPS = 2e-4
    m = np.asarray(o["margins"])
    print(f"default heads: {res['decisions']} decisions, {res['differences']} differ (all near-ties); "
          f"{int((m < 1e-2).sum())} decisions have an oracle margin < 1e-2, {int((m < 2e-4).sum())} < 2e-4")
    assert res["decisions"] == steps * 8
    err = np.abs(r.hidden[0, :steps] - o["hidden"][:steps]).max(axis=1)
    print(f"hidden max abs err {err.max():.3g} (step {int(err.argmax())})")
    assert err.max() < HIDDEN_TOL


def test_device_reused_across_xa_forms(ma, small_model):
    """One Device running batches whose cross-attention forms differ (AUTO: direct
    above 160 text tokens, reassociated below; then forced forms): every batch
    equals the same batch on a fresh Device bit for bit."""
    long_tok, short_tok = ma.synthetic_tokens(200, seed=77), ma.synthetic_tokens(100, seed=78)
    kw = dict(max_dec_steps=10, ignore_eos=True, trace=True)

    def fresh(tok, xa):
        d = ma.Device(small_model, xa=xa)
        r = d.synthesize([tok], **kw)
        d.close()
        return r

    dev = ma.Device(small_model)  # auto
    for tok in (long_tok, short_tok, long_tok):
        r = dev.synthesize([tok], **kw)
        f = fresh(tok, "auto")
        assert np.array_equal(r.codes[0], f.codes[0]) and np.array_equal(r.hidden, f.hidden)
    dev.close()
    for first, second in (("direct", "reassoc"), ("reassoc", "direct")):
        dev = ma.Device(small_model, xa=first)
        dev.synthesize([short_tok], **kw)
        dev.lib.mp_hip_set_xa_mode(dev.h, ma.Device.XA_MODES[second])
        r = dev.synthesize([short_tok], **kw)
        dev.close()
        f = fresh(short_tok, second)
        assert np.array_equal(r.codes[0], f.codes[0]) and np.array_equal(r.hidden, f.hidden), (first, second)


@pytest.mark.parametrize("max_steps", [5, 6, 7, 64])
def test_eos_stopped_slot_hidden_matches_oracle(ma, oracle, eos_model, max_steps):
    """A slot that stops on EOS keeps running with the batch until the host's next
    poll (every 8 frames) or the max_dec_steps-th iteration; its hidden trace must
    still be the oracle's up to and including the state that produced the EOS frame
    (row n_frames). eos_model stops at frame 4 (iteration 5): max_steps 5 runs no
    iteration after the stop, 6 exactly one (the iteration must already get the
    slot's frozen input, not the last FFN output), 7 two, 64 three (poll at 8)."""
    toks = [ma.synthetic_tokens(16, seed=7), ma.synthetic_tokens(12, seed=9)]
    dev = ma.Device(eos_model)
    r = dev.synthesize(toks, speakers=[0, 1], max_dec_steps=max_steps, trace=True)
    dev.close()
    om = oracle.Model(eos_model)
    for b in range(2):
        o = om.synthesize(toks[b], speaker=b, max_steps=max_steps, trace=True)
        n = int(r.n_frames[b])
        assert n == o["n_frames"] and n < 8, (n, o["n_frames"])  # stopped before the first poll
        compare_codes(r.codes[b], o["codes"], o["margins"])
        err = np.abs(r.hidden[b, :n + 1] - o["hidden"][:n + 1]).max()
        print(f"max_steps {max_steps} slot {b}: {n} frames, hidden max abs err {err:.3g}")
        assert err < HIDDEN_TOL, f"slot {b}: hidden err {err} over rows 0..{n}"
    om.close()
