"""The Q8_0 weight mode's fused launches against its separate ones.

A Q8_0 (or Q4_0) file runs the decoder layer in four launches (up to 8 slots): the
int8 MFMA QKV projection with the self-attention riding in it (EPI_QKV_SA, the
hand-off the f32 and 16-bit families use), the int8 O-projection with the whole
direct Q8_0 cross-attention riding in it (EPI_RESID_XQ8: q_net workgroups on a
hand-off of x1, attention + o_net workgroups on a hand-off of q), then the two F32
FFN convs. MAGPIE_Q8_UNFUSED=1 runs the same arithmetic as seven separate launches
(QKV, sa_attn, O-projection, the q_net GEMV, xa_q8_kernel, FFN); the fused forms must
reproduce them bit for bit: codes and every hidden state, greedy and sampled, at
every batch size, for texts inside the prefetched first 64 keys and beyond them
(T > 64). Agreement with the oracle's Q8_0
mode is checked by tests/test_decode_gpu.py and tests/test_configs_gpu.py on the
default (fused) path.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ma():
    import magpie_amd
    if magpie_amd.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return magpie_amd


def _run(ma, path, toks, unfused, weights="q8", **kw):
    if unfused:
        os.environ["MAGPIE_Q8_UNFUSED"] = "1"
    try:
        dev = ma.Device(path, weights=weights)
        r = dev.synthesize(toks, speakers=[b % 5 for b in range(len(toks))], trace=True, **kw)
        ops = dev.ops()
        dev.close()
    finally:
        os.environ.pop("MAGPIE_Q8_UNFUSED", None)
    return r, ops


@pytest.mark.parametrize("B,T", [(1, 24), (1, 100), (4, 40), (16, 70)])
def test_q8_fused_equals_unfused(ma, q8_model, B, T):
    toks = [ma.synthetic_tokens(T - 3 * b, seed=8100 + b) for b in range(B)]
    kw = dict(max_dec_steps=24, ignore_eos=True)
    rf, ops_f = _run(ma, q8_model, toks, False, **kw)
    ru, ops_u = _run(ma, q8_model, toks, True, **kw)
    assert "xq" in ops_u and "oproj" in ops_u and "xa_q8" in ops_u and "oproj_xa_q8" not in ops_u, sorted(set(ops_u))
    assert "xa" not in ops_f and "xa" not in ops_u  # no reassociated-XA launch in the Q8_0 mode
    if B < 16:  # (16 slots keep the separate launches)
        assert "oproj_xa_q8" in ops_f and "xq" not in ops_f and "xa_q8" not in ops_f, sorted(set(ops_f))
        assert "qkv_sa" in ops_f and "sa_attn" not in ops_f
    print(f"B={B} T={T}: {len(ops_f)} launches per iteration fused, {len(ops_u)} unfused")
    for b in range(B):
        assert np.array_equal(rf.codes[b], ru.codes[b]), f"slot {b} codes"
        assert np.array_equal(rf.hidden[b], ru.hidden[b]), f"slot {b} hidden"


def test_q8_fused_sampled_equals_unfused(ma, q8_model):
    toks = [ma.synthetic_tokens(30 + 4 * b, seed=8200 + b) for b in range(3)]
    kw = dict(max_dec_steps=32, temperature=0.7, top_k=80, seed=5, ignore_eos=True)
    rf, _ = _run(ma, q8_model, toks, False, **kw)
    ru, _ = _run(ma, q8_model, toks, True, **kw)
    for b in range(3):
        assert np.array_equal(rf.codes[b], ru.codes[b]) and np.array_equal(rf.hidden[b], ru.hidden[b]), b


def test_q4_fused_equals_unfused(ma, q4_model):
    toks = [ma.synthetic_tokens(20, seed=8300)]
    rf, _ = _run(ma, q4_model, toks, False, weights="q4", max_dec_steps=16, ignore_eos=True)
    ru, _ = _run(ma, q4_model, toks, True, weights="q4", max_dec_steps=16, ignore_eos=True)
    assert np.array_equal(rf.codes[0], ru.codes[0]) and np.array_equal(rf.hidden, ru.hidden)


def test_q8_full_model_fused_equals_unfused(ma, q8_full_model):
    toks = [ma.synthetic_tokens(64, seed=1000)]
    rf, _ = _run(ma, q8_full_model, toks, False, max_dec_steps=32, ignore_eos=True)
    ru, _ = _run(ma, q8_full_model, toks, True, max_dec_steps=32, ignore_eos=True)
    assert np.array_equal(rf.codes[0], ru.codes[0]) and np.array_equal(rf.hidden, ru.hidden)


@pytest.mark.parametrize("B", [1, 16])
def test_q4_nibbles_equal_int8_repack(ma, q4_model, B):
    """A Q4_0 file's decode projections stream their nibbles (pack_q4: 18 B per 32
    weights, as in the file, convert_magpie_to_gguf.py:107-138) and correct the MFMA's
    unsigned-nibble dot by -8 x the activation block sum: the exact integer dot of
    ggml's q - 8 (vec_dot_q4_0_q8_0). MAGPIE_Q4_AS_Q8=1 repacks the same blocks to
    int8 q - 8 (34 B per 32); both must give the same bits, and the nibble form must
    read fewer bytes per op."""
    toks = [ma.synthetic_tokens(20 + 3 * b, seed=8400 + b) for b in range(B)]
    kw = dict(max_dec_steps=16, ignore_eos=True)

    def run(as_q8):
        if as_q8:
            os.environ["MAGPIE_Q4_AS_Q8"] = "1"
        try:
            dev = ma.Device(q4_model, weights="q4")
            r = dev.synthesize(toks, speakers=[b % 5 for b in range(B)], trace=True, **kw)
            names = dev.ops()
            by = {n: dev.op_bytes(i) for i, n in enumerate(names)}
            dev.close()
        finally:
            os.environ.pop("MAGPIE_Q4_AS_Q8", None)
        return r, by

    rn, bn = run(False)
    r8, b8 = run(True)
    for b in range(B):
        assert np.array_equal(rn.codes[b], r8.codes[b]) and np.array_equal(rn.hidden[b], r8.hidden[b]), b
    assert bn["lt_e"] < b8["lt_e"] and bn["qkv" if B == 16 else "qkv_sa"] < b8["qkv" if B == 16 else "qkv_sa"]


def _lt_dump(ma, path, toks, mode, tmp_path, weights="q8"):
    """Eager run with MAGPIE_LTQ8=mode, slot 0's LT state after every LT step
    (MAGPIE_DUMP_LT: the previous head's logits, codes, X, y per record)."""
    dump = str(tmp_path / f"lt_{weights}_{mode}_{len(toks)}.bin")
    env = {"MAGPIE_LTQ8": str(mode), "MAGPIE_EAGER": "1", "MAGPIE_DUMP_LT": dump}
    os.environ.update(env)
    try:
        dev = ma.Device(path, weights=weights)
        r = dev.synthesize(toks, speakers=[b % 5 for b in range(len(toks))], trace=True,
                           max_dec_steps=6, ignore_eos=True)
        dev.close()
    finally:
        for k in env:
            os.environ.pop(k, None)
    rec = np.fromfile(dump, dtype=np.float32).reshape(-1, 2024 + 8 + 4 * 256)
    return r, rec[:, :2024 + 8 + 2 * 256].view(np.uint32)  # (lty2 / ltq are not outputs of every form)


@pytest.mark.parametrize("weights", ["q8", "q4"])
def test_q8_lt_step_forms_equal(ma, q8_model, q4_model, weights, tmp_path):
    """The Q8_0 LT step (lt_slot_q8_kernel) in its three forms -- o_net rows split over the
    workgroups with a y hand-off and the FFN merge in the launch (MAGPIE_LTQ8=0), every
    workgroup all 256 o_net rows from the transposed copy (1), and at batch 1 the FFN
    merge deferred to the Q8_0 head's prologue (2, the default) -- give the same bits:
    every head's logits, the codes, X and y of every LT step, and the decoder hidden."""
    model = q8_model if weights == "q8" else q4_model
    toks = [ma.synthetic_tokens(30, seed=8500)]
    runs = {m: _lt_dump(ma, model, toks, m, tmp_path, weights) for m in (0, 1, 2)}
    r0, d0 = runs[0]
    assert d0.shape[0] >= 8 * 5, d0.shape
    for m in (1, 2):
        r, d = runs[m]
        assert d.shape == d0.shape and np.array_equal(d, d0), f"MAGPIE_LTQ8={m}: LT state differs"
        assert np.array_equal(r.codes[0], r0.codes[0]) and np.array_equal(r.hidden, r0.hidden), m
    # batched: the split and the all-rows o_net forms (the deferred merge is batch 1 only)
    toks4 = [ma.synthetic_tokens(30 + 5 * b, seed=8500 + b) for b in range(4)]
    (ra, da), (rb, db) = (_lt_dump(ma, model, toks4, m, tmp_path, weights) for m in (0, 1))
    assert np.array_equal(da, db)
    for b in range(4):
        assert np.array_equal(ra.codes[b], rb.codes[b]) and np.array_equal(ra.hidden[b], rb.hidden[b]), b
    # and slot 0 of the batch is the single utterance (batch = single across the forms)
    assert np.array_equal(ra.codes[0], r0.codes[0]) and np.array_equal(da[:d0.shape[0]], d0)
