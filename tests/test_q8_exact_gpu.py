"""Q8_0 / Q4_0 integer work, bit for bit.

ggml multiplies a Q8_0 / Q4_0 weight by quantising the activation row to Q8_0
(quantize_row_q8_0: d = amax/127 rounded to fp16, q = roundf(x / d)) and summing, per
32-block, the exact integer dot times d_w * d_a (ggml_vec_dot_q8_0_q8_0 /
vec_dot_q4_0_q8_0; the blocks as the reference converter writes them,
scripts/convert_magpie_to_gguf.py:79-138). Both halves before the f32 sum are integer
work, so given the same f32 input row they must agree exactly, not within a tolerance.

With MAGPIE_Q8DUMP=1 every int8-MFMA decode GEMM launch of the iteration (QKV, the
O-projection, the cross-attention q_net with MAGPIE_Q8_UNFUSED=1, the LT in_proj, the LT
q|k|v at position 0 and the 8 heads) writes the f32 rows its prologue built, the Q8_0
blocks it quantised them to, and the int32 block dots its MFMAs formed from its weight
fragments (mp_decode_q8.hip, GemvP::q8dump). Here the oracle's quantiser
(oracle/magpie_oracle.c quant_row_q8, the function its Q8_0 mul_mat uses) is fed the
GPU's f32 rows and its integer block dots are formed from the GGUF's own blocks: every
int8, every fp16 d and every int32 dot must be identical. A mis-packed fragment, a wrong
rounding rule or a lost block would show here as a nonzero count, whatever the f32
tolerance downstream."""
import os
import struct

import numpy as np
import pytest

from gguf_raw import GgufRaw

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ma():
    import magpie_amd
    if magpie_amd.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return magpie_amd


def _tensor(name, layer, cb):
    if name in ("qkv", "qkv_sa"):
        return f"decoder.layers.{layer}.self_attention.qkv_net.weight"
    if name in ("oproj", "oproj_xa_q8"):
        return f"decoder.layers.{layer}.self_attention.o_net.weight"
    if name == "xq":
        return f"decoder.layers.{layer}.cross_attention.q_net.weight"
    if name in ("lt_in0", "lt_inh"):
        return "local_transformer_in_projection.weight"
    if name == "lt_a":
        return "local_transformer.layers.0.self_attention.qkv_net.weight"
    if name in ("lt_b", "lt_bg", "lt_bo"):
        return "local_transformer.layers.0.self_attention.o_net.weight"
    if name == "lt_e":
        return f"local_transformer_out_projections.{cb}.weight"
    raise KeyError(name)


def _records(dev):
    idx = np.frombuffer(dev.debug_bytes("q8dump_index"), np.int32).reshape(-1, 16)
    out = []
    for r in idx:
        name = struct.pack("<10i", *r[6:16]).split(b"\0")[0].decode()
        out.append(dict(N=int(r[0]), K=int(r[1]), NB=int(r[2]), layer=int(r[3]), cb=int(r[4]), off=int(r[5]),
                        name=name))
    return out


def _check_dump(ma, orc, path, B, steps, unfused):
    os.environ["MAGPIE_Q8DUMP"] = "1"
    if unfused:
        os.environ["MAGPIE_Q8_UNFUSED"] = "1"
    try:
        dev = ma.Device(path, weights="q8")
        toks = [ma.synthetic_tokens(20 + 3 * b, seed=2100 + b) for b in range(B)]
        dev.synthesize(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=steps, ignore_eos=True)
        recs = _records(dev)
        blob = dev.debug_bytes("q8dump")
        dev.close()
    finally:
        os.environ.pop("MAGPIE_Q8DUMP", None)
        os.environ.pop("MAGPIE_Q8_UNFUSED", None)
    g = GgufRaw(path)
    seen, n_q, n_d, n_dot = set(), 0, 0, 0
    for r in recs:
        N, K, NB, off = r["N"], r["K"], r["NB"], r["off"]
        nblk = K // 32
        act = np.frombuffer(blob, np.float32, NB * K, off).reshape(NB, K)
        q_gpu = np.frombuffer(blob, np.int8, NB * K, off + NB * K * 4).reshape(NB, K)
        d_gpu = np.frombuffer(blob, np.float32, NB * nblk, off + NB * K * 5).reshape(NB, nblk)
        dots_gpu = np.frombuffer(blob, np.int32, N * nblk * NB, off + NB * K * 5 + NB * nblk * 4).reshape(N, nblk, NB)
        typ, ne, raw = g.raw(_tensor(r["name"], r["layer"], r["cb"]))
        assert typ in (8, 2) and ne == [K, N], (r, typ, ne)
        for b in range(B):
            q_o, d_o = orc.q8_quantize_row(act[b])
            bad_q = np.flatnonzero(q_o != q_gpu[b])
            bad_d = np.flatnonzero(d_o.view(np.uint32) != d_gpu[b].view(np.uint32))
            assert bad_q.size == 0 and bad_d.size == 0, (r, b, bad_q[:8], bad_d[:8])
            dots_o = orc.qblock_dots(raw, typ, N, K, q_gpu[b])
            bad = np.argwhere(dots_o != dots_gpu[:, :, b])
            assert bad.size == 0, (r, b, bad[:8])
            n_q += K
            n_d += nblk
            n_dot += N * nblk
        seen.add(r["name"])
    print(f"{os.path.basename(path)} B={B}: {len(recs)} launches ({sorted(seen)}), {n_q} int8 / {n_d} fp16 d / "
          f"{n_dot} int32 block dots identical")
    return seen


def test_q8_full_model_integer_work_exact(ma, oracle, q8_full_model):
    """Magpie-357M Q8_0 (the shipped shape), batch 1, step 6: every quantised operand and
    block dot of the iteration's int8 GEMMs, fused layer (qkv_sa, oproj_xa_q8)."""
    seen = _check_dump(ma, oracle, q8_full_model, 1, 6, unfused=False)
    assert {"qkv_sa", "oproj_xa_q8", "lt_in0", "lt_a", "lt_e"} <= seen


def test_q8_unfused_xq_and_batch(ma, oracle, q8_model):
    """The separate launches (MAGPIE_Q8_UNFUSED=1) add the cross-attention q_net GEMV; batch 3
    (NB = 4: the padded column reads the zero row, never dumped)."""
    seen = _check_dump(ma, oracle, q8_model, 3, 5, unfused=True)
    assert {"qkv", "oproj", "xq", "lt_in0", "lt_e"} <= seen


def test_q4_integer_work_exact(ma, oracle, q4_model):
    """Q4_0: the nibble fragments' unsigned dot minus 8 x the activation block sum equals
    ggml's (q - 8) integer dot."""
    seen = _check_dump(ma, oracle, q4_model, 1, 4, unfused=False)
    assert "lt_e" in seen
