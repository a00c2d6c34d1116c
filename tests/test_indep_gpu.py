"""The HIP path held directly to the INDEPENDENT f64 restatement of the reference
(tests/golden/make_indep.py, fixtures tests/golden/indep_*.npz): a second reading of
src/magpie.cpp / src/nano-codec.cpp that shares no code with the oracle or the
kernels (tests/test_indep_cpu.py holds the oracle to the same fixtures).

Bars: f32 decode (2-layer synthetic model, decisive heads) codes identical to the
restatement at every frame, hidden state after every step within 2e-5 abs (the
decode path's f32 bar, tests/test_decode_gpu.py); codec waveform with f16 MFMA
operands within 1e-2 abs of the f64 restatement (test_codec_gpu.py's bar against
plain f32 operands).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def ma():
    import magpie_amd
    if magpie_amd.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return magpie_amd


def test_gpu_decode_matches_independent_restatement(ma, small_model):
    d = np.load(os.path.join(GOLD, "indep_small.npz"))
    dev = ma.Device(small_model)
    try:
        i = 0
        while f"c{i}_tokens" in d:
            spk, steps = (int(v) for v in d[f"c{i}_meta"])
            r = dev.synthesize([d[f"c{i}_tokens"]], speakers=[spk], max_dec_steps=steps, ignore_eos=False, trace=True)
            ref_codes, ref_hidden = d[f"c{i}_codes"], d[f"c{i}_hidden"]
            assert int(r.n_frames[0]) == len(ref_codes) >= 12
            np.testing.assert_array_equal(r.codes[0], ref_codes)
            nh = len(ref_hidden)
            err = np.abs(r.hidden[0, :nh].astype(np.float64) - ref_hidden).max()
            print(f"case {i}: {len(ref_codes)} frames identical to the f64 restatement, hidden max abs err {err:.2e}")
            assert err < 2e-5
            i += 1
        assert i >= 2
    finally:
        dev.close()


def test_gpu_codec_matches_independent_restatement(ma, codec_model):
    d = np.load(os.path.join(GOLD, "indep_codec.npz"))
    c = ma.Codec(codec_model)
    try:
        g = c.decode(d["codes"]).astype(np.float64)
    finally:
        c.close()
    ref = d["audio"]
    err = np.abs(g - ref).max()
    rel = np.linalg.norm(g - ref) / np.linalg.norm(ref)
    print(f"codec: {ref.size} samples, max abs err {err:.2e}, relative L2 {rel:.2e} vs the f64 restatement")
    assert g.shape == ref.shape
    assert err < 1e-2 and rel < 1e-2


def test_gpu_full_shape_matches_independent_restatement(ma, full_model):
    """Magpie-357M's shape (12 / 6 layers), the bench's T = 64 prompt, 32 frames on the bench's
    f32 batch-1 path: codes identical to the f64 restatement, hidden within the f32 bar."""
    d = np.load(os.path.join(GOLD, "indep_full.npz"))
    spk, steps = (int(v) for v in d["meta"])
    dev = ma.Device(full_model)
    try:
        r = dev.synthesize([d["tokens"]], speakers=[spk], max_dec_steps=steps, ignore_eos=False, trace=True)
    finally:
        dev.close()
    ref_codes, ref_hidden = d["codes"], d["hidden"].astype(np.float64)
    assert int(r.n_frames[0]) == len(ref_codes) == 32
    np.testing.assert_array_equal(r.codes[0], ref_codes)
    err = np.abs(r.hidden[0, :len(ref_hidden)].astype(np.float64) - ref_hidden).max()
    print(f"Magpie-357M: 32 frames identical to the f64 restatement, hidden max abs err {err:.2e}")
    assert err < 2e-5


def test_gpu_codec_32_frame_chunk_matches_independent_restatement(ma, codec_model):
    d = np.load(os.path.join(GOLD, "indep_codec32.npz"))
    c = ma.Codec(codec_model)
    try:
        g = c.decode_chunks(d["codes"][None]).astype(np.float64)[0]
    finally:
        c.close()
    ref = d["audio"].astype(np.float64)
    err = np.abs(g - ref).max()
    rel = np.linalg.norm(g - ref) / np.linalg.norm(ref)
    print(f"codec 32-frame chunk: {ref.size} samples, max abs err {err:.2e}, relative L2 {rel:.2e}")
    assert g.shape == ref.shape
    assert err < 1e-2 and rel < 1e-2
