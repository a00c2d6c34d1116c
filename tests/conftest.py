"""Shared fixtures. GPU tests are marked `gpu`; everything else runs on CPU.

Synthetic GGUFs are generated deterministically from a seed (no weights ship)
into $MAGPIE_CACHE (default /tmp/magpie_amd_cache), outside the repository.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "magpie-tts.cpp_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, REPO)

CACHE = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C-ABI on HIP)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _gguf(name, kind="magpie", **kw):
    import magpie_amd as ma
    os.makedirs(CACHE, exist_ok=True)
    return ma.synth_gguf(os.path.join(CACHE, name), kind=kind, **kw)


# Parity models use decisive LT heads (magpie_amd.DECISIVE): >= 98 % of greedy
# decisions have an oracle top-1/top-2 gap above 1e-2, so code identity is a real
# test, not a run of near-ties.
@pytest.fixture(scope="session")
def small_model():
    """2 decoder layers / 1 encoder layer: same kernels, fast oracle."""
    import magpie_amd as ma
    return _gguf("magpie_small_l2e1_k32.gguf", dec_layers=2, enc_layers=1, lt_head_scale=ma.DECISIVE)


@pytest.fixture(scope="session")
def full_model():
    import magpie_amd as ma
    return _gguf("magpie_357m_f32_k32.gguf", lt_head_scale=ma.DECISIVE)


@pytest.fixture(scope="session")
def full_model_default_heads():
    """Magpie-357M shapes with the survey's default LT head distribution (scale 1.0):
    near-flat logits, so most decisions are close calls (the margin rule's hard case)."""
    return _gguf("magpie_357m_f32.gguf")


@pytest.fixture(scope="session")
def eos_model():
    import magpie_amd as ma
    os.makedirs(CACHE, exist_ok=True)
    path = os.path.join(CACHE, "magpie_small_eos.gguf")
    if not os.path.exists(path):
        import subprocess
        subprocess.run([ma.SYNTH_BIN, "magpie", path, "--dec-layers", "2", "--enc-layers", "1", "--eos-bias", "8"],
                       check=True)
    return path


@pytest.fixture(scope="session")
def q8_model():
    import magpie_amd as ma
    return _gguf("magpie_small_q8_k32.gguf", dtype="q8_0", dec_layers=2, enc_layers=1, lt_head_scale=ma.DECISIVE)


@pytest.fixture(scope="session")
def q4_model():
    import magpie_amd as ma
    return _gguf("magpie_small_q4_k32.gguf", dtype="q4_0", dec_layers=2, enc_layers=1, lt_head_scale=ma.DECISIVE)


@pytest.fixture(scope="session")
def f16_model():
    import magpie_amd as ma
    return _gguf("magpie_small_f16_k32.gguf", dtype="f16", dec_layers=2, enc_layers=1, lt_head_scale=ma.DECISIVE)


@pytest.fixture(scope="session")
def q8_full_model():
    """Magpie-357M shapes, the reference converter's default Q8_0 patterns."""
    import magpie_amd as ma
    return _gguf("magpie_357m_q8_k32.gguf", dtype="q8_0", lt_head_scale=ma.DECISIVE)


@pytest.fixture(scope="session")
def codec_model():
    return _gguf("nano_codec.gguf", kind="codec")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as orc
    orc.set_mode(acc64=True, gelu_f16=False, threads=min(16, os.cpu_count() or 1))
    return orc
