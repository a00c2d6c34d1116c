"""The §8e work-queue on the device (world size 1 here; the multi-rank claim logic is
tests/test_dist_cpu.py's gloo test): with EOS live the utterances end at different
frames, the queue regroups them into device batches longest-text first, and every
utterance's codes equal the same utterance decoded alone (batch == single holds for
any grouping)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ma():
    import magpie_amd
    if magpie_amd.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return magpie_amd


def test_queue_equals_single_runs_eos_live(ma):
    import os
    from magpie_amd.dist import device_synth, gather_results, synthesize_queue
    cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
    os.makedirs(cache, exist_ok=True)
    # a small EOS bias: these prompts end at 4..48 frames (oracle: 4 4 48 48 48 5 4 39 17 48)
    eos_model = ma.synth_gguf(os.path.join(cache, "magpie_small_eosb0.09.gguf"), dec_layers=2, enc_layers=1,
                              eos_bias=0.09)
    toks = [ma.synthetic_tokens(8 + 5 * ((7 * i) % 9), seed=1700 + i) for i in range(10)]
    spks = [i % 5 for i in range(10)]
    dev = ma.Device(eos_model)
    mine = synthesize_queue(device_synth(dev, max_dec_steps=48), toks, spks, batch=4)
    got = gather_results(mine, len(toks))
    lens = []
    for i, t in enumerate(toks):
        ref = dev.synthesize([t], speakers=[spks[i]], max_dec_steps=48).codes[0]
        assert np.array_equal(got[i], ref), i
        lens.append(len(ref))
    dev.close()
    print("frames per utterance (EOS live):", lens)
    assert len(set(lens)) >= 3, lens  # the queue really regrouped unequal lengths
