"""Helpers for GPU-vs-oracle code parity at temperature 0.

Codes must be bit-identical. The one admissible deviation is a genuine near-tie:
if the first differing codebook decision is one where the oracle's top-1/top-2
logit gap is below TIE_EPS, the f32 GPU and the f64-accumulating oracle may
legitimately pick different argmaxes; the comparison then stops there (the
trajectories diverge afterwards by construction) and reports it.
"""
import numpy as np

TIE_EPS = 2e-4  # logit units; GPU f32 vs oracle f64 logit error is ~1e-6


def compare_codes(gpu_codes, orc_codes, orc_margins, tie_eps=TIE_EPS, min_frames=None):
    """Returns {"identical", "frames" (frames compared before the first difference),
    "decisions"}. min_frames: the comparison must cover at least that many frames
    (None: every frame the oracle produced), so a near-tie in an early frame cannot
    make a test pass vacuously."""
    g = np.asarray(gpu_codes)
    o = np.asarray(orc_codes)
    n = min(len(g), len(o))
    need = len(o) if min_frames is None else min_frames
    diff = np.argwhere(g[:n] != o[:n])
    if len(diff) == 0:
        assert len(g) == len(o), f"frame counts differ: gpu {len(g)} vs oracle {len(o)}"
        print(f"codes identical over {n} frames ({n * 8} decisions)")
        assert n >= need, f"only {n} frames compared, {need} required"
        return {"identical": True, "frames": n, "decisions": n * 8}
    f, cb = diff[0]
    margin = float(orc_margins[f, cb])
    assert margin < tie_eps, (f"codes differ at frame {f} cb {cb}: gpu {g[f].tolist()} oracle {o[f].tolist()} "
                              f"with oracle margin {margin:.3g} >= {tie_eps}")
    print(f"codes identical over {f} frames, then a near-tie at frame {f} cb {cb} (margin {margin:.3g})")
    assert f >= need, f"near-tie at frame {f}: only {f} frames compared, {need} required"
    return {"identical": False, "frames": int(f), "decisions": int(f) * 8 + int(cb), "tie_margin": margin}


def compare_forced(gpu_codes, forced_orc, tie_eps=TIE_EPS, max_ties=None):
    """Every decision of a GPU run against a teacher-forced oracle run along the GPU's
    own codes (oracle.Model.synthesize_forced): a decision may differ only where the
    oracle's margin is below tie_eps (a genuine near-tie). max_ties bounds how many
    such decisions are tolerated (None: no bound beyond the margin rule)."""
    g = np.asarray(gpu_codes).reshape(-1, 8)
    o = np.asarray(forced_orc["codes"])
    m = np.asarray(forced_orc["margins"])
    assert g.shape == o.shape, f"{g.shape} vs {o.shape}"
    diff = np.argwhere(g != o)
    for f, cb in diff:
        assert m[f, cb] < tie_eps, (f"frame {f} cb {cb}: gpu {g[f, cb]} oracle {o[f, cb]} "
                                    f"with oracle margin {m[f, cb]:.3g} >= {tie_eps}")
    if max_ties is not None:
        assert len(diff) <= max_ties, f"{len(diff)} near-tie decisions, at most {max_ties} expected"
    dm = [float(m[f, c]) for f, c in diff]
    print(f"teacher-forced: {g.size} decisions checked over {len(g)} frames, {len(diff)} near-tie differences"
          f" (margins {[round(v, 5) for v in dm[:4]]}, largest {max(dm) if dm else 0.0:.4g})")
    return {"decisions": int(g.size), "differences": int(len(diff))}
