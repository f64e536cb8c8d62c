"""CPU checks of the dense-half tolerance model in oracle/check_dlrm.py (no GPU): the fp32 oracle
step's twelve MLP gradients must lie within the stated per-element tolerances of a float64
evaluation of the same step, and a 1 % error in one batch-deep sum (A_top = Σ_b h_b·G_b, the
factored backward's operand) must exceed them — so the GPU check can fail."""
import numpy as np

from oracle.check_dlrm import dense_half_tolerances
from oracle.ctr import DLRMState, dlrm_sgd_step
from recommender_amd.synthetic import criteo_batch, criteo_cardinalities


def _state(rng, V, D, S, dtype):
    def lay(sizes, n_in):
        out = []
        for n in sizes:
            k = rng.uniform(-1, 1, (n_in, n)) * np.sqrt(6.0 / (n_in + n))
            out.append((k, np.zeros(n)))
            n_in = n
        return out
    F = S + 1
    table = rng.uniform(-0.05, 0.05, (V, D))
    bottom = lay([32, 16, D], 13)
    top = lay([32, 16, 1], F * F + D)
    cast = lambda ls: [(k.astype(dtype), b.astype(dtype)) for k, b in ls]  # noqa: E731
    return table.astype(dtype), cast(bottom), cast(top)


def _run(seed=4, B=512, S=26, D=16, V=20_000):
    rng = np.random.default_rng(seed)
    cards = criteo_cardinalities(V, S)
    cat, dn, lb = criteo_batch(rng, B, cards)
    so = np.concatenate([[0], np.cumsum(cards)]).astype(np.int64)
    out = {}
    for dt in (np.float32, np.float64):
        t, b, tp = _state(np.random.default_rng(7), V, D, S, dt)
        st = DLRMState(t, so, b, tp)
        det = {}
        dlrm_sgd_step(st, cat, dn.astype(dt), lb.astype(dt), 0.01, det)
        out[dt] = det
    return out[np.float32], out[np.float64], B


def _ratio(got, ref, tol):
    worst = 0.0
    for (gk, gb), (rk, rb), (tk, tb) in zip(got, ref, tol):
        for g, r, t in ((gk, rk, tk), (gb, rb, tb)):
            err = np.abs(np.asarray(g, np.float64) - np.asarray(r, np.float64))
            worst = max(worst, float((err / (np.asarray(t).reshape(err.shape) + 1e-38)).max()))
    return worst


def test_dense_half_tolerances_hold_fp32_vs_fp64():
    d32, d64, B = _run()
    top_tol, bot_tol = dense_half_tolerances(d32, B)
    assert _ratio(d32["top_grads"], d64["top_grads"], top_tol) <= 1.0
    assert _ratio(d32["bottom_grads"], d64["bottom_grads"], bot_tol) <= 1.0


def test_dense_half_detects_a_perturbed_batch_sum():
    d32, d64, B = _run()
    top_tol, _ = dense_half_tolerances(d32, B)
    # A_top[i] off by 1 %: dK1[i, :] = A_top[i]·Q1ᵀ moves by 1 % of itself
    dk1 = d32["top_grads"][0][0].copy()
    i = int(np.argmax(np.abs(dk1).sum(1)))
    dk1[i] *= 1.01
    bad = [(dk1, d32["top_grads"][0][1])] + list(d32["top_grads"][1:])
    assert _ratio(bad, d64["top_grads"], top_tol) > 1.0
