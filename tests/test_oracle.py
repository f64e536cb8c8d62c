"""CPU tests: the oracle against hand-derived known answers and against the committed golden
fixtures (tests/golden/make_golden.py), plus host-side logic. No GPU needed."""
import os

import numpy as np
import pytest

from oracle import ctr as OC
from oracle import embedding as OE
from oracle import interaction as OI

GOLD = os.path.join(os.path.dirname(__file__), "golden")


# ---- known-answer tests ----
def test_dot_interaction_known_answer():
    x = np.array([[[1., 2.], [3., 4.], [5., 6.]]])
    # Z = [[5,11,17],[11,25,39],[17,39,61]]
    np.testing.assert_array_equal(OI.dot_interaction(x, False, False), [[11, 17, 39]])
    np.testing.assert_array_equal(OI.dot_interaction(x, True, False), [[5, 11, 25, 17, 39, 61]])
    np.testing.assert_array_equal(OI.dot_interaction(x, False, True), [[0, 11, 17, 0, 0, 39, 0, 0, 0]])
    np.testing.assert_array_equal(OI.dot_interaction(x, True, True), [[5, 0, 0, 11, 25, 0, 17, 39, 61]])


def test_dot_interaction_bwd_finite_difference(rng):
    x = rng.standard_normal((2, 5, 3))
    for si in (False, True):
        for sg in (False, True):
            g = rng.standard_normal(OI.dot_interaction(x, si, sg).shape)
            gx = OI.dot_interaction_bwd(x, g, si, sg)
            eps = 1e-6
            num = np.zeros_like(x)
            for idx in np.ndindex(*x.shape):
                xp = x.copy(); xp[idx] += eps
                xm = x.copy(); xm[idx] -= eps
                num[idx] = ((OI.dot_interaction(xp, si, sg) - OI.dot_interaction(xm, si, sg)) * g).sum() / (2 * eps)
            np.testing.assert_allclose(gx, num, rtol=1e-5, atol=1e-7)


def test_fm_identity(rng):
    e = rng.standard_normal((4, 6, 3))
    pair = sum((e[:, i] * e[:, j]).sum(-1) for i in range(6) for j in range(i + 1, 6))
    np.testing.assert_allclose(OI.fm(e), pair, rtol=1e-12)


def test_adam_closed_form_first_step():
    # step 1: m = (1-b1) g, v = (1-b2) g^2, lr_t = lr*sqrt(1-b2)/(1-b1) → update = lr*sign(g) (eps small)
    c = OE.keras_adam_coefficients(1)
    w = np.zeros((3, 2), np.float32)
    g = np.array([[0.5, -2.0]], np.float32)
    w2, m2, v2 = OE.apply_lazy_adam(w, w.copy(), w.copy(), np.array([1]), g, c)
    np.testing.assert_allclose(w2[1], -1e-3 * np.sign(g[0]), rtol=1e-4)
    assert (w2[0] == 0).all() and (w2[2] == 0).all()
    w3, m3, v3 = OE.apply_keras_adam(w, w.copy(), w.copy(), np.array([1]), g, c)
    np.testing.assert_array_equal(w3, w2)


def test_segment_sum_order_is_tiled_then_grouped():
    # one row repeated 70 times: tiles of 32 → pieces of 32, 32, 6 inside one aligned group
    n = 70
    g = (np.arange(n, dtype=np.float32) * 0.1 + 1e-3).reshape(n, 1)
    rows, pos = np.zeros(n, np.uint32), np.arange(n, dtype=np.int32)
    _, out = OE.segment_sum_tiled(rows, pos, g, 10)
    p = [np.float32(0)] * 3
    for k in range(n):
        p[k // 32] = np.float32(p[k // 32] + g[k, 0])
    ref = np.float32(np.float32(p[0] + p[1]) + p[2])
    assert out[0, 0] == ref


def test_sort_ids_stable_and_oob():
    ids = np.array([5, 3, 5, 99, 3, 5])
    sr, sp, nu = OE.sort_ids(ids, 10)
    np.testing.assert_array_equal(sr, [3, 3, 5, 5, 5, 10])
    np.testing.assert_array_equal(sp, [1, 4, 0, 2, 5, 3])
    assert nu == 2


def test_oob_semantics():
    t = np.arange(6, dtype=np.float32).reshape(3, 2)
    with pytest.raises(IndexError):
        OE.embedding_lookup(t, np.array([0, 3]))
    np.testing.assert_array_equal(OE.embedding_lookup(t, np.array([0, 3]), raise_oob=False), [[0, 1], [0, 0]])


def test_dlrm_step_oracle_reduces_loss(rng):
    from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

    cards = criteo_cardinalities(20_000, 26)
    so = np.concatenate([[0], np.cumsum(cards)]).astype(np.int64)
    D = 8

    def mk(units, fin):
        out = []
        for u in units:
            lim = np.sqrt(6.0 / (fin + u))
            out.append((rng.uniform(-lim, lim, (fin, u)).astype(np.float32), np.zeros(u, np.float32)))
            fin = u
        return out

    st = OC.DLRMState(rng.uniform(-0.05, 0.05, (sum(cards), D)).astype(np.float32), so,
                      mk([16, D], 13), mk([16, 1], 27 * 27 + D))
    r = np.random.default_rng(0)
    batch = criteo_batch(r, 256, cards)
    l0 = OC.dlrm_sgd_step(st, *batch, 0.5)
    for _ in range(20):
        l1 = OC.dlrm_sgd_step(st, *batch, 0.5)
    assert l1 < l0


# ---- golden fixtures ----
def test_golden_embedding():
    f = np.load(os.path.join(GOLD, "embedding.npz"))
    so, ids, table, grad = f["slot_offsets"], f["ids"], f["table"], f["grad"]
    V = int(so[-1])
    np.testing.assert_array_equal(OE.embedding_lookup(table, ids, so, raise_oob=False), f["emb"])
    sr, sp, nu = OE.sort_ids(ids, V, so)
    np.testing.assert_array_equal(sr, f["sorted_rows"])
    np.testing.assert_array_equal(sp, f["sorted_pos"])
    assert nu == int(f["n_unique"])
    ur, ug = OE.segment_sum_tiled(sr, sp, grad, V)
    np.testing.assert_array_equal(ur, f["uniq_rows"])
    np.testing.assert_array_equal(ug, f["uniq_grad"])
    np.testing.assert_array_equal(OE.apply_sgd(table, ur, ug, np.float32(0.05)), f["sgd"])
    c = OE.keras_adam_coefficients(1)
    z = np.zeros_like(table)
    for name, fn in (("lazy", OE.apply_lazy_adam), ("keras", OE.apply_keras_adam)):
        w, m, v = fn(table, z, z, ur, ug, c)
        np.testing.assert_array_equal(w, f[f"{name}_w"])
        np.testing.assert_array_equal(m, f[f"{name}_m"])
        np.testing.assert_array_equal(v, f[f"{name}_v"])


def test_golden_interaction():
    f = np.load(os.path.join(GOLD, "interaction.npz"))
    x = f["x"]
    for si in (0, 1):
        for sg in (0, 1):
            np.testing.assert_allclose(OI.dot_interaction(x, bool(si), bool(sg)), f[f"z_{si}{sg}"], rtol=1e-12)
            np.testing.assert_allclose(OI.dot_interaction_bwd(x, f[f"g_{si}{sg}"], bool(si), bool(sg)),
                                       f[f"gx_{si}{sg}"], rtol=1e-12)
    np.testing.assert_allclose(OI.fm(f["fm_e"]), f["fm_out"], rtol=1e-12)
    np.testing.assert_allclose(OI.fm_bwd(f["fm_e"], f["fm_g"]), f["fm_ge"], rtol=1e-12)


def test_deepfm_oracle_fm_pairs_and_table_gradient():
    """oracle/ctr.py DeepFM: the FM term is the sum of the distinct pair dot products
    (ctr/model.py:21-23), and the table gradient rows match float64 finite differences of the
    mean BCE loss."""
    from oracle.ctr import bce, deepfm_forward, deepfm_keras_adam_step

    rng = np.random.default_rng(0)
    V, D, B, S = 40, 4, 6, 5
    t = rng.standard_normal((V, D)).astype(np.float32) * 0.3
    cat = rng.integers(0, V, (B, S))
    dn = rng.standard_normal((B, 3)).astype(np.float32)
    y = (rng.random(B) < 0.5).astype(np.float32)
    layers = [(rng.standard_normal((S * D + 3, 7)).astype(np.float32) * 0.1, np.zeros(7, np.float32)),
              (rng.standard_normal((7, 1)).astype(np.float32) * 0.1, np.full(1, 0.1, np.float32))]
    p, c = deepfm_forward(t, cat, dn, layers)
    e = t[cat].astype(np.float64)
    fm = sum((e[:, i] * e[:, j]).sum(1) for i in range(S) for j in range(i + 1, S))
    np.testing.assert_allclose(c["logit"], fm + c["cache"][-1][:, 0], rtol=1e-5, atol=1e-6)
    zeros = [(np.zeros_like(k), np.zeros_like(b)) for k, b in layers]
    _, _, det = deepfm_keras_adam_step(t, np.zeros_like(t), np.zeros_like(t), layers, zeros, zeros,
                                       cat, dn, y, 1)
    b0, s0 = 2, 3
    h = 1e-3
    t64 = t.astype(np.float64)

    def loss_at(delta):
        tt = t64.copy()
        tt[cat[b0, s0], 1] += delta
        pp, _ = deepfm_forward(tt, cat, dn.astype(np.float64), [(k.astype(np.float64), bb.astype(np.float64)) for k, bb in layers])
        return bce(y.astype(np.float64), pp).mean()

    fd = (loss_at(h) - loss_at(-h)) / (2 * h)
    # the row's gradient is the sum over every position that looks it up
    occ = np.flatnonzero(cat.reshape(-1) == cat[b0, s0])
    got = det["dx"][occ, 1].astype(np.float64).sum()
    np.testing.assert_allclose(got, fd, rtol=2e-3, atol=1e-7)
