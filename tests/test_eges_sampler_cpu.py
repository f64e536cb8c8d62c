"""CPU checks of the EGES pair-pipeline oracle (oracle/eges.py) against the documented
behaviour of the three samplers at eges/data_loader.py:28-62 (parity unpinned: DGL / TF are
absent, so these are properties and hand-worked cases, not reference vectors)."""
import numpy as np

from oracle import eges as O
from recommender_amd.eges.sampler import log_uniform_cdf, skipgram_slots
from tests.eges_graph import make_graph


def test_skipgrams_hand_case():
    # keras skipgrams([1, 2, 0, 3], window_size=1, negative_samples=0) minus the shuffle
    tgt, ctx = O.skipgram_pairs(np.array([[1, 2, 0, 3]]), 1)
    assert list(zip(tgt, ctx)) == [(1, 2), (2, 1)]
    tgt, ctx = O.skipgram_pairs(np.array([[4, 5, 6, -1]]), 5)
    assert list(zip(tgt, ctx)) == [(4, 5), (4, 6), (5, 4), (5, 6), (6, 4), (6, 5)]


def test_skipgram_slot_count():
    for n in (1, 2, 7, 11):
        for w in (1, 3, 5, 20):
            tr = np.arange(1, n + 1)[None]
            assert O.skipgram_pairs(tr, w)[0].size == skipgram_slots(n, w)


def test_log_uniform_cdf_matches_product_and_distribution():
    V = 1000
    cdf = O.log_uniform_cdf(V)
    assert np.array_equal(cdf, log_uniform_cdf(V))
    assert np.all(np.diff(cdf.astype(np.int64)) >= 0) and cdf[-1] == 0xFFFFFFFF
    s = O.log_uniform_sample(cdf, 0, 4000, 1, seed=3, step=0)[:, 0]
    p = np.log((np.arange(V) + 2.0) / (np.arange(V) + 1.0)) / np.log(V + 1.0)
    for k in (0, 1, 2, 10):
        assert abs(np.mean(s == k) - p[k]) < 4 * np.sqrt(p[k] / 4000)


def test_log_uniform_unique():
    cdf = O.log_uniform_cdf(20)
    out = O.log_uniform_sample(cdf, 7, 50, 15, seed=1, step=2)
    assert all(len(set(r)) == 15 for r in out) and out.min() >= 0 and out.max() < 20


def test_weighted_walk_follows_weights():
    rng = np.random.default_rng(0)
    indptr, indices, w = make_graph(rng)
    cumw = O.weight_prefix(indptr, w)
    tr = O.weighted_walks(indptr, indices, cumw, 300, 0, 3000, 1, seed=5, step=0)
    assert tr[:, 0].min() >= 1
    for i in range(3000):
        v, u = tr[i]
        lo, hi = indptr[v], indptr[v + 1]
        if hi == lo or w[lo:hi].sum() == 0:
            assert u == -1
        else:  # the chosen edge exists and has positive weight
            ok = (indices[lo:hi] == u) & (w[lo:hi] > 0)
            assert ok.any()
    # empirical transition frequencies from one heavy node
    v = int(np.argmax(np.diff(indptr)))
    lo, hi = indptr[v], indptr[v + 1]
    gi = np.arange(20000)
    r = O.draw(5, O.PURPOSE_WALK, gi, 0, 0, 0)
    tgt = (r.astype(np.float64) + 0.5) * 2.3283064365386963e-10 * cumw[hi - 1]
    e = np.searchsorted(cumw[lo:hi], tgt, side="right")
    freq = np.bincount(e, minlength=hi - lo) / 20000
    pw = w[lo:hi] / w[lo:hi].sum()
    assert np.abs(freq - pw).max() < 0.02
