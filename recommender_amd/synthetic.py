"""Synthetic Criteo-shaped inputs (no datasets are reachable offline).

- 26 categorical slots with Criteo-Kaggle-like cardinality skew, scaled so the slab holds
  exactly `total_rows` rows (40M for the north star);
- ids: per-slot bounded Zipf(alpha=1.05) ranks (inverse-CDF of the bounded power law), mapped
  to rows by a fixed multiplicative permutation so hot ids are spread over the slot;
- 13 dense features log1p(x), x ~ Geometric(p=0.01) (the log(x+1) of ctr/tfrecord_io.py:53);
- labels ~ Bernoulli(0.256).
Seeded with numpy PCG64(seed); seed 4 = the reference default (ctr/train.py:18).
"""
from __future__ import annotations

import numpy as np

# Criteo Kaggle (display advertising challenge) per-column cardinalities
CRITEO_KAGGLE_CARDINALITIES = [
    1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593, 3194, 27,
    14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105, 142572,
]


def criteo_cardinalities(total_rows: int = 40_000_000, n_slots: int = 26) -> list[int]:
    base = np.array(CRITEO_KAGGLE_CARDINALITIES[:n_slots], dtype=np.float64)
    small = base < 100_000
    budget = total_rows - base[small].sum()
    if budget <= 0:
        out = np.maximum(1, np.floor(base * total_rows / base.sum())).astype(np.int64)
    else:
        big = base[~small]
        out = base.copy()
        out[~small] = np.floor(big * budget / big.sum())
        out = out.astype(np.int64)
    out[np.argmax(out)] += total_rows - out.sum()
    assert out.sum() == total_rows and (out >= 1).all()
    return out.tolist()


def bounded_zipf(rng: np.random.Generator, n: int, card: int, alpha: float = 1.05) -> np.ndarray:
    """Ranks in [0, card) with P(k) ~ (k+1)^-alpha (continuous inverse-CDF approximation)."""
    if card <= 1:
        return np.zeros(n, np.int64)
    u = rng.random(n)
    a1 = 1.0 - alpha
    x = ((card ** a1 - 1.0) * u + 1.0) ** (1.0 / a1)
    return np.minimum(np.floor(x).astype(np.int64) - 1, card - 1).clip(0)


def _spread(ranks: np.ndarray, card: int) -> np.ndarray:
    """Bijective rank → id map inside a slot (multiplier coprime with card)."""
    mult = 2654435761 % card if card > 2 else 1
    while np.gcd(mult, card) != 1:
        mult += 1
    return (ranks * mult) % card


def criteo_batch(rng: np.random.Generator, batch: int, cards, alpha: float = 1.05,
                 num_int_fea: int = 13, id_dtype=np.int64):
    cat = np.empty((batch, len(cards)), dtype=id_dtype)
    for s, c in enumerate(cards):
        cat[:, s] = _spread(bounded_zipf(rng, batch, c, alpha), c)
    dense = np.log1p(rng.geometric(0.01, size=(batch, num_int_fea)).astype(np.float32))
    label = (rng.random(batch) < 0.256).astype(np.float32)
    return cat, dense.astype(np.float32), label


def scaled_vocab(vocab: dict, total_rows: int) -> dict:
    """Scale a per-feature vocabulary to `total_rows` rows keeping the ratios (SURVEY §8d cfg4:
    the esmm/train.py:197-215 ratios scaled to 40M rows); every feature keeps >= its original
    size when that is smaller than the scale would give."""
    base = np.array(list(vocab.values()), dtype=np.float64)
    out = np.maximum(1, np.floor(base * total_rows / base.sum())).astype(np.int64)
    out[np.argmax(out)] += total_rows - out.sum()
    return dict(zip(vocab.keys(), out.tolist()))


def aliccp_batch(rng: np.random.Generator, batch: int, vocab: dict, alpha: float = 1.05):
    """Ali-CCP-shaped features {feat: [B, 1] int32 ids in 1..n} (0 = OOV, esmm/
    process_public_dataset.py:100,110) and labels [B, 2] = [click, purchase] with the dataset's
    rates (click 3.9%, purchase given click 0.54%; esmm/tfrecord_io.py:27-29)."""
    feats = {}
    for f, n in vocab.items():
        ids = 1 + _spread(bounded_zipf(rng, batch, max(int(n) - 1, 1), alpha), max(int(n) - 1, 1))
        feats[f] = ids.astype(np.int32).reshape(batch, 1)
    click = rng.random(batch) < 0.0389
    buy = click & (rng.random(batch) < 0.0054)
    return feats, np.stack([click, buy], 1).astype(np.float32)


# ---- MovieLens-shaped bipartite graph ---------------------------------
ML20M = dict(n_users=138_493, n_items=26_744, n_edges=20_000_263)


def movielens_graph(rng: np.random.Generator, n_users: int, n_items: int, n_edges: int,
                    min_user_deg: int = 20, n_genres: int = 20, n_years: int = 120):
    """ML-20M-shaped user–item rating graph: user degrees min_user_deg + Pareto(1.2) tail
    (ML-20M keeps users with >= 20 ratings), item popularity power law P(rank r) ~ (r+1)^-0.5
    (top item ≈ 0.3% of ratings, as in ML-20M), each (user, item) pair at most once; item
    features year id < n_years and a 1–3-hot genre vector [n_items, n_genres] (int8).
    Returns (users, items) edge arrays sorted user-major, plus year, genre."""
    budget = n_edges - min_user_deg * n_users
    raw = rng.pareto(1.2, n_users) + 1.0
    cap = max(min_user_deg, n_items // 3)
    pop = (np.arange(n_items, dtype=np.float64) + 1.0) ** -0.5
    cdf = np.cumsum(rng.permutation(pop))
    cdf /= cdf[-1]
    deg = np.minimum(min_user_deg + np.floor(budget * raw / raw.sum()).astype(np.int64), cap)
    users = np.repeat(np.arange(n_users, dtype=np.int64), deg)
    items = np.minimum(np.searchsorted(cdf, rng.random(users.size)), n_items - 1)
    keys = np.unique(users * n_items + items)
    for _ in range(4):  # top up the edges lost to duplicate (user, item) draws
        missing = n_edges - keys.size
        if missing <= 0:
            break
        users = rng.choice(n_users, size=int(missing * 1.2) + 16, p=deg / deg.sum())
        items = np.minimum(np.searchsorted(cdf, rng.random(users.size)), n_items - 1)
        keys = np.unique(np.concatenate([keys, users * n_items + items]))
    if keys.size > n_edges:
        keys = np.sort(rng.choice(keys, n_edges, replace=False))
    users, items = keys // n_items, keys % n_items
    year = rng.integers(0, n_years, n_items).astype(np.int64)
    genre = np.zeros((n_items, n_genres), np.int8)
    ng = rng.integers(1, 4, n_items)
    for k in range(3):
        m = ng > k
        genre[np.nonzero(m)[0], rng.integers(0, n_genres, int(m.sum()))] = 1
    return users, items, year, genre
