"""Synthetic weighted item graph for the EGES sampler tests: symmetric session co-occurrence
counts (the reference's train_g edge 'weight', eges/data_loader.py:31), node 0 = OOV with no
edges, a few isolated items (dead ends → -1 padding), weights including zeros."""
import numpy as np


def make_graph(rng, n_items=300, n_edges=2000, n_isolated=5):
    src = rng.integers(1, n_items, n_edges)
    dst = rng.integers(1, n_items, n_edges)
    iso = rng.choice(np.arange(1, n_items), n_isolated, replace=False)
    keep = ~np.isin(src, iso) & ~np.isin(dst, iso) & (src != dst)
    src, dst = src[keep], dst[keep]
    s = np.concatenate([src, dst])
    d = np.concatenate([dst, src])
    w = rng.integers(0, 6, s.size).astype(np.float32)  # some zero-weight edges
    w[rng.random(s.size) < 0.3] *= 1.37
    order = np.lexsort((d, s))
    s, d, w = s[order], d[order], w[order]
    indptr = np.zeros(n_items + 1, np.int64)
    np.add.at(indptr, s + 1, 1)
    return np.cumsum(indptr), d.astype(np.int32), w
