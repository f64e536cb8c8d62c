"""Oracle: EGES training-pair pipeline (weighted walk → skip-grams → log-uniform negatives).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Parity unpinned — DGL 0.6.1 and TensorFlow
are absent; the three third-party samplers are restated from their documented behaviour [3p]
at the reference's call sites:
  eges/data_loader.py:30       seeds = np.random.randint(1, len(idx2item))   (0 is OOV)
  eges/data_loader.py:31-32    dgl.sampling.random_walk(g, seeds, length=10, prob='weight',
                                                        restart_prob=0)
  eges/data_loader.py:34-36    tf.keras.preprocessing.sequence.skipgrams(seq, window_size=5,
                                                                        negative_samples=0)
  eges/data_loader.py:40-46    tf.random.log_uniform_candidate_sampler(num_sampled=num_ns,
                                                                        unique=True, range_max=V)
Draws follow the engine's Philox scheme (oracle/pinsage.py: key (seed_lo, seed_hi ^ purpose),
counter (a, b, step, draw // 4)). Choices fixed by this restatement: an edge is chosen as the
first whose per-node inclusive float64 prefix weight exceeds (r + 0.5) / 2^32 · W_v; a
log-uniform class is the first k whose cdf[k] = floor(log(k+2) / log(V+1) · 2^32) exceeds the
raw 32-bit draw; trace entries ≤ 0 (OOV 0, the walk's -1 padding) make no skip-gram pair; pairs
keep enumeration order (the reference's shuffles only permute them).
"""
from __future__ import annotations

import numpy as np

from .pinsage import bounded, draw

PURPOSE_SEED = 0x400
PURPOSE_WALK = 0x500
PURPOSE_NEG = 0x600


def weight_prefix(indptr, weights):
    """Per-node inclusive prefix of the CSR edge weights, summed sequentially in float64."""
    w = np.asarray(weights, np.float32).astype(np.float64)
    out = np.empty_like(w)
    for v in range(len(indptr) - 1):
        lo, hi = int(indptr[v]), int(indptr[v + 1])
        if hi > lo:
            out[lo:hi] = np.cumsum(w[lo:hi])
    return out


def weighted_walks(indptr, indices, cumw, n_items, walk_base, n_walks, length, seed, step):
    gi = np.arange(walk_base, walk_base + n_walks, dtype=np.int64)
    node = 1 + bounded(draw(seed, PURPOSE_SEED, gi, 0, step, 0), n_items - 1)
    traces = np.full((n_walks, length + 1), -1, np.int32)
    traces[:, 0] = node
    for h in range(length):
        r = draw(seed, PURPOSE_WALK, gi, 0, step, h)
        for i in range(n_walks):
            v = int(node[i])
            if v < 0:
                continue
            lo, hi = int(indptr[v]), int(indptr[v + 1])
            if hi <= lo or not cumw[hi - 1] > 0.0:
                node[i] = -1
                continue
            target = (float(r[i]) + 0.5) * 2.3283064365386963e-10 * cumw[hi - 1]
            e = lo + int(np.searchsorted(cumw[lo:hi], target, side="right"))
            node[i] = indices[min(e, hi - 1)]
        traces[:, h + 1] = node
    return traces


def skipgram_pairs(traces, window):
    tgt, ctx = [], []
    for tr in np.asarray(traces):
        n = len(tr)
        for i in range(n):
            for j in range(max(0, i - window), min(n, i + window + 1)):
                if j != i and tr[i] > 0 and tr[j] > 0:
                    tgt.append(tr[i])
                    ctx.append(tr[j])
    return np.asarray(tgt, np.int32), np.asarray(ctx, np.int32)


def log_uniform_cdf(range_max):
    k = np.arange(range_max, dtype=np.float64)
    c = np.floor(np.log(k + 2.0) / np.log(range_max + 1.0) * 4294967296.0)
    return np.minimum(c, 4294967295.0).astype(np.uint32)


def log_uniform_sample(cdf, pair_base, n_pairs, num_sampled, seed, step):
    out = np.zeros((n_pairs, num_sampled), np.int32)
    for p in range(n_pairs):
        got, d = [], 0
        while len(got) < num_sampled:
            r = int(draw(seed, PURPOSE_NEG, [pair_base + p], 0, step, d)[0])
            k = min(int(np.searchsorted(cdf, r, side="right")), len(cdf) - 1)
            if k not in got:
                got.append(k)
            d += 1
        out[p] = got
    return out
