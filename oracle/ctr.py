"""Oracle: DLRM / DeepFM forward, backward and one sparse-SGD train step in NumPy float32.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py; parity unpinned). Used by tests/ for the
end-to-end step parity and by bench.py as the timed CPU baseline ("port").

References: ctr/layers.py:5-14 (MLP: hidden Dense layers linear, last one activated),
ctr/model.py:34-58 (DLRM), ctr/model.py:6-31 (DeepFM), ctr/train.py:74-79 (DLRM topology and
the SGD path), keras binary_crossentropy [3p] (clip to [eps, 1-eps], log(p + eps)).
"""
from __future__ import annotations

import numpy as np

from .embedding import global_rows, segment_sum_tiled, sort_ids

EPS = np.float32(1e-7)


def mlp_forward(x, layers, final_activation):
    """layers = [(kernel [in,out], bias [out]), ...]; returns (out, cache)."""
    cache = [x]
    h = x
    for li, (k, b) in enumerate(layers):
        h = h @ k + b
        if li == len(layers) - 1:
            if final_activation == "relu":
                h = np.maximum(h, 0)
            elif final_activation == "sigmoid":
                h = 1.0 / (1.0 + np.exp(-h))
        cache.append(h)
    return h, cache


def mlp_backward(dout, layers, cache, final_activation, need_dx=True):
    """Returns (dx, [(dk, db), ...])."""
    grads = [None] * len(layers)
    d = dout
    for li in range(len(layers) - 1, -1, -1):
        k, _ = layers[li]
        y = cache[li + 1]
        if li == len(layers) - 1:
            if final_activation == "relu":
                d = d * (y > 0)
            elif final_activation == "sigmoid":
                d = d * y * (1 - y)
        x = cache[li]
        grads[li] = (x.T @ d, d.sum(0))
        if li > 0 or need_dx:
            d = d @ k.T
    return d, grads


def bce(y, p):
    pc = np.clip(p, EPS, 1 - EPS)
    return -(y * np.log(pc + EPS) + (1 - y) * np.log(1 - pc + EPS))


def bce_grad(y, p):
    """d/dp of mean BCE (the clip passes the gradient only inside [eps, 1-eps])."""
    pc = np.clip(p, EPS, 1 - EPS)
    inside = (p >= EPS) & (p <= 1 - EPS)
    g = -(y / (pc + EPS)) + (1 - y) / (1 - pc + EPS)
    return (g * inside / y.size).astype(np.float32)


class DLRMState:
    def __init__(self, table, slot_offsets, bottom, top):
        self.table = table            # [V, D] float32 (mutated in place by step)
        self.slot_offsets = slot_offsets
        self.bottom = bottom          # [(k, b)]
        self.top = top


def dlrm_forward(st: DLRMState, cat, dense_in):
    B, S = cat.shape
    D = st.table.shape[1]
    F = S + 1
    bot, bcache = mlp_forward(dense_in, st.bottom, "relu")
    rows = global_rows(cat, st.table.shape[0], st.slot_offsets).reshape(B, S)
    emb = np.where(rows[..., None] >= 0, st.table[np.maximum(rows, 0)], 0).astype(np.float32)
    x = np.concatenate([emb, bot[:, None, :]], axis=1)               # [B, F, D]
    z = np.matmul(x, x.transpose(0, 2, 1))                           # [B, F, F]
    z = z * np.triu(np.ones((F, F), np.float32), 1)[None]            # strict upper kept
    tin = np.concatenate([z.reshape(B, F * F), bot], axis=1)
    p, tcache = mlp_forward(tin, st.top, "sigmoid")
    return p[:, 0], dict(bcache=bcache, tcache=tcache, x=x, rows=rows)


def dlrm_sgd_step(st: DLRMState, cat, dense_in, y, lr):
    """One DLRM train step: forward, mean BCE, backward, SGD on every parameter (dense: plain
    SGD; table: deduplicated sparse SGD with the kernel's summation order). Returns loss."""
    B, S = cat.shape
    D = st.table.shape[1]
    F = S + 1
    p, c = dlrm_forward(st, cat, dense_in)
    loss = float(bce(y, p).mean())
    dp = bce_grad(y, p)[:, None]
    dtin, tgrads = mlp_backward(dp, st.top, c["tcache"], "sigmoid")
    dz = dtin[:, : F * F].reshape(B, F, F) * np.triu(np.ones((F, F), np.float32), 1)[None]
    sm = dz + dz.transpose(0, 2, 1)
    dx = np.matmul(sm, c["x"])                                       # [B, F, D]
    dbot = dx[:, S, :] + dtin[:, F * F:]
    _, bgrads = mlp_backward(dbot, st.bottom, c["bcache"], "relu", need_dx=False)
    lr = np.float32(lr)
    for layers, grads in ((st.top, tgrads), (st.bottom, bgrads)):
        for i, ((k, b), (dk, db)) in enumerate(zip(layers, grads)):
            layers[i] = (k - lr * dk, b - lr * db)
    sr, sp, _ = sort_ids(cat, st.table.shape[0], st.slot_offsets)
    ur, ug = segment_sum_tiled(sr, sp, dx[:, :S, :].reshape(B * S, D), st.table.shape[0])
    u = ur.astype(np.int64)
    st.table[u] = st.table[u] - lr * ug
    return loss
