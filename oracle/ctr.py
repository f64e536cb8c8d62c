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


def mlp_forward(x, layers, final_activation, pre=None):
    """layers = [(kernel [in,out], bias [out]), ...]; returns (out, cache). `pre` (a list)
    receives the last layer's pre-activation values."""
    cache = [x]
    h = x
    for li, (k, b) in enumerate(layers):
        h = h @ k + b
        if li == len(layers) - 1:
            if pre is not None:
                pre.append(h)
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
    pre = []
    p, tcache = mlp_forward(tin, st.top, "sigmoid", pre)
    return p[:, 0], dict(bcache=bcache, tcache=tcache, x=x, rows=rows, logit=pre[0][:, 0])


def magnitude_chain(x_abs, layers):
    """Float64 magnitude bound of an MLP chain's pre-activation outputs: every rounding of
    either evaluation order (layer by layer, or the composed affine map) is bounded relative
    to this, |x|·|K1|·…·|Kn| with the |biases| carried along."""
    h = np.asarray(x_abs, np.float64)
    for k, b in layers:
        h = h @ np.abs(k).astype(np.float64) + np.abs(b).astype(np.float64)
    return h


def dlrm_sgd_step(st: DLRMState, cat, dense_in, y, lr, detail=None):
    """One DLRM train step: forward, mean BCE, backward, SGD on every parameter (dense: plain
    SGD; table: deduplicated sparse SGD with the kernel's summation order). Returns loss.

    detail (a dict, optional) receives the step's intermediates for the full-size parity test:
    p, logit (pre-sigmoid) and its float64 magnitude bound, the table grad rows dx [B*S, D] in
    position order and their magnitude bound, the deduplicated (uniq_rows, uniq_grad), the dense
    gradients and the sorted (rows, pos)."""
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
    top_old = list(st.top)
    lr = np.float32(lr)
    for layers, grads in ((st.top, tgrads), (st.bottom, bgrads)):
        for i, ((k, b), (dk, db)) in enumerate(zip(layers, grads)):
            layers[i] = (k - lr * dk, b - lr * db)
    sr, sp, _ = sort_ids(cat, st.table.shape[0], st.slot_offsets)
    ur, ug = segment_sum_tiled(sr, sp, dx[:, :S, :].reshape(B * S, D), st.table.shape[0])
    u = ur.astype(np.int64)
    if detail is not None:
        tin_abs = np.abs(c["tcache"][0]).astype(np.float64)
        # |d logit / d tin| chain and the bound of the strict-upper dZ fed to the interaction
        mag_logit = magnitude_chain(tin_abs, top_old)[:, 0]
        g_abs = np.abs(dp[:, 0]).astype(np.float64) * 0.25  # |sigma'| <= 1/4
        q = np.ones((1, 1))
        for k, _ in reversed(top_old):
            q = np.abs(k).astype(np.float64) @ q
        dz_b = (g_abs[:, None] * q[None, : F * F, 0]).reshape(B, F, F)
        dz_b = dz_b * np.triu(np.ones((F, F)), 1)[None]
        dx_b = np.matmul(dz_b + dz_b.transpose(0, 2, 1), np.abs(c["x"]).astype(np.float64))
        detail.update(p=p, logit=c["logit"], logit_bound=mag_logit,
                      dx=dx[:, :S, :].reshape(B * S, D), dx_bound=dx_b[:, :S, :].reshape(B * S, D),
                      uniq_rows=u, uniq_grad=ug, top_grads=tgrads, bottom_grads=bgrads,
                      sorted_rows=sr, sorted_pos=sp)
    st.table[u] = st.table[u] - lr * ug
    return loss
