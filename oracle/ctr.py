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
    bpre = []
    bot, bcache = mlp_forward(dense_in, st.bottom, "relu", bpre)
    rows = global_rows(cat, st.table.shape[0], st.slot_offsets).reshape(B, S)
    emb = np.where(rows[..., None] >= 0, st.table[np.maximum(rows, 0)], 0).astype(np.float32)
    x = np.concatenate([emb, bot[:, None, :]], axis=1)               # [B, F, D]
    z = np.matmul(x, x.transpose(0, 2, 1))                           # [B, F, F]
    z = z * np.triu(np.ones((F, F), np.float32), 1)[None]            # strict upper kept
    tin = np.concatenate([z.reshape(B, F * F), bot], axis=1)
    pre = []
    p, tcache = mlp_forward(tin, st.top, "sigmoid", pre)
    return p[:, 0], dict(bcache=bcache, tcache=tcache, x=x, rows=rows, logit=pre[0][:, 0],
                         bot_pre=bpre[0])


def magnitude_chain(x_abs, layers):
    """Float64 magnitude bound of an MLP chain's pre-activation outputs: every rounding of
    either evaluation order (layer by layer, or the composed affine map) is bounded relative
    to this, |x|·|K1|·…·|Kn| with the |biases| carried along."""
    h = np.asarray(x_abs, np.float64)
    for k, b in layers:
        h = h @ np.abs(k).astype(np.float64) + np.abs(b).astype(np.float64)
    return h


def chain_grad_bounds(x, layers, G):
    """Float64 magnitude bounds of an MLP chain's parameter gradients for BOTH evaluation
    orders (layer by layer, or factored from the last layer's G): h_{l-1} = x·R + c, so
    |h_{l-1}ᵀ·g_l| <= (|R|ᵀ·|x|ᵀ·|G| + |c|⊗Σ|G|)·|Q_l|ᵀ with Q_l = K_{l+1}···K_L.
    layers = [(kernel [in, out], bias [out])] as the input sees them; G [B, n_L] (its absolute
    value is taken). Linear in |G|. Returns ([(kernel bound, bias bound)] per layer,
    dx bound [B, in])."""
    aG = np.abs(np.asarray(G, np.float64))
    base = np.abs(np.asarray(x, np.float64)).T @ aG
    Mb, absR, absc = [], None, None
    for i, (k, b) in enumerate(layers):
        k, b = np.asarray(k, np.float64), np.asarray(b, np.float64)
        Mb.append(base if i == 0 else absR.T @ base + np.outer(absc, aG.sum(0)))
        absR = np.abs(k) if absR is None else absR @ np.abs(k)
        absc = np.abs(b) if absc is None else np.abs(k).T @ absc + np.abs(b)
    out = [None] * len(layers)
    absQ = None
    for i in range(len(layers) - 1, -1, -1):
        kb, bb = Mb[i], aG.sum(0)
        if absQ is not None:
            kb, bb = kb @ absQ.T, bb @ absQ.T
        out[i] = (kb, bb)
        ak = np.abs(np.asarray(layers[i][0], np.float64))
        absQ = ak if absQ is None else ak @ absQ
    return out, aG @ absQ.T


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
    top_old, bottom_old = list(st.top), list(st.bottom)
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
        # the top input's own float64 magnitude bound: the bottom output's |x|·|K1|·|K2|·|K3| +
        # |biases| chain, the pair values' Cauchy–Schwarz |x_i|·|x_j| (with that bottom bound in
        # the bottom row). Any fp32 evaluation of an input rounds relative to this, not to its value.
        bot_bound = magnitude_chain(np.abs(dense_in), bottom_old)
        xb = np.abs(c["x"]).astype(np.float64)
        xb[:, S, :] = bot_bound
        zb = np.matmul(xb, xb.transpose(0, 2, 1)) * np.triu(np.ones((F, F)), 1)[None]
        top_in_bound = np.concatenate([zb.reshape(B, F * F), bot_bound], axis=1)
        del xb, zb
        detail.update(p=p, logit=c["logit"], logit_bound=mag_logit, top_in_bound=top_in_bound,
                      dx=dx[:, :S, :].reshape(B * S, D), dx_bound=dx_b[:, :S, :].reshape(B * S, D),
                      uniq_rows=u, uniq_grad=ug, top_grads=tgrads, bottom_grads=bgrads,
                      sorted_rows=sr, sorted_pos=sp,
                      # the dense half: each chain's input, its last-layer gradient G (the
                      # factored backward's only batch-deep operand) and the pre-step layers
                      top_in=c["tcache"][0], top_G=dp * c["tcache"][-1] * (1 - c["tcache"][-1]),
                      top_layers=top_old, top_Q=q[:, 0], bottom_in=dense_in,
                      bottom_G=dbot * (c["bcache"][-1] > 0), bottom_dout=dbot,
                      bottom_pre=c["bot_pre"], bottom_layers=bottom_old,
                      dbot_interaction_bound=dx_b[:, S, :])
    st.table[u] = st.table[u] - lr * ug
    return loss


# ---- DeepFM (ctr/model.py:6-31) with Keras Adam (ctr/train.py:81-84) ------------------------

def keras_adam_dense(w, m, v, g, c):
    """Keras Adam _resource_apply_dense [3p TF 2.2] in float32, Keras op order:
    m = b1*m + (1-b1)*g; v = b2*v + (1-b2)*g*g; w -= lr_t*m/(sqrt(v)+eps)."""
    f32 = np.float32
    m2 = (m * c["beta1"] + g * c["one_minus_beta1"]).astype(f32)
    v2 = (v * c["beta2"] + (g * g) * c["one_minus_beta2"]).astype(f32)
    w2 = (w - (c["lr"] * m2) / (np.sqrt(v2, dtype=f32) + c["epsilon"])).astype(f32)
    return w2, m2, v2


def deepfm_forward(table, cat, dense_in, layers, slot_offsets=None):
    """ctr/model.py:15-30: FM second-order term on the [B, S, D] lookups (no first-order term,
    no bias) plus the linear-hidden MLP over [emb.reshape(B, S*D), int features]; sigmoid."""
    B, S = cat.shape
    D = table.shape[1]
    rows = global_rows(cat, table.shape[0], slot_offsets).reshape(B, S)
    emb = table[rows]                                                # [B, S, D]
    s = emb.sum(1)
    fm = np.float32(0.5) * (s * s - (emb * emb).sum(1)).sum(1)       # ctr/model.py:21-23
    deep = np.concatenate([emb.reshape(B, S * D), dense_in], axis=1)  # ctr/model.py:25-26
    out, cache = mlp_forward(deep, layers, None)
    logit = fm + out[:, 0]
    p = (1.0 / (1.0 + np.exp(-logit))).astype(np.float32)
    return p, dict(emb=emb, s=s, cache=cache, logit=logit, rows=rows)


def deepfm_keras_adam_step(table, m, v, layers, dense_m, dense_v, cat, dense_in, y, step,
                           lr=1e-3, slot_offsets=None, grad_rows=None):
    """One DeepFM train step with Keras Adam on every parameter (mean BCE, ctr/train.py:84-85).
    `step` is 1-based (Keras local_step = iterations + 1). The table update is the sparse
    Keras apply: duplicates summed in the tiled order of oracle/embedding.segment_sum_tiled,
    then dense m/v decay and a dense var update of every row. grad_rows (optional, [B*S, D] in
    position order) replaces the oracle's own table gradient — the checker feeds the kernel's
    rows to pin the apply bit for bit. Returns (loss, new state dict, detail dict)."""
    from .embedding import apply_keras_adam, keras_adam_coefficients

    B, S = cat.shape
    D = table.shape[1]
    p, c = deepfm_forward(table, cat, dense_in, layers, slot_offsets)
    loss = float(bce(y, p).mean())
    dp = bce_grad(y, p)
    dlogit = (dp * p * (1 - p)).astype(np.float32)
    ddeep, grads = mlp_backward(dlogit[:, None], layers, c["cache"], None)
    d_emb = ddeep[:, : S * D].reshape(B, S, D) + dlogit[:, None, None] * (c["s"][:, None, :] - c["emb"])
    dx = d_emb.reshape(B * S, D).astype(np.float32)
    co = keras_adam_coefficients(step, lr)
    new_layers, nm, nv = [], [], []
    for (k, b), (dk, db), (mk, mb), (vk, vb) in zip(layers, grads, dense_m, dense_v):
        k2, mk2, vk2 = keras_adam_dense(k, mk, vk, dk.astype(np.float32), co)
        b2, mb2, vb2 = keras_adam_dense(b, mb, vb, db.astype(np.float32), co)
        new_layers.append((k2, b2))
        nm.append((mk2, mb2))
        nv.append((vk2, vb2))
    g_use = dx if grad_rows is None else grad_rows
    sr, sp, _ = sort_ids(cat, table.shape[0], slot_offsets)
    ur, ug = segment_sum_tiled(sr, sp, g_use, table.shape[0])
    t2, m2, v2 = apply_keras_adam(table, m, v, ur.astype(np.int64), ug, co)
    # float64 magnitude bounds: logit (fm + chain) and the table gradient rows
    a_emb = np.abs(c["emb"]).astype(np.float64)
    a_s = a_emb.sum(1)
    fm_b = 0.5 * (a_s * a_s + (a_emb * a_emb).sum(1)).sum(1)
    chain_b = magnitude_chain(np.abs(c["cache"][0]), layers)[:, 0]
    q = np.ones((1, 1))
    for k, _ in reversed(layers):
        q = np.abs(k).astype(np.float64) @ q
    ad = np.abs(dlogit).astype(np.float64)
    dx_b = ad[:, None, None] * (q[: S * D, 0].reshape(1, S, D) + a_s[:, None, :] + a_emb)
    detail = dict(p=p, logit=c["logit"], logit_bound=fm_b + chain_b, dx=dx,
                  dx_bound=dx_b.reshape(B * S, D), sorted_rows=sr, sorted_pos=sp,
                  dense_grads=grads)
    return loss, dict(table=t2, m=m2, v=v2, layers=new_layers, dense_m=nm, dense_v=nv), detail
