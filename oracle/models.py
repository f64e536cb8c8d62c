"""Torch-fp32 restatements of the float-only model families (esmm BASE / ESMM / MMOE) and of
their Keras-Adam train step — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py; parity
unpinned: the reference's arithmetic is TF 2.2, absent here).

These are plain torch ops (indexing, matmul, activations, autograd) on copies of a model's
parameters; nothing here calls recommender_amd. References: esmm/layers.py:4-13 (MLP: relu
hidden layers, `last_activation` on the last), esmm/esmm.py:15-31 (compute_embedding in input
order, p_ctcvr = p_ctr * p_cvr), esmm/mmoe.py:19-46 (experts relu-last, softmax gates,
outputs[1] = outputs[0] * outputs[1]), esmm/base.py:14-19, esmm/train.py:97-106 (mean BCE,
Adam), Keras binary_crossentropy [3p] (clip to [eps, 1-eps], log(p + eps)).
"""
from __future__ import annotations

import numpy as np
import torch

EPS = 1e-7
_ACT = {0: lambda x: x, 1: torch.relu, 2: torch.sigmoid}


def _leaf(t, dtype=None):
    t = t.detach()
    return (t.to(dtype) if dtype is not None else t).clone().requires_grad_(True)


def _mlp(mlp, dtype=None):
    """[(kernel, bias, act)] leaf copies of an esmm MLP's Dense layers."""
    return [(_leaf(l.kernel, dtype), _leaf(l.bias, dtype), l.act_code) for l in mlp.mlp]


def esmm_family_params(model, dtype=None) -> dict:
    kind = type(model).__name__
    if kind == "ESMM":
        return {"kind": kind, "ctr": _mlp(model.ctr, dtype), "cvr": _mlp(model.cvr, dtype)}
    if kind == "BaseModel":
        return {"kind": kind, "mlp": _mlp(model.mlp, dtype)}
    return {"kind": kind, "experts": [_mlp(e, dtype) for e in model.experts],
            "gates": [(_leaf(g.kernel, dtype), _leaf(g.bias, dtype)) for g in model.gates],
            "towers": [_mlp(t, dtype) for t in model.task_towers]}


def flat_params(P) -> list:
    """The leaves in the model's named_parameters order (embedding handle excluded)."""
    out = []
    if P["kind"] == "ESMM":
        mlps = [P["ctr"], P["cvr"]]
    elif P["kind"] == "BaseModel":
        mlps = [P["mlp"]]
    else:
        out_e = [x for m in P["experts"] for k, b, _ in m for x in (k, b)]
        out_g = [x for g in P["gates"] for x in g]
        out_t = [x for m in P["towers"] for k, b, _ in m for x in (k, b)]
        return out_e + out_g + out_t
    return [x for m in mlps for k, b, _ in m for x in (k, b)]


def _run(mlp, x):
    for k, b, act in mlp:
        x = _ACT[act](x @ k + b)
    return x


def esmm_family_forward(P, e):
    """e: [B, F*D] concatenated embeddings (input-dict order). Returns y [B, 2] ([B, 1] BASE)."""
    if P["kind"] == "ESMM":
        c, v = _run(P["ctr"], e), _run(P["cvr"], e)
        return torch.cat([c, c * v], 1)
    if P["kind"] == "BaseModel":
        return _run(P["mlp"], e)
    ex = torch.stack([_run(m, e) for m in P["experts"]], 1)            # [B, E, H]
    outs = []
    for (gk, gb), t in zip(P["gates"], P["towers"]):
        gw = torch.softmax(e @ gk + gb, -1)                           # [B, E]
        outs.append(_run(t, (gw.unsqueeze(1) @ ex).squeeze(1)))
    outs[1] = outs[0] * outs[1]
    return torch.cat(outs, 1)


def keras_bce_mean(y, p):
    pc = p.clamp(EPS, 1 - EPS)
    return (-(y * torch.log(pc + EPS) + (1 - y) * torch.log(1 - pc + EPS))).mean()


def keras_adam_torch(w, m, v, g, c):
    """Keras Adam on torch tensors in the op order of oracle/ctr.keras_adam_dense."""
    m2 = m * c["beta1"] + g * c["one_minus_beta1"]
    v2 = v * c["beta2"] + (g * g) * c["one_minus_beta2"]
    return w - (m2 * c["lr"]) / (torch.sqrt(v2) + c["epsilon"]), m2, v2


def esmm_family_step(model, table, slot_offsets, feats: dict, label, dtype=torch.float32,
                     perm=None):
    """Loss, dense gradients (flat_params order) and the table's gradient rows [B*F, D] in
    position order (p = b*F + f) of one esmm-family step, by torch autograd in `dtype`
    (float64: the accuracy reference; float32 with a batch permutation `perm`: a sample of the
    rounding another fp32 evaluation order shows — the outputs come back in batch order)."""
    P = esmm_family_params(model, dtype)
    ids = torch.stack([feats[f].reshape(-1).long() for f in feats], 1)   # [B, F]
    lab = label.to(dtype)
    if perm is not None:
        ids, lab = ids[perm], lab[perm]
    rows = ids + slot_offsets[:-1].to(ids.device)[None, :]
    E = table[rows].detach().to(dtype).clone().requires_grad_(True)      # [B, F, D]
    y = esmm_family_forward(P, E.reshape(E.shape[0], -1))
    loss = keras_bce_mean(lab, y)
    leaves = flat_params(P)
    grads = torch.autograd.grad(loss, leaves + [E])
    gE = grads[-1]
    y = y.detach()
    if perm is not None:
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(perm.numel(), device=perm.device)
        y, gE = y[inv], gE[inv]
    return float(loss.detach()), y, list(grads[:-1]), gE.reshape(-1, table.shape[1])


def esmm_grad_magnitude(model, table, slot_offsets, feats: dict, label, chunks=32):
    """Float64 magnitude of every dense gradient over the batch: Σ_k |g_k| over `chunks`
    contiguous chunks of the batch, g_k = chunk k's contribution to the batch-mean gradient.
    Any fp32 reduction over the batch errs by a small multiple of eps·Σ_k |g_k| (the chunks still
    cancel inside); the tests use it as the per-element floor of the dense-gradient check where
    the gradient itself is a near-cancelling sum of 10^5 terms."""
    B = label.shape[0]
    c = B // chunks
    mag = None
    for k in range(chunks):
        sl = slice(k * c, (k + 1) * c if k < chunks - 1 else B)
        n = sl.stop - sl.start
        g = esmm_family_step(model, table, slot_offsets, {f: v[sl] for f, v in feats.items()},
                             label[sl], dtype=torch.float64)[2]
        g = [(t * (n / B)).abs() for t in g]
        mag = g if mag is None else [a + b for a, b in zip(mag, g)]
    return mag


# ---- EGES / GES / DeepWalk (eges/model.py:20-102, eges/train.py:14-24) ---------------------
def eges_step(model, inputs, labels):
    """Loss (sigmoid CE on the 1 + num_ns skip-gram logits, reduce_mean) and, per table, its
    gradient rows in lookup-position order, by torch autograd in fp32 on gathered copies of the
    rows: DeepWalk: hidden = Emb_in(q); GES: mean of the id / cat / brand rows; EGES:
    softmax(Emb_w(q)) · [id, cat, brand] rows; logits = Emb_out(match) · hiddenᵀ.
    Returns (loss, logits, {table name: (ids [N] int64, rows [N, D])})."""
    kind = type(model).__name__
    looked = {}

    def rows(name, ids):
        E = getattr(model, name).weight[ids.long()].detach().clone().requires_grad_(True)
        looked[name] = (ids.reshape(-1).long(), E)
        return E

    if kind == "DeepWalk":
        q, m = inputs
        hidden = rows("input_embedding", q)                                   # [B, 1, D]
    else:
        q, c, b, m = inputs
        side = torch.cat([rows("id_embedding", q), rows("cat_embedding", c),
                          rows("brand_embedding", b)], 1)                     # [B, 3, D]
        if kind == "EGES":
            hidden = torch.matmul(torch.softmax(rows("weight_embedding", q), -1), side)
        else:
            hidden = (side[:, 0:1] + side[:, 1:2] + side[:, 2:3]) / 3
    logits = torch.matmul(rows("output_embedding", m), hidden.transpose(1, 2)).squeeze(-1)
    z, x = labels, logits
    loss = (torch.clamp(x, min=0) - x * z + torch.log1p(torch.exp(-x.abs()))).mean()
    names = list(looked)
    grads = torch.autograd.grad(loss, [looked[n][1] for n in names])
    out = {n: (looked[n][0], g.reshape(-1, g.shape[-1])) for n, g in zip(names, grads)}
    return float(loss.detach()), logits.detach(), out
