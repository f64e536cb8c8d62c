"""Torch-fp32 restatements of the dien model family (BASE / DIN / DIEN) — TEST INFRASTRUCTURE
ONLY (see oracle/__init__.py; parity unpinned: Keras GRU / RNN / BatchNormalization are TF 2.2
[3p], absent here). Plain torch ops with explicit time loops; nothing here calls
recommender_amd. Each function cites the reference lines it restates.
"""
from __future__ import annotations

import torch

_ACT = {None: lambda x: x, "relu": torch.relu, "sigmoid": torch.sigmoid}


def gru(x, W, U, bias, mask):
    """Keras GRU(reset_after=True) [3p] as used by InterestExtract (dien/layers.py:78):
    z, r = σ(xW + b + hU + b_r); h̃ = tanh(xW_h + b_h + r ⊙ (hU_h + b_rh));
    h = z ⊙ h_prev + (1 - z) ⊙ h̃; a masked step carries the state; return_sequences."""
    B, T, X = x.shape
    H = U.shape[0]
    h = torch.zeros(B, H, device=x.device, dtype=x.dtype)
    outs = []
    for t in range(T):
        xw = x[:, t] @ W + bias[0]
        inner = h @ U + bias[1]
        z = torch.sigmoid(xw[:, :H] + inner[:, :H])
        r = torch.sigmoid(xw[:, H:2 * H] + inner[:, H:2 * H])
        hh = torch.tanh(xw[:, 2 * H:] + r * inner[:, 2 * H:])
        hn = z * h + (1 - z) * hh
        h = torch.where(mask[:, t:t + 1], hn, h)
        outs.append(h)
    return torch.stack(outs, 1)


def augru(x, a, ku, bu, kr, br, kh, bh, mask):
    """AUGRUCell + InterestEvolve (dien/layers.py:161-204): c = [h, x]; u = σ(c·K_u + b),
    r = σ(c·K_r + b), h̃ = tanh([x, r ⊙ h]·K_h + b); u ← a·u; h = u ⊙ h̃ + (1 - u) ⊙ h;
    masked steps carry the state; returns the last state."""
    B, T, X = x.shape
    H = ku.shape[1]
    h = torch.zeros(B, H, device=x.device, dtype=x.dtype)
    for t in range(T):
        c = torch.cat([h, x[:, t]], -1)
        u = torch.sigmoid(c @ ku + bu)
        r = torch.sigmoid(c @ kr + br)
        hh = torch.tanh(torch.cat([x[:, t], r * h], -1) @ kh + bh)
        u = u * a[:, t]
        hn = u * hh + (1 - u) * h
        h = torch.where(mask[:, t:t + 1], hn, h)
    return h


def attention(target, hs, K, mask):
    """DIENAttention (dien/layers.py:136-158): s = (H·K)·tᵀ + (1 - m)·(-1e9), softmax over L."""
    s = (hs @ K) @ target.transpose(1, 2)
    s = s + (1.0 - mask.unsqueeze(-1).to(s.dtype)) * -1e9
    return torch.softmax(s, dim=1)


def his_average(his, mask):
    """compute_his_average (dien/layers.py:5-17): masked mean; 0 / 0 = NaN on an empty history."""
    m = mask.unsqueeze(-1).to(his.dtype)
    return (his * m).sum(1) / m.sum(1)


def dense_stack(x, layers):
    """[(kernel, bias, activation name)] applied in order (keras Dense)."""
    for k, b, act in layers:
        x = _ACT[act](x @ k + b)
    return x


def local_activation(target, his, mask, layers):
    """LocalActivationUnit (dien/layers.py:34-59): weights = Dense(80σ)·Dense(40σ)·Dense(1) on
    [t, h, t - h, t ⊙ h], masked, UNnormalised; returns weightsᵀ·H."""
    B, T, D = his.shape
    t = target.expand(B, T, D)
    w = dense_stack(torch.cat([t, his, t - his, t * his], -1), layers)     # [B, T, 1]
    w = w * mask.unsqueeze(-1).to(w.dtype)
    return (w.transpose(1, 2) @ his).squeeze(1)


def sigmoid_ce(labels, logits):
    """tf.nn.sigmoid_cross_entropy_with_logits: max(x, 0) - x·z + log(1 + exp(-|x|))."""
    return torch.clamp(logits, min=0) - logits * labels + torch.log1p(torch.exp(-logits.abs()))


def aux_loss(hidden, pos, neg, mask, aux_layers):
    """InterestExtract.compute_auxiliary_loss (dien/layers.py:89-108): logits of
    [h_t, e_{t+1}] for the positive and negative next items, sigmoid CE (labels 1 / 0), masked,
    summed over both and divided by 2·Σ mask[:, 1:] (NaN for a length-1 history)."""
    h = hidden[:, :-1, :]
    m = mask[:, 1:].to(h.dtype)
    pl = dense_stack(torch.cat([h, pos[:, 1:, :]], -1), aux_layers).squeeze(-1)
    nl = dense_stack(torch.cat([h, neg[:, 1:, :]], -1), aux_layers).squeeze(-1)
    pos_loss = sigmoid_ce(torch.ones_like(pl), pl) * m
    neg_loss = sigmoid_ce(torch.zeros_like(nl), nl) * m
    return torch.cat([pos_loss, neg_loss], -1).sum(-1) / (m.sum(-1) * 2.0)


def batch_norm_inference(x, mean, var, gamma, beta, eps):
    """keras BatchNormalization in inference mode [3p]: (x - mean)/sqrt(var + eps)·γ + β."""
    return (x - mean) * torch.rsqrt(var + eps) * gamma + beta


# ---- the whole DIEN train step (dien/train.py:14-22) ------------------------------------------
_LOOKUPS = (("item", "target_item"), ("cat", "target_cat"), ("item", "pos_his_item"),
            ("cat", "pos_his_cat"), ("item", "neg_his_item"), ("cat", "neg_his_cat"))


def keras_bce_mean(y, p, eps=1e-7):
    """tf.reduce_mean(keras.losses.binary_crossentropy(label [B,1], pred [B,1])) [3p]: clip to
    [eps, 1 - eps], -(y·log(p + eps) + (1 - y)·log(1 - p + eps)), mean over the last axis
    (size 1) then over the batch."""
    pc = p.clamp(eps, 1 - eps)
    return (-(y * torch.log(pc + eps) + (1 - y) * torch.log(1 - pc + eps))).mean()


def dien_params(model, dtype):
    """Leaf copies (dtype) of every trainable DIEN parameter, by the model's parameter names
    (the embedding tables are not leaves here: their rows are gathered per lookup)."""
    return {n: p.detach().to(dtype).clone().requires_grad_(True)
            for n, p in model.named_parameters() if not n.endswith("grad_handle")}


def dien_forward(model, P, E, mask, mlp_training, bn_stats=None):
    """DIEN.call (dien/model.py:67-80) from parameter leaves P and the flat embeddings
    E = {target [B,1,36], pos [B,L,36], neg [B,L,36]}: InterestExtract (GRU + aux loss),
    DIENAttention, InterestEvolve (AUGRU), concat, MLP (BatchNormalization with batch
    statistics when `mlp_training`, moving statistics otherwise; dien/layers.py:20-31).
    Returns (prob [B,1], aux [B], (moving mean, moving variance) after the step, or None)."""
    pre = "interest_extract_layer."
    hidden = gru(E["pos"], P[pre + "gru.kernel"], P[pre + "gru.recurrent_kernel"],
                 P[pre + "gru.bias"], mask)
    aux_layers = [(P[f"{pre}auxiliary_net.layers.{i}.kernel"], P[f"{pre}auxiliary_net.layers.{i}.bias"],
                   act) for i, act in enumerate(("sigmoid", "sigmoid", None))]
    aux = aux_loss(hidden, E["pos"], E["neg"], mask, aux_layers)
    score = attention(E["target"], hidden, P["attention.kernel"], mask)
    a = "interest_evolve.augru."
    rep = augru(hidden, score, P[a + "update_gate.kernel"], P[a + "update_gate.bias"],
                P[a + "reset_gate.kernel"], P[a + "reset_gate.bias"],
                P[a + "hidden_layer.kernel"], P[a + "hidden_layer.bias"], mask)
    x = torch.cat([E["target"].squeeze(1), rep], -1)
    bn = model.mlp.bn
    stats = None
    if mlp_training and bn_stats is not None:  # given batch statistics, held constant
        mean, var = (t.to(x.dtype) for t in bn_stats)
    elif mlp_training:  # batch statistics; the moving averages after the step [3p keras]
        mean, var = x.mean(0), x.var(0, unbiased=False)
        d = 1.0 - bn.momentum
        mm = bn.moving_mean.to(x.dtype)
        mv = bn.moving_variance.to(x.dtype)
        stats = (mm - (mm - mean.detach()) * d, mv - (mv - var.detach()) * d)
    else:
        mean = bn.moving_mean.to(x.dtype)
        var = bn.moving_variance.to(x.dtype)
    x = batch_norm_inference(x, mean, var, P["mlp.bn.gamma"], P["mlp.bn.beta"], bn.epsilon)
    n = len(model.mlp.mlp)
    layers = [(P[f"mlp.mlp.{i}.kernel"], P[f"mlp.mlp.{i}.bias"], "relu" if i < n - 1 else "sigmoid")
              for i in range(n)]
    return dense_stack(x, layers), aux, stats


def dien_step(model, feats, label, dtype=torch.float64, mlp_training=None, perm=None,
              bn_stats=None):
    """One DIEN train step's loss and gradients (dien/train.py:14-22: mean Keras BCE + mean aux,
    gradients of every trainable variable) by torch autograd in `dtype` on copies of the model's
    parameters and of the looked-up table rows. mlp_training None: the model's own setting.
    bn_stats (optional, (mean, var)): training-mode BN with these statistics held constant
    (the tests' per-chunk magnitude pass).
    perm (optional, a permutation of the batch): evaluate on the permuted batch and map the
    per-example outputs back — the same function in exact arithmetic, another fp32 rounding
    order (the tests sample the fp32 rounding noise this way).
    Returns dict(loss, prob, aux, grads {param name: grad}, rows {lookup key: grad rows [N, 18]},
    stats (the BN moving averages after a training-mode step, else None))."""
    if perm is not None:
        inv = torch.argsort(perm)
        out = dien_step(model, {k: v[perm] for k, v in feats.items()}, label[perm], dtype,
                        mlp_training, bn_stats=bn_stats)
        out["prob"], out["aux"] = out["prob"][inv], out["aux"][inv]
        for k, r in out["rows"].items():
            B = label.shape[0]
            out["rows"][k] = r.reshape(B, -1, r.shape[-1])[inv].reshape(-1, r.shape[-1])
        return out
    if mlp_training is None:  # DIEN.head_bn_mode (recommender_amd/dien/model.py)
        mlp_training = getattr(model, "head_bn_mode", "inference") == "propagate"
    P = dien_params(model, dtype)
    W = {"item": model.item_embedding.weight.detach().to(dtype),
         "cat": model.cat_embedding.weight.detach().to(dtype)}
    leaves = {}
    for table, key in _LOOKUPS:
        leaves[key] = W[table][feats[key].long()].clone().requires_grad_(True)

    def flat(a, b):
        return torch.cat([leaves[a], leaves[b]], -1)

    E = {"target": flat("target_item", "target_cat"), "pos": flat("pos_his_item", "pos_his_cat"),
         "neg": flat("neg_his_item", "neg_his_cat")}
    mask = feats["pos_his_item"] != 0
    prob, aux, stats = dien_forward(model, P, E, mask, mlp_training, bn_stats)
    loss = keras_bce_mean(label.to(dtype), prob) + aux.mean()
    names = list(P)
    keys = [k for _, k in _LOOKUPS]
    g = torch.autograd.grad(loss, [P[n] for n in names] + [leaves[k] for k in keys])
    if bn_stats is None and mlp_training:
        bn_stats = tuple(t.detach() for t in _bn_batch_stats(model, P, E, mask))
    return dict(loss=float(loss.detach()), prob=prob.detach(), aux=aux.detach(),
                bn_batch=bn_stats,
                grads=dict(zip(names, g[:len(names)])),
                rows={k: gr.reshape(-1, gr.shape[-1]) for k, gr in zip(keys, g[len(names):])},
                stats=stats)


def _bn_batch_stats(model, P, E, mask):
    """The head BN's batch mean / variance of this forward (for the magnitude pass)."""
    with torch.no_grad():
        pre = "interest_extract_layer."
        hidden = gru(E["pos"], P[pre + "gru.kernel"], P[pre + "gru.recurrent_kernel"],
                     P[pre + "gru.bias"], mask)
        score = attention(E["target"], hidden, P["attention.kernel"], mask)
        a = "interest_evolve.augru."
        rep = augru(hidden, score, P[a + "update_gate.kernel"], P[a + "update_gate.bias"],
                    P[a + "reset_gate.kernel"], P[a + "reset_gate.bias"],
                    P[a + "hidden_layer.kernel"], P[a + "hidden_layer.bias"], mask)
        x = torch.cat([E["target"].squeeze(1), rep], -1)
        return x.mean(0), x.var(0, unbiased=False)


def dien_grad_magnitude(model, feats, label, chunks=16, mlp_training=None, bn_stats=None):
    """Float64 magnitude of every dense gradient over the batch: Σ_k |g_k| over `chunks`
    contiguous chunks of the batch, g_k = chunk k's contribution to the batch-mean gradient
    (BN batch statistics of the whole batch held constant). A reduction over the batch in any
    fp32 order errs by a small multiple of eps·Σ_k |g_k|; the tests use it as the per-element
    floor of the dense-gradient check."""
    B = label.shape[0]
    c = B // chunks
    mag = None
    for k in range(chunks):
        sl = slice(k * c, (k + 1) * c if k < chunks - 1 else B)
        n = sl.stop - sl.start
        out = dien_step(model, {f: v[sl] for f, v in feats.items()}, label[sl], torch.float64,
                        mlp_training, bn_stats=bn_stats)
        g = {nm: (t * (n / B)).abs() for nm, t in out["grads"].items()}
        mag = g if mag is None else {nm: mag[nm] + g[nm] for nm in mag}
    return mag
