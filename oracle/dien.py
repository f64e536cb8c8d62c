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
