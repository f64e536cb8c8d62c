"""Oracle: DLRM DotInteraction and the DeepFM FM term (forward and backward).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py; parity unpinned).
Computed in float64 (the GPU's fp32 result is compared within the north-star 1e-5 relative
tolerance).

References: ctr/layers.py:17-43 (DotInteraction), ctr/model.py:21-23 (FM),
ctr/model.py:45-55 (DLRM concat / reshape).
"""
from __future__ import annotations

import numpy as np


def kept_mask(F: int, self_interaction: bool) -> np.ndarray:
    """ctr/layers.py:26-34: band_part(ones,-1,0) is the lower triangle incl. the diagonal.
    self_interaction → the kept matrix is that lower triangle (i >= j); otherwise it is
    ones - lower = the strict upper triangle (i < j)."""
    lower = np.tril(np.ones((F, F), bool))
    return lower if self_interaction else ~lower


def out_width(F, self_interaction, skip_gather):
    if skip_gather:
        return F * F
    return F * (F + 1) // 2 if self_interaction else F * (F - 1) // 2


def dot_interaction(x: np.ndarray, self_interaction: bool, skip_gather: bool) -> np.ndarray:
    """x [B, F, D] → skip_gather: where(kept, X·Xᵀ, 0).reshape(B, F*F) (ctr/layers.py:35-38);
    else boolean_mask(X·Xᵀ, kept) in row-major order (ctr/layers.py:39-42)."""
    x = np.asarray(x, np.float64)
    B, F, _ = x.shape
    z = np.einsum("bid,bjd->bij", x, x)
    keep = kept_mask(F, self_interaction)
    if skip_gather:
        return np.where(keep[None], z, 0.0).reshape(B, F * F)
    return z[:, keep]


def dot_interaction_bwd(x, grad_out, self_interaction, skip_gather):
    """dX = (M + Mᵀ)·X, M = grad on the kept pairs (tf.where / boolean_mask route the gradient
    only to kept entries)."""
    x = np.asarray(x, np.float64)
    B, F, _ = x.shape
    keep = kept_mask(F, self_interaction)
    g = np.asarray(grad_out, np.float64)
    m = np.zeros((B, F, F))
    if skip_gather:
        m = np.where(keep[None], g[:, : F * F].reshape(B, F, F), 0.0)
    else:
        m[:, keep] = g[:, : keep.sum()]
    s = m + np.transpose(m, (0, 2, 1))
    return np.einsum("bik,bkd->bid", s, x)


def dlrm_interaction(table, ids, dense, slot_offsets=None):
    """ctr/model.py:49-55: X = [emb(ids) (S rows), bottom-MLP output]; out = [Z (F*F, strict
    upper kept), dense] (DotInteraction(False, True), ctr/model.py:43)."""
    from .embedding import embedding_lookup

    B, S = ids.shape
    emb = embedding_lookup(table, ids, slot_offsets, raise_oob=False).astype(np.float64)
    x = np.concatenate([emb, np.asarray(dense, np.float64)[:, None, :]], axis=1)
    z = dot_interaction(x, False, True)
    return np.concatenate([z, np.asarray(dense, np.float64)], axis=1)


def dlrm_interaction_bwd(table, ids, dense, grad_out, slot_offsets=None):
    """Returns (grad_emb [B*S, D] in position order p = b*S + s, grad_dense [B, D])."""
    from .embedding import embedding_lookup

    B, S = ids.shape
    D = table.shape[1]
    F = S + 1
    emb = embedding_lookup(table, ids, slot_offsets, raise_oob=False).astype(np.float64)
    x = np.concatenate([emb, np.asarray(dense, np.float64)[:, None, :]], axis=1)
    gx = dot_interaction_bwd(x, np.asarray(grad_out)[:, : F * F], False, True)
    gd = gx[:, S, :] + np.asarray(grad_out, np.float64)[:, F * F: F * F + D]
    return gx[:, :S, :].reshape(B * S, D), gd


def fm(emb):
    """ctr/model.py:21-23: 0.5 * Σ_d (square(Σ_f e) - Σ_f square(e))."""
    e = np.asarray(emb, np.float64)
    s = e.sum(axis=1)
    return 0.5 * (s * s - (e * e).sum(axis=1)).sum(axis=1)


def fm_bwd(emb, grad_out):
    e = np.asarray(emb, np.float64)
    s = e.sum(axis=1, keepdims=True)
    return np.asarray(grad_out, np.float64)[:, None, None] * (s - e)
