"""PinSage evaluation on the device (pinsage/train/evaluation.py, util.py).

get_item_reprs   evaluation.py:6-24   every item's representation through the sampler + model,
                 in batches of batch_size seeds (the reference's test_batch_size 32). Every
                 batch of one pass uses the same sampler step. The result DOES depend on
                 batch_size, as the reference's does: Convolve divides by the Frobenius norm of
                 the whole batch (layers.py:28-29).
recommend        evaluation.py:27-51  latest item per user (rs_latest_item) → similarity rows
                 latest_repr · item_reprsᵀ (one fp32 GEMM per row chunk) → the user's training
                 items set to -inf and top-k (rs_masked_topk). Returns [n_users, top_k] int32
                 on the device, best first (the reference's argpartition gives the same set
                 in no order). batch_size only sizes the chunks; it does not change results.
hit_rate_eval    evaluation.py:54-65  mean over users of any(recommended ∈ ground truth).
train_test_split_by_time / build_val_test_matrix   util.py:5-39 (numpy instead of pandas:
                 per user by time, the last rating → test and the second-to-last → val;
                 equal timestamps keep edge order).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _lib as L
from .graph import HeteroGraph

_SCORE_CHUNK_BYTES = 1 << 30  # similarity rows per GEMM chunk: ≤ 1 GiB of fp32 scores


def train_test_split_by_time(users, timestamps):
    """(train_idx, val_idx, test_idx) edge indices (util.py:5-24)."""
    users = np.asarray(users)
    ts = np.asarray(timestamps)
    order = np.lexsort((np.arange(users.size), ts, users))  # by user, then time, then edge
    u = users[order]
    last = np.ones(u.size, bool)
    last[:-1] = u[1:] != u[:-1]
    second = np.zeros(u.size, bool)
    second[:-1] = last[1:] & (u[1:] == u[:-1])
    first = np.ones(u.size, bool)
    first[1:] = u[1:] != u[:-1]
    test = last & ~first  # users with > 1 rating
    # second-to-last → val for users with > 2 ratings (its predecessor is the same user)
    prev_same = np.zeros(u.size, bool)
    prev_same[1:] = u[1:] == u[:-1]
    val = second & prev_same
    train = ~(test | val)
    return (np.sort(order[train]), np.sort(order[val]), np.sort(order[test]))


def build_val_test_matrix(users, items, val_idx, test_idx, n_users, n_items):
    """scipy COO (n_users, n_items) matrices of ones for the val / test edges (util.py:27-39)."""
    from scipy import sparse as ssp

    users, items = np.asarray(users), np.asarray(items)
    mats = []
    for idx in (val_idx, test_idx):
        mats.append(ssp.coo_matrix((np.ones(len(idx)), (users[idx], items[idx])),
                                   (n_users, n_items)))
    return tuple(mats)


def get_item_reprs(model, pinsage_sampler, train_g: HeteroGraph, itype: str, batch_size: int):
    n = train_g.number_of_nodes(itype)
    dev = train_g.device
    step0 = pinsage_sampler.step
    out = None
    with torch.no_grad():
        for b0 in range(0, n, batch_size):
            pinsage_sampler.step = step0
            seeds = torch.arange(b0, min(n, b0 + batch_size), dtype=torch.int32, device=dev)
            reprs = model.get_repr(pinsage_sampler.generate_blocks(seeds))
            if out is None:
                out = torch.empty(n, reprs.shape[1], device=dev, dtype=reprs.dtype)
            out[b0:b0 + seeds.numel()] = reprs
    pinsage_sampler.step = step0 + 1
    return out


def latest_items(full_graph: HeteroGraph, timestamp: str) -> torch.Tensor:
    ts = full_graph.u2i_edata[timestamp].to(torch.int64).contiguous()
    dev = full_graph.device
    latest = torch.empty(full_graph.n_users, dtype=torch.int32, device=dev)
    missing = torch.zeros(1, dtype=torch.int32, device=dev)
    L.call("rs_latest_item", L.ptr(full_graph.u2i_indptr), L.ptr(full_graph.u2i), L.ptr(ts),
           full_graph.n_users, L.ptr(latest), L.ptr(missing), L.stream_ptr(dev))
    if int(missing.item()):
        raise ValueError("recommend: every user needs at least one interaction "
                         "(pinsage/train/evaluation.py:36)")
    return latest


def masked_topk(scores: torch.Tensor, top_k: int, user_base: int = 0,
                excl: HeteroGraph | None = None, with_scores: bool = False):
    L.require_device(scores, "scores")
    scores = scores.contiguous()
    R, n_items = scores.shape
    idx = torch.empty(R, top_k, dtype=torch.int32, device=scores.device)
    val = torch.empty(R, top_k, device=scores.device) if with_scores else None
    ip, it = (excl.u2i_indptr, excl.u2i) if excl is not None else (None, None)
    L.call("rs_masked_topk", L.ptr(scores), n_items, R, n_items, user_base, L.ptr(ip), L.ptr(it),
           top_k, L.ptr(idx), L.ptr(val), L.stream_ptr(scores.device))
    return (idx, val) if with_scores else idx


def recommend(full_graph: HeteroGraph, top_k: int, item_reprs: torch.Tensor,
              user2item_etype=None, utype=None, timestamp: str = "timestamp",
              batch_size: int = 32):
    L.require_device(item_reprs, "item_reprs")
    reprs = item_reprs.float().contiguous()
    n_users, n_items = full_graph.n_users, reprs.shape[0]
    latest = latest_items(full_graph, timestamp)
    rows = max(batch_size, min(n_users, _SCORE_CHUNK_BYTES // (4 * n_items)))
    recs = torch.empty(n_users, top_k, dtype=torch.int32, device=reprs.device)
    for b0 in range(0, n_users, rows):
        b1 = min(n_users, b0 + rows)
        scores = torch.matmul(reprs[latest[b0:b1].long()], reprs.t())
        recs[b0:b1] = masked_topk(scores, top_k, b0, full_graph)
    return recs


def hit_rate_eval(recommendations: torch.Tensor, ground_truth) -> float:
    """ground_truth: scipy sparse (n_users, n_items), e.g. val_matrix.tocsr()."""
    L.require_device(recommendations, "recommendations")
    csr = ground_truth.tocsr()
    csr.sort_indices()
    dev = recommendations.device
    indptr = torch.from_numpy(csr.indptr.astype(np.int64)).to(dev)
    items = torch.from_numpy(csr.indices.astype(np.int32)).to(dev)
    recs = recommendations.to(torch.int32).contiguous()
    U, K = recs.shape
    hit = torch.empty(U, dtype=torch.int32, device=dev)
    L.call("rs_hit_flags", L.ptr(recs), U, K, 0, L.ptr(indptr), L.ptr(items), L.ptr(hit),
           L.stream_ptr(dev))
    return float(hit.float().mean())
