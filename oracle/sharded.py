"""Oracle: the row-sharded embedding step over W ranks — TEST INFRASTRUCTURE ONLY
(see oracle/__init__.py; parity unpinned).

Restates recommender_amd/sharded.py's semantics: rows dealt cyclically (owner = row % W, local
row = row // W); each rank deduplicates its gradient with the tiled fold over owner-major keys;
owners receive (local row, grad) lists rank-major, fold them with the same tiled order and
apply SGD with lr/W. The reference itself only has replicated MirroredStrategy tables
(ctr/train.py:71); the all-to-all layout is required by BASELINE.json's north star.
"""
from __future__ import annotations

import numpy as np

from .embedding import (apply_keras_adam, apply_lazy_adam, global_rows, keras_adam_coefficients,
                        segment_sum_tiled, sort_ids)


def owner_keys(rows: np.ndarray, n_rows: int, world: int):
    stride = -(-n_rows // world)
    key_space = n_rows if world == 1 else stride * world
    keys = np.where(rows < 0, key_space, (rows % world) * stride + rows // world)
    return keys, stride, key_space


def sharded_sgd_step(full_table, per_rank_ids, per_rank_grads, lr, world, slot_offsets=None,
                     global_grads=False):
    """Returns the updated full table after one sharded SGD step. global_grads: the rows are
    gradients of the global mean loss (the fused DLRM step), applied with lr as given;
    otherwise of each rank's local mean, applied with lr/W."""
    V, D = full_table.shape
    stride = -(-V // world)
    recv = [[] for _ in range(world)]  # recv[o] = list of (local rows, grads) from rank 0..W-1
    for r in range(world):
        rows = global_rows(per_rank_ids[r], V, slot_offsets)
        keys, _, key_space = owner_keys(rows, V, world)
        order = np.argsort(keys, kind="stable")
        sk = keys[order].astype(np.uint32)
        uk, ug = segment_sum_tiled(sk, order.astype(np.int32), per_rank_grads[r], key_space)
        uk = uk.astype(np.int64)
        for o in range(world):
            sel = (uk // stride) == o
            recv[o].append((uk[sel] - o * stride, ug[sel]))
    out = full_table.copy()
    lr_w = (np.float32(float(np.float32(lr)) / world) if world > 1 and not global_grads
            else np.float32(lr))
    for o in range(world):
        local = np.concatenate([x[0] for x in recv[o]])
        grads = np.concatenate([x[1] for x in recv[o]]) if local.size else np.zeros((0, D), np.float32)
        if local.size == 0:
            continue
        shard_rows = (V - o + world - 1) // world
        sr, sp, _ = sort_ids(local, shard_rows)
        ur, ug = segment_sum_tiled(sr, sp, grads, shard_rows)
        g_rows = ur.astype(np.int64) * world + o
        out[g_rows] = out[g_rows] - lr_w * ug
    return out


def sharded_owner_grads(per_rank_ids, per_rank_grads, world, n_rows, slot_offsets=None,
                        scale=True):
    """The owners' side of one sharded step (recommender_amd/sharded.py backward_exchange)
    before the optimizer: each rank folds its gradient rows per owner-major key with the tiled
    order, each owner receives the per-source (local row, grad) lists rank-major, scales them by
    float32(1/W) (world > 1, `scale`: rows of each rank's local mean loss) and folds them with
    the same tiled order over its shard. Returns, per owner o, (the shard's local rows that got a
    gradient, sorted; their folded gradients). Depends on the ids and gradient rows only, so a
    test can apply it to any compacted copy of the touched rows' optimizer state."""
    V = n_rows
    D = per_rank_grads[0].shape[1]
    stride = -(-V // world)
    recv = [[] for _ in range(world)]
    for r in range(world):
        rows = global_rows(per_rank_ids[r], V, slot_offsets)
        keys, _, key_space = owner_keys(rows, V, world)
        order = np.argsort(keys, kind="stable")
        sk = keys[order].astype(np.uint32)
        uk, ug = segment_sum_tiled(sk, order.astype(np.int32), per_rank_grads[r], key_space)
        uk = uk.astype(np.int64)
        for o in range(world):
            sel = (uk // stride) == o
            recv[o].append((uk[sel] - o * stride, ug[sel]))
    out = []
    for o in range(world):
        local = np.concatenate([x[0] for x in recv[o]])
        grads = (np.concatenate([x[1] for x in recv[o]]) if local.size
                 else np.zeros((0, D), np.float32))
        if world > 1 and scale:
            grads = grads * np.float32(1.0 / world)
        shard_rows = (V - o + world - 1) // world
        if local.size:
            sr, sp, _ = sort_ids(local, shard_rows)
            ur, ug = segment_sum_tiled(sr, sp, grads, shard_rows)
            out.append((ur.astype(np.int64), ug))
        else:
            out.append((np.zeros(0, np.int64), np.zeros((0, D), np.float32)))
    return out


def sharded_adam_step(full_table, m, v, per_rank_ids, per_rank_grads, world, step, mode,
                      lr=1e-3, slot_offsets=None):
    """One sharded lazy / Keras Adam step (recommender_amd/sharded.py backward_exchange): each
    owner scales the received per-source unique grads by float32(1/W) (world > 1), folds them
    with the tiled order and applies Adam (coefficients of 1-based `step`) to its shard. Keras
    mode is dense: every row of every shard decays m / v and moves, including shards that
    received no row this step. Returns (table, m, v) in full-slab layout."""
    V, D = full_table.shape
    c = keras_adam_coefficients(step, lr)
    owners = sharded_owner_grads(per_rank_ids, per_rank_grads, world, V, slot_offsets)
    t, m2, v2 = full_table.copy(), m.copy(), v.copy()
    for o in range(world):
        g_all = np.arange(o, V, world)  # this owner's global rows, local order
        ur, ug = owners[o]
        fn = apply_keras_adam if mode == "keras" else apply_lazy_adam
        if mode != "keras" and not ur.size:
            continue
        ts, ms, vs = fn(t[g_all], m2[g_all], v2[g_all], ur, ug, c)
        t[g_all], m2[g_all], v2[g_all] = ts, ms, vs
    return t, m2, v2
