"""Oracle: PinSage sampling, block construction and the Convolve / SageNet forward.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py; parity unpinned — DGL 0.6.1 is absent, so
the sampler semantics are restated from its documented behaviour [3p]).

References (read as text):
  a-14 item2item_batch_sampler           pinsage/train/data_loader.py:6-18
  a-15 PinSageSampler.generate_blocks    pinsage/train/data_loader.py:21-43
       (dgl.sampling.PinSAGESampler :26-27 → random_walk + to_simple(return_counts) +
        select_topk; remove_edges :34-39; to_block :40)
  a-16 sample_from_item_pairs            pinsage/train/data_loader.py:45-51 (compact_graphs)
  a-17 FeatureProjector                  pinsage/train/layers.py:49-81
  a-18 Convolve                          pinsage/train/layers.py:7-30
  a-19 SageNet / scorer / margin loss    pinsage/train/layers.py:33-46,
                                         pinsage/train/model.py:14-39, pinsage/train/train.py:17-20

Random draws follow the engine's declared scheme (include/recsys_hip.h, PinSage section):
Philox4x32-10 with key (seed_lo, seed_hi ^ purpose), counter (a, b, step, draw // 4), word
draw % 4; bounded ints (r * n) >> 32. Choices the DGL sources leave open and this restatement
fixes: top-k ties by smaller item id; compact/to_block node order = first appearance;
restart: the trace ends after a transition whose stop draw < floor(p * 2^32).
"""
from __future__ import annotations

import numpy as np

PURPOSE_WALK = 0x100  # +1: stop draws
PURPOSE_PAIR = 0x200
PURPOSE_PAIR_WALK = 0x300

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr: np.ndarray, k0, k1) -> np.ndarray:
    """Philox4x32-10 (Salmon et al., SC'11) over rows of ctr [n, 4] uint32 → [n, 4] uint32.
    k0 / k1 may be scalars or [n] arrays."""
    c = np.asarray(ctr, dtype=np.uint64).reshape(-1, 4).copy()
    k0 = np.asarray(k0, dtype=np.uint64) & _MASK32
    k1 = np.asarray(k1, dtype=np.uint64) & _MASK32
    x, y, z, w = c[:, 0], c[:, 1], c[:, 2], c[:, 3]
    for _ in range(10):
        p0 = _M0 * x
        p1 = _M1 * z
        x, y, z, w = ((p1 >> np.uint64(32)) ^ y ^ k0, p1 & _MASK32,
                      (p0 >> np.uint64(32)) ^ w ^ k1, p0 & _MASK32)
        k0 = (k0 + np.uint64(_W0)) & _MASK32
        k1 = (k1 + np.uint64(_W1)) & _MASK32
    return np.stack([x, y, z, w], 1).astype(np.uint32)


def draw(seed: int, purpose: int, a, b, step: int, idx) -> np.ndarray:
    a = np.asarray(a, dtype=np.int64).astype(np.uint32)
    n = a.size
    b = np.broadcast_to(np.asarray(b, dtype=np.int64).astype(np.uint32), (n,))
    idx = np.broadcast_to(np.asarray(idx, dtype=np.int64), (n,))
    ctr = np.stack([a.reshape(-1), b, np.full(n, step & 0xFFFFFFFF, np.uint32),
                    (idx >> 2).astype(np.uint32)], 1)
    k0 = seed & 0xFFFFFFFF
    k1 = ((seed >> 32) & 0xFFFFFFFF) ^ purpose
    r = philox4x32_10(ctr, k0, k1)
    return r[np.arange(n), idx & 3]


def bounded(r: np.ndarray, n) -> np.ndarray:
    return ((r.astype(np.uint64) * np.asarray(n, dtype=np.uint64)) >> np.uint64(32)).astype(np.int64)


def stop_threshold(p: float) -> int:
    p = float(np.float32(p))
    if not p > 0.0:
        return 0
    t = np.floor(p * 4294967296.0)
    return 0xFFFFFFFF if t >= 4294967295.0 else int(t)


class BipartiteGraph:
    """item↔user CSR pair (numpy): i2u_indptr [n_items+1], i2u [E] user ids, u2i_indptr
    [n_users+1], u2i [E] item ids (the heterograph of pinsage/train/graph_builder.py)."""

    def __init__(self, i2u_indptr, i2u, u2i_indptr, u2i):
        self.i2u_indptr = np.asarray(i2u_indptr, np.int64)
        self.i2u = np.asarray(i2u, np.int64)
        self.u2i_indptr = np.asarray(u2i_indptr, np.int64)
        self.u2i = np.asarray(u2i, np.int64)
        self.n_items = self.i2u_indptr.size - 1
        self.n_users = self.u2i_indptr.size - 1

    @staticmethod
    def from_edges(users, items, n_users, n_items):
        users = np.asarray(users, np.int64)
        items = np.asarray(items, np.int64)
        o = np.lexsort((items, users))
        u2i_indptr = np.zeros(n_users + 1, np.int64)
        np.add.at(u2i_indptr, users + 1, 1)
        o2 = np.lexsort((users, items))
        i2u_indptr = np.zeros(n_items + 1, np.int64)
        np.add.at(i2u_indptr, items + 1, 1)
        return BipartiteGraph(np.cumsum(i2u_indptr), users[o2], np.cumsum(u2i_indptr), items[o])


def _hop(ptr, nbr, node, r):
    out = np.full(node.shape, -1, np.int64)
    alive = node >= 0
    nd = np.where(alive, node, 0)
    lo = ptr[nd]
    deg = ptr[nd + 1] - lo
    ok = alive & (deg > 0)
    k = bounded(r, np.maximum(deg, 1))
    out[ok] = nbr[(lo + k)[ok]]
    return out


def _metapath(g: BipartiteGraph, start, T, restart_prob, seed, purpose, a, b, step):
    """[n, 2T] visited nodes (hop h → column h), -1 after the trace ends."""
    start = np.asarray(start, np.int64)
    thr = stop_threshold(restart_prob)
    node = start.copy()
    out = np.full((start.size, 2 * T), -1, np.int64)
    for h in range(2 * T):
        r = draw(seed, purpose, a, b, step, h)
        node = _hop(g.u2i_indptr, g.u2i, node, r) if h & 1 else _hop(g.i2u_indptr, g.i2u, node, r)
        out[:, h] = node
        if thr:
            stop = (node >= 0) & (draw(seed, purpose + 1, a, b, step, h) < thr)
            node = np.where(stop, -1, node)
    return out


def metapath_walk(g: BipartiteGraph, seeds, num_walks, n_traversals, restart_prob, seed, step,
                  layer):
    """dgl.sampling.random_walk(g, repeat(seeds, num_walks), metapath=[i→u, u→i]*T) [3p]:
    traces [n*num_walks, 2T+1] (trace s*num_walks + j = walk j of seed s)."""
    seeds = np.asarray(seeds, np.int64)
    start = np.repeat(seeds, num_walks)
    j = np.tile(np.arange(num_walks, dtype=np.int64), seeds.size)
    vis = _metapath(g, start, n_traversals, restart_prob, seed, PURPOSE_WALK, start,
                    j | (layer << 16), step)
    return np.concatenate([start[:, None], vis], 1)


def item_pairs(g: BipartiteGraph, pair_base, batch, seed, step):
    """item2item_batch_sampler (data_loader.py:6-18): heads, neg ~ U[0, n_items); pos = item
    two hops along [item→user, user→item] from head (:13); keep pos != -1 (:15-18)."""
    gi = (pair_base + np.arange(batch, dtype=np.int64)) & 0xFFFFFFFF
    ctr = np.stack([gi, np.zeros(batch, np.int64), np.full(batch, step & 0xFFFFFFFF),
                    np.zeros(batch, np.int64)], 1)
    r = philox4x32_10(ctr, seed & 0xFFFFFFFF, ((seed >> 32) & 0xFFFFFFFF) ^ PURPOSE_PAIR)
    heads = bounded(r[:, 0], g.n_items)
    neg = bounded(r[:, 1], g.n_items)
    pos = _metapath(g, heads, 1, 0.0, seed, PURPOSE_PAIR_WALK, gi, 0, step)[:, 1]
    m = pos != -1
    return heads[m], pos[m], neg[m]


def pinsage_neighbors(g: BipartiteGraph, seeds, num_walks, n_traversals, restart_prob,
                      num_neighbors, seed, step, layer, exclude=None):
    """PinSAGESampler(g, item, user, T, p, num_walks, k) [3p DGL 0.6.1] (data_loader.py:26-27)
    then frontier.remove_edges of (head → tail) pairs (:34-39).

    RandomWalkNeighborSampler: traces of repeat(seeds, num_walks); visited items at every
    traversal end (columns 2, 4, ..) are edges src=item → dst=seed; to_simple merges repeats
    into one edge with weight = count; select_topk keeps the k heaviest in-edges per dst
    (ties: smaller src first). Removal happens after top-k, leaving the slot empty.
    exclude: set of (src, dst) item pairs. Returns nbr, cnt [n_seeds, k] (-1 / 0 = empty)."""
    seeds = np.asarray(seeds, np.int64)
    tr = metapath_walk(g, seeds, num_walks, n_traversals, restart_prob, seed, step, layer)
    visits = tr[:, 2::2].reshape(seeds.size, num_walks * n_traversals)
    k = num_neighbors
    nbr = np.full((seeds.size, k), -1, np.int64)
    cnt = np.zeros((seeds.size, k), np.int64)
    for s in range(seeds.size):
        counts = {}
        for v in visits[s]:
            if v >= 0:
                counts[int(v)] = counts.get(int(v), 0) + 1
        ranked = sorted(counts.items(), key=lambda kv: (-kv[1], kv[0]))[:k]
        for r, (v, c) in enumerate(ranked):
            if exclude is not None and (v, int(seeds[s])) in exclude:
                continue
            nbr[s, r], cnt[s, r] = v, c
    return nbr, cnt


def unique_first(ids):
    """Distinct ids >= 0 in order of first appearance + each position's index (-1 for < 0)."""
    ids = np.asarray(ids, np.int64).reshape(-1)
    first = {}
    uniq = []
    local = np.full(ids.size, -1, np.int64)
    for i, v in enumerate(ids.tolist()):
        if v < 0:
            continue
        if v not in first:
            first[v] = len(uniq)
            uniq.append(v)
        local[i] = first[v]
    return np.asarray(uniq, np.int64), local


class Block:
    """dgl.to_block result: src nodes (dst nodes first), CSR by dst and its transpose."""

    def __init__(self, src_nodes, n_dst, indptr, edge_src, edge_dst, edge_w):
        self.src_nodes = src_nodes
        self.n_dst = n_dst
        self.indptr = indptr
        self.edge_src = edge_src
        self.edge_dst = edge_dst
        self.edge_w = edge_w
        self.n_src = src_nodes.size
        o = np.argsort(edge_src, kind="stable")
        self.t_edge = o
        self.t_indptr = np.searchsorted(edge_src[o], np.arange(self.n_src + 1), side="left")


def to_block(dst_nodes, nbr, cnt):
    """dgl.to_block(frontier, dst_nodes) (data_loader.py:40)."""
    dst_nodes = np.asarray(dst_nodes, np.int64)
    n_dst, k = nbr.shape
    uniq, local = unique_first(np.concatenate([dst_nodes, nbr.reshape(-1)]))
    nl = local[n_dst:].reshape(n_dst, k)
    valid = nl >= 0
    counts = valid.sum(1)
    indptr = np.zeros(n_dst + 1, np.int64)
    indptr[1:] = np.cumsum(counts)
    edge_src = nl[valid]
    edge_dst = np.repeat(np.arange(n_dst), counts)
    edge_w = cnt[valid].astype(np.float32)
    return Block(uniq, n_dst, indptr, edge_src, edge_dst, edge_w)


def sample_from_item_pairs(g: BipartiteGraph, heads, pos, neg, num_layers, num_walks,
                           n_traversals, restart_prob, num_neighbors, seed, step):
    """sample_from_item_pairs + generate_blocks (data_loader.py:29-51): seeds =
    compact_graphs node order; pos/neg edges in seed-local ids; blocks[0] = outermost layer."""
    heads, pos, neg = (np.asarray(a, np.int64) for a in (heads, pos, neg))
    seeds, local = unique_first(np.concatenate([heads, pos, neg]))
    n = heads.size
    pos_edges = (local[:n], local[n:2 * n])
    neg_edges = (local[:n], local[2 * n:])
    exclude = set(zip(heads.tolist(), pos.tolist())) | set(zip(heads.tolist(), neg.tolist()))
    blocks = []
    dst = seeds
    for layer in range(num_layers):
        nbr, cnt = pinsage_neighbors(g, dst, num_walks, n_traversals, restart_prob,
                                     num_neighbors, seed, step, layer, exclude)
        b = to_block(dst, nbr, cnt)
        blocks.insert(0, b)
        dst = b.src_nodes
    return seeds, pos_edges, neg_edges, blocks


# ---- float path (fp32 numpy; the GPU parity tests use a torch fp32 autograd restatement) --
def weighted_mean_agg(u, block: Block):
    """Convolve :17-24: nv[d] = Σ w u[src] / max(Σ w, 1)."""
    H = u.shape[1]
    nv = np.zeros((block.n_dst, H), np.float32)
    ws = np.zeros(block.n_dst, np.float32)
    for d in range(block.n_dst):
        acc = np.zeros(H, np.float32)
        w_acc = np.float32(0)
        for e in range(block.indptr[d], block.indptr[d + 1]):
            acc = acc + block.edge_w[e] * u[block.edge_src[e]]
            w_acc = np.float32(w_acc + block.edge_w[e])
        ws[d] = w_acc
        nv[d] = acc / max(w_acc, np.float32(1))
    return nv, ws


def dense(x, W, b, act=None):
    y = x.astype(np.float32) @ W.astype(np.float32) + b.astype(np.float32)
    return np.maximum(y, 0) if act == "relu" else y


def convolve(block: Block, h_src, params):
    """Convolve.call (layers.py:13-30)."""
    h_dst = h_src[:block.n_dst]
    u = dense(h_src, params["W1"], params["b1"], "relu")
    nv, _ = weighted_mean_agg(u, block)
    new = dense(np.concatenate([nv, h_dst], 1), params["W2"], params["b2"], "relu")
    return new / np.sqrt(np.sum(new.astype(np.float64) ** 2)).astype(np.float32)


def feature_projector(nodes, year, genre, tables):
    """FeatureProjector.call (layers.py:62-81): [year_emb | mean_g genre_emb[genre01] | id_emb]."""
    ye = tables["year"][year[nodes]]
    ge = tables["genre"][genre[nodes].astype(np.int64)].mean(1)
    ie = tables["id"][nodes]
    return np.concatenate([ye, ge, ie], 1).astype(np.float32)


def get_repr(blocks, year, genre, tables, conv_params, head_params):
    """PinSageModel.get_repr (model.py:32-39) → SageNet.call (layers.py:40-46)."""
    h = feature_projector(blocks[0].src_nodes, year, genre, tables)
    for b, p in zip(blocks, conv_params):
        h = convolve(b, h, p)
    h = dense(h, head_params["W1"], head_params["b1"], "relu")
    return dense(h, head_params["W2"], head_params["b2"])


def margin_loss(pos_score, neg_score, delta=1.0):
    """train.py:17-20: mean(clip(neg + delta - pos, 0, inf))."""
    return float(np.mean(np.clip(neg_score + delta - pos_score, 0, np.inf)))


# ---- evaluation (pinsage/train/evaluation.py:27-65, util.py:5-24) --------------------------
def latest_item(u2i_indptr, u2i, ts):
    """select_topk(k=1, timestamp) per user (:33-34); ties → smaller item; -1 without edges."""
    out = np.full(len(u2i_indptr) - 1, -1, np.int32)
    for u in range(len(out)):
        lo, hi = int(u2i_indptr[u]), int(u2i_indptr[u + 1])
        if hi > lo:
            t, it = ts[lo:hi], u2i[lo:hi]
            m = t == t.max()
            out[u] = it[m].min()
    return out


def masked_topk_scores(scores, excl_indptr=None, excl=None, user_base=0):
    """similarity[i, interacted] = -inf (:41-44)."""
    s = np.array(scores, np.float32, copy=True)
    if excl_indptr is not None:
        for r in range(s.shape[0]):
            u = user_base + r
            s[r, excl[excl_indptr[u]:excl_indptr[u + 1]]] = -np.inf
    return s


def masked_topk(scores, k, excl_indptr=None, excl=None, user_base=0):
    """top-k of the masked similarity rows by (score desc, item asc) (:45-46)."""
    s = masked_topk_scores(scores, excl_indptr, excl, user_base)
    out = np.empty((s.shape[0], k), np.int32)
    items = np.arange(s.shape[1])
    for r in range(s.shape[0]):
        out[r] = np.lexsort((items, -s[r].astype(np.float64)))[:k]
    return out


def hit_rate(recs, truth_indptr, truth):
    """relevance.any(axis=1).mean() (:54-65)."""
    hits = [np.isin(recs[u], truth[truth_indptr[u]:truth_indptr[u + 1]]).any()
            for u in range(len(recs))]
    return float(np.mean(hits)), np.asarray(hits, np.int32)


def split_by_time(users, ts):
    """util.py:5-24: per user sorted by time, last → test (> 1 rating), second-to-last → val
    (> 2 ratings); ties keep edge order. Returns the three sorted edge-index arrays."""
    tr, va, te = [], [], []
    for u in np.unique(users):
        e = np.nonzero(users == u)[0]
        e = e[np.argsort(ts[e], kind="stable")]
        if e.size > 1:
            te.append(e[-1])
        if e.size > 2:
            va.append(e[-2])
        tr.extend(e[: e.size - min(e.size - 1, 2)] if e.size > 1 else e)
    return np.sort(np.asarray(tr, np.int64)), np.sort(np.asarray(va, np.int64)), \
        np.sort(np.asarray(te, np.int64))


# ---- one train step on the host (torch fp32 autograd; the CPU baseline of cfg5) ------------
def torch_train_step(model_cpu, blocks, pos_edges, neg_edges, year, genre, delta=1.0):
    """pinsage/train/train.py:17-20,40-48 on the CPU: get_repr (FeatureProjector → Convolve x L →
    fc_1 / fc_2, layers.py / model.py) from a CPU-built PinSageModel's parameters and the numpy
    blocks of sample_from_item_pairs, u_dot_v scores, margin loss, and the gradients of every
    dense parameter and table (torch autograd; index_add aggregation). Used only to time the
    reference's CPU path beside the GPU step (benchmarks/bench_models.py). Returns (loss, grads)."""
    import torch

    fp = model_cpu.feature_projector
    leaves = []

    def leaf(t):
        x = t.detach().clone().requires_grad_(True)
        leaves.append(x)
        return x

    ids = torch.from_numpy(np.asarray(blocks[0].src_nodes, np.int64))
    ye = leaf(fp.year_embedding.weight)[torch.from_numpy(np.asarray(year, np.int64))[ids]]
    ge = leaf(fp.genre_embedding.weight)[torch.from_numpy(np.asarray(genre, np.int64))[ids]].mean(1)
    ie = leaf(fp.id_embedding.weight)[ids]
    h = torch.cat([ye, ge, ie], -1)
    for conv, b in zip(model_cpu.sagenet.convolves, blocks):
        h_dst = h[: b.n_dst]
        u = torch.relu(h @ leaf(conv.fc_1.kernel) + leaf(conv.fc_1.bias))
        src = torch.from_numpy(np.asarray(b.edge_src, np.int64))
        dst = torch.from_numpy(np.asarray(b.edge_dst, np.int64))
        w = torch.from_numpy(np.asarray(b.edge_w, np.float32))
        vs = torch.zeros(b.n_dst, u.shape[1]).index_add(0, dst, u[src] * w[:, None])
        ws = torch.zeros(b.n_dst).index_add(0, dst, w)
        nv = vs / torch.clamp(ws, min=1)[:, None]
        new = torch.relu(torch.cat([nv, h_dst], -1) @ leaf(conv.fc_2.kernel) + leaf(conv.fc_2.bias))
        h = new / torch.norm(new)
    s = model_cpu.sagenet
    h = torch.relu(h @ leaf(s.fc_1.kernel) + leaf(s.fc_1.bias))
    h = h @ leaf(s.fc_2.kernel) + leaf(s.fc_2.bias)

    def score(edges):
        a = torch.from_numpy(np.asarray(edges[0], np.int64))
        c = torch.from_numpy(np.asarray(edges[1], np.int64))
        return (h[a] * h[c]).sum(-1)

    loss = torch.clamp(score(neg_edges) + delta - score(pos_edges), min=0).mean()
    grads = torch.autograd.grad(loss, leaves)
    return float(loss.detach()), grads
