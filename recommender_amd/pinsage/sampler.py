"""Device sampling for PinSage through the C ABI.

item2item_batch_sampler  ← pinsage/train/data_loader.py:6-18   (rs_item_pairs)
PinSageSampler           ← pinsage/train/data_loader.py:21-51  (rs_pair_set_build,
                           rs_pinsage_neighbors, rs_unique_first, rs_pinsage_block)

Every draw is keyed by (seed, step, subject) — pair index for the pair sampler, (item, walk,
layer) for the neighbour walks — so a batch sharded over ranks samples exactly what one rank
would. Host syncs per step: the valid-pair count, the seed count and each
layer's src count (tensor shapes).

Sync-free form (`sample_pairs_static` + `sample_static`, used by PinSageStep.capture): every
tensor is capacity-shaped and lives in the sampler's persistent buffers (same addresses every
call, so a HIP graph captured over one batch reads the next), the live counts stay on the
device, and padding is -1 ids / empty CSR rows. Capacities: pairs B, seeds S0 = min(3B, items),
layer sources min(cap_dst·(1+k), items). The live part equals the dynamic form bit for bit.
"""
from __future__ import annotations

import torch

from .. import _lib as L
from .graph import Block, HeteroGraph, PairGraph


class _Scratch:
    def __init__(self):
        self.bufs = {}

    def get(self, name, nbytes, device):
        b = self.bufs.get(name)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
            self.bufs[name] = b
        return b


def item_pairs(g: HeteroGraph, batch: int, seed: int, step: int, pair_base: int = 0,
               scratch: _Scratch | None = None):
    dev = g.device
    heads, pos, neg = (torch.empty(batch, dtype=torch.int32, device=dev) for _ in range(3))
    n_valid = torch.zeros(1, dtype=torch.int32, device=dev)
    scratch = scratch or _Scratch()
    ws = scratch.get("pairs", L.lib().rs_item_pairs_workspace_size(batch), dev)
    L.call("rs_item_pairs", *(L.ptr(t) for t in g.csr_args()), g.n_items, pair_base, batch,
           seed, step & 0xFFFFFFFF, L.ptr(heads), L.ptr(pos), L.ptr(neg), L.ptr(n_valid),
           L.ptr(ws), ws.numel(), L.stream_ptr(dev))
    n = int(n_valid.item())
    return heads[:n], pos[:n], neg[:n]


def item2item_batch_sampler(g: HeteroGraph, utype: str, itype: str, batch_size: int,
                            seed: int = 4, rank: int = 0, world: int = 1):
    """Yields (heads, pos_tails, neg_tails) int32 device tensors forever
    (pinsage/train/data_loader.py:6-18). With world > 1, rank r draws pairs
    [r*batch_size, (r+1)*batch_size) of the global batch of world*batch_size."""
    scratch = _Scratch()
    step = 0
    while True:
        yield item_pairs(g, batch_size, seed, step, rank * batch_size, scratch)
        step += 1


def _pow2_above(n: int) -> int:
    c = 1
    while c <= n:
        c <<= 1
    return c


class PinSageSampler:
    def __init__(self, g: HeteroGraph, itype: str, utype: str, num_layers: int,
                 random_walk_length: int, num_random_walks: int, termination_prob: float,
                 num_neighbors: int, weight_column: str = "weight", seed: int = 4):
        """Same argument order as pinsage/train/data_loader.py:22-27 (random_walk_length is
        PinSAGESampler's num_traversals)."""
        if not 1 <= num_random_walks <= 64 or not 1 <= random_walk_length <= 8:
            raise ValueError("num_random_walks must be in [1, 64], random_walk_length in [1, 8]")
        self.g = g
        self.itype, self.utype = itype, utype
        self.num_layers = num_layers
        self.num_traversals = random_walk_length
        self.num_random_walks = num_random_walks
        self.termination_prob = float(termination_prob)
        self.num_neighbors = num_neighbors
        self.weight_column = weight_column
        self.seed = int(seed)
        self.step = 0
        self.scratch = _Scratch()
        self.err_flag = torch.zeros(1, dtype=torch.int32, device=g.device)

    # -- pieces ------------------------------------------------------------------------------
    def _exclusion(self, heads, pos_tails, neg_tails):
        dev = self.g.device
        src = torch.cat([heads, heads]).to(torch.int32).contiguous()
        dst = torch.cat([pos_tails, neg_tails]).to(torch.int32).contiguous()
        cap = _pow2_above(2 * src.numel() + 1)
        table = torch.full((cap,), -1, dtype=torch.int64, device=dev)
        L.call("rs_pair_set_build", L.ptr(src), L.ptr(dst), src.numel(), L.ptr(table), cap,
               L.stream_ptr(dev))
        return table, cap

    def neighbors(self, dst_nodes: torch.Tensor, layer: int, excl=None, step: int | None = None):
        dev = self.g.device
        n, k = dst_nodes.numel(), self.num_neighbors
        nbr = torch.empty(n, k, dtype=torch.int32, device=dev)
        cnt = torch.empty(n, k, dtype=torch.int32, device=dev)
        table, cap = excl if excl is not None else (None, 0)
        L.call("rs_pinsage_neighbors", *(L.ptr(t) for t in self.g.csr_args()),
               L.ptr(dst_nodes), n, self.num_random_walks, self.num_traversals,
               self.termination_prob, self.seed, (self.step if step is None else step) & 0xFFFFFFFF,
               layer, k, L.ptr(table), cap, L.ptr(nbr), L.ptr(cnt), L.stream_ptr(dev))
        return nbr, cnt

    def unique_first(self, ids: torch.Tensor, n_nodes: int):
        dev = ids.device
        n = ids.numel()
        uniq = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        local = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        n_unique = torch.zeros(1, dtype=torch.int32, device=dev)
        ws = self.scratch.get("uniq", L.lib().rs_unique_first_workspace_size(n_nodes, n), dev)
        L.call("rs_unique_first", L.ptr(ids), n, n_nodes, L.ptr(uniq), L.ptr(local),
               L.ptr(n_unique), L.ptr(self.err_flag), L.ptr(ws), ws.numel(), L.stream_ptr(dev))
        return uniq, local[:n], n_unique

    def to_block(self, dst_nodes: torch.Tensor, nbr: torch.Tensor, cnt: torch.Tensor) -> Block:
        dev = self.g.device
        n_dst, k = nbr.shape
        ids = torch.cat([dst_nodes.to(torch.int32), nbr.reshape(-1)])
        uniq, local, n_unique = self.unique_first(ids, self.g.n_items)
        n_src = int(n_unique.item())
        cap = n_dst * k
        nbr_local = local[n_dst:].contiguous()
        indptr = torch.empty(n_dst + 1, dtype=torch.int32, device=dev)
        edge_src = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
        edge_dst = torch.empty_like(edge_src)
        edge_w = torch.empty(max(cap, 1), dtype=torch.float32, device=dev)
        n_edges = torch.zeros(1, dtype=torch.int32, device=dev)
        t_indptr = torch.empty(n_src + 1, dtype=torch.int32, device=dev)
        t_edge = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
        ws = self.scratch.get("block", L.lib().rs_pinsage_block_workspace_size(n_dst, k), dev)
        L.call("rs_pinsage_block", L.ptr(nbr_local), L.ptr(cnt), n_dst, k, n_src, L.ptr(indptr),
               L.ptr(edge_src), L.ptr(edge_dst), L.ptr(edge_w), L.ptr(n_edges), L.ptr(t_indptr),
               L.ptr(t_edge), L.ptr(ws), ws.numel(), L.stream_ptr(dev))
        return Block(uniq[:n_src], n_dst, indptr, edge_src, edge_dst, edge_w, n_edges, t_indptr,
                     t_edge)

    # -- reference surface -----------------------------------------------------------------------
    def generate_blocks(self, seeds, heads=None, pos_tails=None, neg_tails=None):
        """data_loader.py:29-43: per layer frontier = sampler(dst), leak edges removed,
        to_block; blocks[0] is the outermost layer."""
        L.require_device(seeds, "seeds")
        excl = self._exclusion(heads, pos_tails, neg_tails) if heads is not None else None
        blocks = []
        dst = seeds.to(torch.int32).contiguous()
        for layer in range(self.num_layers):
            nbr, cnt = self.neighbors(dst, layer, excl)
            block = self.to_block(dst, nbr, cnt)
            dst = block.src_nodes
            blocks.insert(0, block)
        self.step += 1
        return blocks

    def sample_from_item_pairs(self, heads, pos_tails, neg_tails, itype=None):
        """data_loader.py:45-51: compact the pos/neg pair graphs (seed order = first
        appearance over heads, pos_tails, neg_tails), then the blocks."""
        n = heads.numel()
        ids = torch.cat([heads, pos_tails, neg_tails]).to(torch.int32).contiguous()
        seeds, local, n_seeds = self.unique_first(ids, self.g.n_items)
        seeds = seeds[: int(n_seeds.item())]
        pos_graph = PairGraph(local[:n], local[n:2 * n], seeds)
        neg_graph = PairGraph(local[:n], local[2 * n:], seeds)
        blocks = self.generate_blocks(seeds, heads, pos_tails, neg_tails)
        return pos_graph, neg_graph, blocks

    # -- capacity-shaped, sync-free batches ----------------------------------------------------
    def _buf(self, name, shape, dtype):
        """Persistent device buffer (allocated once per name / shape / dtype)."""
        if not hasattr(self, "_static"):
            self._static = {}
        key = (name, tuple(shape), dtype)
        t = self._static.get(key)
        if t is None:
            t = torch.empty(shape, dtype=dtype, device=self.g.device)
            self._static[key] = t
        return t

    def _unique_static(self, name, ids, cap):
        """rs_unique_first into persistent buffers: (uniq [cap] padded with -1 past the device
        count, local [n] (-1 for ids < 0), count [1] device)."""
        n = ids.numel()
        uniq = self._buf(name + ".uniq", (n,), torch.int32)
        uniq.fill_(-1)
        local = self._buf(name + ".local", (n,), torch.int32)
        count = self._buf(name + ".n", (1,), torch.int32)
        count.zero_()
        ws = self.scratch.get("uniq." + name, L.lib().rs_unique_first_workspace_size(
            self.g.n_items, n), ids.device)
        L.call("rs_unique_first", L.ptr(ids), n, self.g.n_items, L.ptr(uniq), L.ptr(local),
               L.ptr(count), L.ptr(self.err_flag), L.ptr(ws), ws.numel(), L.stream_ptr(ids.device))
        return uniq[:cap], local, count

    def sample_pairs_static(self, batch: int, seed: int, step: int, pair_base: int = 0,
                            step_dev: torch.Tensor | None = None):
        """item_pairs without the host read of the valid count: (heads, pos, neg) [batch] with
        -1 past the device count n_valid [1] (data_loader.py:6-18, dropped pairs at the end).
        step_dev ([1] int32 device): the RNG step is read from it instead (`step` ignored)."""
        dev = self.g.device
        heads, pos, neg = (self._buf(n, (batch,), torch.int32) for n in ("heads", "pos", "neg"))
        n_valid = self._buf("n_valid", (1,), torch.int32)
        n_valid.zero_()
        ws = self.scratch.get("pairs", L.lib().rs_item_pairs_workspace_size(batch), dev)
        if step_dev is None:
            L.call("rs_item_pairs", *(L.ptr(t) for t in self.g.csr_args()), self.g.n_items,
                   pair_base, batch, seed, step & 0xFFFFFFFF, L.ptr(heads), L.ptr(pos),
                   L.ptr(neg), L.ptr(n_valid), L.ptr(ws), ws.numel(), L.stream_ptr(dev))
        else:
            L.call("rs_item_pairs_at", *(L.ptr(t) for t in self.g.csr_args()), self.g.n_items,
                   pair_base, batch, seed, L.ptr(step_dev), L.ptr(heads), L.ptr(pos),
                   L.ptr(neg), L.ptr(n_valid), L.ptr(ws), ws.numel(), L.stream_ptr(dev))
        pad = self._buf("pair_pad", (batch,), torch.bool)
        torch.ge(self._arange(batch), n_valid, out=pad)
        for t in (heads, pos, neg):
            t.masked_fill_(pad, -1)
        return heads, pos, neg, n_valid

    def _arange(self, n):
        key = ("arange", (n,), torch.int32)
        if not hasattr(self, "_static") or key not in self._static:
            self._buf("arange", (n,), torch.int32).copy_(
                torch.arange(n, dtype=torch.int32, device=self.g.device))
        return self._static[key]

    def sample_static(self, heads, pos_tails, neg_tails, n_valid, step_dev=None):
        """sample_from_item_pairs on a sample_pairs_static batch, with no host sync: pair
        graphs carry `valid` / `n_valid`, blocks carry `n_dst_live`, padded src nodes are -1.
        The returned tensors are the sampler's buffers, overwritten by its next call.
        step_dev ([1] int32 device): the walks' RNG step is read from it instead of self.step
        (self.step still advances on the host)."""
        B = heads.numel()
        n_items, k = self.g.n_items, self.num_neighbors
        ids = self._buf("pair_ids", (3 * B,), torch.int32)
        torch.cat([heads, pos_tails, neg_tails], out=ids)
        cap = min(3 * B, n_items)
        seeds, local, n_seeds = self._unique_static("seeds", ids, cap)
        valid = self._buf("pair_valid", (B,), torch.bool)
        torch.ge(heads, 0, out=valid)
        pos_graph = PairGraph(local[:B], local[B:2 * B], seeds, valid, n_valid)
        neg_graph = PairGraph(local[:B], local[2 * B:], seeds, valid, n_valid)
        # leak-edge exclusion set (padding pairs are skipped by the build kernel)
        esrc = self._buf("excl_src", (2 * B,), torch.int32)
        edst = self._buf("excl_dst", (2 * B,), torch.int32)
        torch.cat([heads, heads], out=esrc)
        torch.cat([pos_tails, neg_tails], out=edst)
        ecap = _pow2_above(4 * B + 1)
        table = self._buf("excl_table", (ecap,), torch.int64)
        table.fill_(-1)
        L.call("rs_pair_set_build", L.ptr(esrc), L.ptr(edst), 2 * B, L.ptr(table), ecap,
               L.stream_ptr(self.g.device))
        blocks = []
        dst, n_dst = seeds, n_seeds
        for layer in range(self.num_layers):
            blocks.insert(0, self._block_static(layer, dst, n_dst, (table, ecap), step_dev))
            dst, n_dst = blocks[0].src_nodes, blocks[0].n_src_live
        self.step += 1
        return pos_graph, neg_graph, blocks

    def _block_static(self, layer, dst, n_dst, excl, step_dev=None):
        dev = self.g.device
        cap_dst, k = dst.numel(), self.num_neighbors
        pre = f"l{layer}."
        nbr = self._buf(pre + "nbr", (cap_dst, k), torch.int32)
        cnt = self._buf(pre + "cnt", (cap_dst, k), torch.int32)
        table, ecap = excl
        if step_dev is None:
            L.call("rs_pinsage_neighbors", *(L.ptr(t) for t in self.g.csr_args()), L.ptr(dst),
                   cap_dst, self.num_random_walks, self.num_traversals, self.termination_prob,
                   self.seed, self.step & 0xFFFFFFFF, layer, k, L.ptr(table), ecap, L.ptr(nbr),
                   L.ptr(cnt), L.stream_ptr(dev))
        else:
            L.call("rs_pinsage_neighbors_at", *(L.ptr(t) for t in self.g.csr_args()), L.ptr(dst),
                   cap_dst, self.num_random_walks, self.num_traversals, self.termination_prob,
                   self.seed, L.ptr(step_dev), layer, k, L.ptr(table), ecap, L.ptr(nbr),
                   L.ptr(cnt), L.stream_ptr(dev))
        ids = self._buf(pre + "ids", (cap_dst * (1 + k),), torch.int32)
        torch.cat([dst, nbr.reshape(-1)], out=ids)
        cap_src = min(cap_dst * (1 + k), self.g.n_items)
        src, local, n_src = self._unique_static(pre + "src", ids, cap_src)
        nbr_local = local[cap_dst:]
        E = cap_dst * k
        indptr = self._buf(pre + "indptr", (cap_dst + 1,), torch.int32)
        edge_src = self._buf(pre + "edge_src", (E,), torch.int32)
        edge_dst = self._buf(pre + "edge_dst", (E,), torch.int32)
        edge_w = self._buf(pre + "edge_w", (E,), torch.float32)
        n_edges = self._buf(pre + "n_edges", (1,), torch.int32)
        n_edges.zero_()
        t_indptr = self._buf(pre + "t_indptr", (cap_src + 1,), torch.int32)
        t_edge = self._buf(pre + "t_edge", (E,), torch.int32)
        ws = self.scratch.get("block." + pre, L.lib().rs_pinsage_block_workspace_size(cap_dst, k),
                              dev)
        L.call("rs_pinsage_block", L.ptr(nbr_local), L.ptr(cnt), cap_dst, k, cap_src,
               L.ptr(indptr), L.ptr(edge_src), L.ptr(edge_dst), L.ptr(edge_w), L.ptr(n_edges),
               L.ptr(t_indptr), L.ptr(t_edge), L.ptr(ws), ws.numel(), L.stream_ptr(dev))
        return Block(src, cap_dst, indptr, edge_src, edge_dst, edge_w, n_edges, t_indptr, t_edge,
                     n_dst_live=n_dst, n_src_live=n_src)
