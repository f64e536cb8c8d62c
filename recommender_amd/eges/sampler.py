"""EGES training-pair stream on the device (eges/data_loader.py:28-62).

train_example_generator draws one seed item, walks it (dgl random_walk, prob='weight', length
10), turns the trace into skip-gram couples (keras skipgrams, window 5, no negatives) and gives
every couple num_ns log-uniform negatives (log_uniform_candidate_sampler, unique=True). Here a
refill does that for `walks_per_refill` seeds at once with three kernels:

  rs_eges_walks          seeds + weighted walks    (Philox-keyed per walk and hop)
  rs_skipgram_pairs      couples, compacted in enumeration order by a device scan
  rs_log_uniform_sample  num_ns distinct classes per couple (host-built uint32 CDF table)

One host sync per refill (the couple count sizes the outputs). Entries ≤ 0 of a trace (OOV 0,
the walk's -1 padding after a dead end) make no couple — the reference would feed -1 to its
embedding gather. Batches come out in enumeration order; the reference's shuffles
(skipgrams(shuffle=True), Dataset.shuffle) only permute the stream.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _lib as L


def skipgram_slots(length: int, window: int) -> int:
    """Couples one trace of `length` entries can give (every i, every j ≠ i in its window)."""
    return sum(min(length, i + window + 1) - max(0, i - window) - 1 for i in range(length))


def log_uniform_cdf(range_max: int) -> np.ndarray:
    """cdf[k] = floor(P(class ≤ k) · 2^32) with P(class ≤ k) = log(k+2) / log(range_max+1)."""
    p = np.log(np.arange(2, range_max + 2, dtype=np.float64)) / np.log(range_max + 1.0)
    return np.minimum(np.floor(p * 4294967296.0), 4294967295.0).astype(np.uint32)


class EGESPairSampler:
    def __init__(self, indptr, indices, weights, n_items: int, item2cat=None, item2brand=None,
                 walk_length: int = 10, window: int = 5, num_ns: int = 5, seed: int = 4,
                 walks_per_refill: int = 4096, rank: int = 0, world: int = 1, device="cuda"):
        dev = torch.device(device)
        self.device = dev
        self.indptr = torch.as_tensor(indptr, dtype=torch.int64).to(dev).contiguous()
        self.indices = torch.as_tensor(indices, dtype=torch.int32).to(dev).contiguous()
        w = torch.as_tensor(weights, dtype=torch.float32).to(dev).contiguous()
        n_nodes = self.indptr.numel() - 1
        if n_nodes < n_items or self.indices.numel() != w.numel():
            raise ValueError("EGESPairSampler: CSR must cover n_items nodes with one weight per edge")
        self.cumw = torch.empty(w.numel(), dtype=torch.float64, device=dev)
        L.call("rs_csr_weight_prefix", L.ptr(self.indptr), L.ptr(w), n_nodes, L.ptr(self.cumw),
               L.stream_ptr(dev))
        self.cdf = torch.from_numpy(log_uniform_cdf(n_items).view(np.int32)).to(dev)
        self.item2cat = None if item2cat is None else torch.as_tensor(item2cat).to(dev).int()
        self.item2brand = None if item2brand is None else torch.as_tensor(item2brand).to(dev).int()
        self.n_items, self.length, self.window, self.num_ns = n_items, walk_length, window, num_ns
        self.seed, self.walks_per_refill, self.rank, self.world = seed, walks_per_refill, rank, world
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.refills = 0
        self._target = torch.empty(0, dtype=torch.int32, device=dev)
        self._context = torch.empty(0, 1 + num_ns, dtype=torch.int32, device=dev)
        self._label = torch.zeros(0, 1 + num_ns, device=dev)

    # -- the three stages (also the parity-test surface) ---------------------------------
    def walks(self, n_walks: int, step: int, walk_base: int = 0) -> torch.Tensor:
        tr = torch.empty(n_walks, self.length + 1, dtype=torch.int32, device=self.device)
        L.call("rs_eges_walks", L.ptr(self.indptr), L.ptr(self.indices), L.ptr(self.cumw),
               self.n_items, walk_base, n_walks, self.length, self.seed, step & 0xFFFFFFFF,
               L.ptr(tr), L.stream_ptr(self.device))
        return tr

    def skipgrams(self, traces: torch.Tensor):
        n, ln = traces.shape
        ws = torch.empty(L.lib().rs_skipgram_workspace_size(n, ln, self.window), dtype=torch.uint8,
                         device=self.device)
        cap = max(1, n * skipgram_slots(ln, self.window))
        tgt = torch.empty(cap, dtype=torch.int32, device=self.device)
        ctx = torch.empty(cap, dtype=torch.int32, device=self.device)
        cnt = torch.zeros(1, dtype=torch.int32, device=self.device)
        L.call("rs_skipgram_pairs", L.ptr(traces.contiguous()), n, ln, self.window, L.ptr(tgt),
               L.ptr(ctx), L.ptr(cnt), L.ptr(ws), ws.numel(), L.stream_ptr(self.device))
        m = int(cnt.item())
        return tgt[:m], ctx[:m]

    def negatives(self, n_pairs: int, step: int, pair_base: int = 0) -> torch.Tensor:
        out = torch.empty(n_pairs, self.num_ns, dtype=torch.int32, device=self.device)
        L.call("rs_log_uniform_sample", L.ptr(self.cdf), self.n_items, pair_base, n_pairs,
               self.num_ns, self.seed, step & 0xFFFFFFFF, L.ptr(out), L.ptr(self.err),
               L.stream_ptr(self.device))
        return out

    # -- stream ---------------------------------------------------------------------------
    def refill(self):
        """Rank r of `world` draws walks [r·W, (r+1)·W) of refill `refills` (W = walks_per_refill),
        so the ranks together sample what one process would with world·W walks."""
        w = self.walks_per_refill
        tr = self.walks(w, self.refills, walk_base=self.rank * w)
        tgt, ctx = self.skipgrams(tr)
        neg = self.negatives(tgt.numel(), self.refills, pair_base=self.rank * w * skipgram_slots(self.length + 1, self.window))
        self.refills += 1
        self._target = torch.cat([self._target, tgt])
        self._context = torch.cat([self._context, torch.cat([ctx[:, None], neg], 1)])

    def next_batch(self, batch: int, model_type: str = "EGES"):
        """(target [B,1], cat [B,1], brand [B,1], context [B,1+num_ns], label [B,1+num_ns]) —
        the train dataset's element shapes (eges/data_loader.py:94-100) batched; BGE drops cat
        and brand."""
        while self._target.numel() < batch:
            self.refill()
        t, self._target = self._target[:batch], self._target[batch:]
        c, self._context = self._context[:batch], self._context[batch:]
        if self._label.shape[0] != batch:
            self._label = torch.zeros(batch, 1 + self.num_ns, device=self.device)
            self._label[:, 0] = 1.0
        t = t[:, None]
        if model_type == "BGE":
            return t, c, self._label
        if self.item2cat is None or self.item2brand is None:
            raise ValueError("GES/EGES batches need item2cat and item2brand")
        return t, self.item2cat[t], self.item2brand[t], c, self._label
