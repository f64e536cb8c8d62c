"""eges/model.py on the engine.

DeepWalk (BGE) :20-47   hidden = input_embedding(query); logits = output rows · hidden
GES            :50-80   hidden = (id + cat + brand) / 3
EGES           :83-102  hidden = softmax(weight_embedding(item)) · [id, cat, brand]

Inputs keep the reference's batched shapes: query ids [B, 1], match ids [B, 1+num_ns] → logits
[B, 1+num_ns]; get_hidden returns [B, 1, D]. Gathers run through rs_embedding_fwd, the skip-gram
logits through the fused gather+dot rs_match_logits_*, the side pooling through rs_side_pool_*;
every table's gradient goes to the engine's sparse optimizers (IndexedSlices semantics).
Divergence: the reference's EGES.__init__ calls super().__init__() without GES's arguments and
raises TypeError as written; this EGES builds the tables the code intends.
"""
from __future__ import annotations

import torch
from torch import nn

from .. import _lib as L
from ..embedding import Embedding


class _MatchLogits(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hidden, handle, table: Embedding, match):
        L.require_device(hidden, "hidden")
        h = hidden.reshape(hidden.shape[0], -1).contiguous().float()
        B, D = h.shape
        ids = match.contiguous()
        M = ids.shape[-1]
        logits = torch.empty(B, M, device=h.device)
        L.call("rs_match_logits_fwd", L.ptr(table.weight), table.input_dim, D, L.ptr(ids),
               L.id_dtype_code(ids), M, L.ptr(h), B, L.ptr(logits), L.ptr(table.err_flag),
               L.stream_ptr(h.device))
        ctx.table = table
        ctx.shape = hidden.shape
        ctx.save_for_backward(h, ids)
        return logits

    @staticmethod
    def backward(ctx, g):
        h, ids = ctx.saved_tensors
        t = ctx.table
        B, D = h.shape
        M = ids.shape[-1]
        g = g.contiguous()
        rows = torch.empty(B * M, D, device=h.device)
        gh = torch.empty(B, D, device=h.device)
        L.call("rs_match_logits_bwd", L.ptr(t.weight), t.input_dim, D, L.ptr(ids),
               L.id_dtype_code(ids), M, L.ptr(h), L.ptr(g), B, L.ptr(rows), L.ptr(gh),
               L.stream_ptr(h.device))
        t.accumulate_grad(ids, rows)
        return gh.reshape(ctx.shape), None, None, None


def match_logits(table: Embedding, match: torch.Tensor, hidden: torch.Tensor) -> torch.Tensor:
    """tf.squeeze(tf.matmul(table(match), hidden, transpose_b=True), -1)."""
    return _MatchLogits.apply(hidden, table.grad_handle, table, match)


def _pool_layout_ok(side):
    """side [B, S, D] read in place: contiguous, or rows of D = 4k <= 128 contiguous floats at
    16-byte aligned strides (e.g. MMOE's [E, B, H] expert outputs seen as [B, E, H])."""
    if side.is_contiguous():
        return True
    B, S, D = side.shape
    return (side.stride(2) == 1 and D % 4 == 0 and D <= 128 and side.stride(0) % 4 == 0
            and side.stride(1) % 4 == 0 and side.data_ptr() % 16 == 0)


class _SidePool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, side, wlogits):
        L.require_device(side, "side")
        if not _pool_layout_ok(side):
            side = side.contiguous()
        B, S, D = side.shape
        hidden = torch.empty(B, D, device=side.device)
        attn = None
        wl = None
        if wlogits is not None:
            wl = wlogits.reshape(B, S).contiguous()
            attn = torch.empty(B, S, device=side.device)
        L.call("rs_side_pool_fwd_strided", L.ptr(side), side.stride(0), side.stride(1), L.ptr(wl),
               B, S, D, L.ptr(hidden), L.ptr(attn), L.stream_ptr(side.device))
        ctx.has_w = wlogits is not None
        ctx.wshape = None if wlogits is None else wlogits.shape
        ctx.save_for_backward(side, attn)
        return hidden.reshape(B, 1, D)

    @staticmethod
    def backward(ctx, g):
        side, attn = ctx.saved_tensors
        B, S, D = side.shape
        g = g.reshape(B, D).contiguous()
        gs = torch.empty_like(side)  # the side's layout (preserve_format keeps the permutation)
        if gs.stride() != side.stride():
            raise RuntimeError("side pool: gradient layout differs from the side rows'")
        gw = torch.empty(B, S, device=side.device) if ctx.has_w else None
        L.call("rs_side_pool_bwd_strided", L.ptr(side), side.stride(0), side.stride(1),
               L.ptr(attn), L.ptr(g), B, S, D, L.ptr(gs), L.ptr(gw), L.stream_ptr(side.device))
        return gs, (gw.reshape(ctx.wshape) if gw is not None else None)


def side_pool(side: torch.Tensor, weight_logits: torch.Tensor | None = None) -> torch.Tensor:
    """[B, S, D] → [B, 1, D]: softmax(weight_logits)-weighted (EGES) or mean (GES)."""
    return _SidePool.apply(side, weight_logits)


class Base(nn.Module):
    def evaluation(self, inputs):
        raise NotImplementedError("must implement evaluation method")

    def get_hidden(self, inputs):
        raise NotImplementedError("must implement get_hidden method")

    def tables(self):
        return [m for m in self.modules() if isinstance(m, Embedding)]


class DeepWalk(Base):
    def __init__(self, vocab_size, embedding_size, device=None, generator=None):
        super().__init__()
        self.input_embedding = Embedding(vocab_size, embedding_size, device=device,
                                         generator=generator)
        self.output_embedding = Embedding(vocab_size, embedding_size, device=device,
                                          generator=generator)

    def forward(self, inputs):
        query, match = inputs
        hidden = self.input_embedding(query)  # [B, 1, D]
        return match_logits(self.output_embedding, match, hidden)

    call = forward

    def evaluation(self, inputs):
        q, m, n = inputs
        return self.get_hidden(q), self.get_hidden(m), self.get_hidden(n)

    def get_hidden(self, inputs):
        return self.input_embedding(inputs)


class GES(Base):
    def __init__(self, id_vocab_size, cat_vocab_size, brand_vocab_size, embedding_size,
                 device=None, generator=None):
        super().__init__()
        kw = dict(device=device, generator=generator)
        self.id_embedding = Embedding(id_vocab_size, embedding_size, **kw)
        self.cat_embedding = Embedding(cat_vocab_size, embedding_size, **kw)
        self.brand_embedding = Embedding(brand_vocab_size, embedding_size, **kw)
        self.output_embedding = Embedding(id_vocab_size, embedding_size, **kw)

    def forward(self, inputs):
        query_item_id, query_cat_id, query_brand_id, match = inputs
        hidden = self.get_hidden((query_item_id, query_cat_id, query_brand_id))
        return match_logits(self.output_embedding, match, hidden)

    call = forward

    def evaluation(self, inputs):
        q = self.get_hidden(tuple(inputs[0:3]))
        p = self.get_hidden(tuple(inputs[3:6]))
        n = self.get_hidden(tuple(inputs[6:9]))
        return q, p, n

    def _side(self, inputs):
        item, cat, brand = inputs
        return torch.cat([self.id_embedding(item), self.cat_embedding(cat),
                          self.brand_embedding(brand)], dim=1)  # [B, 3, D]

    def get_hidden(self, inputs):
        return side_pool(self._side(inputs))


class EGES(GES):
    def __init__(self, id_vocab_size, cat_vocab_size, brand_vocab_size, embedding_size, num_side,
                 device=None, generator=None):
        super().__init__(id_vocab_size, cat_vocab_size, brand_vocab_size, embedding_size,
                         device=device, generator=generator)
        self.weight_embedding = Embedding(id_vocab_size, num_side, device=device,
                                          generator=generator)

    def get_hidden(self, inputs):
        side = self._side(inputs)
        weights = self.weight_embedding(inputs[0])  # [B, 1, num_side]
        return side_pool(side, weights)
