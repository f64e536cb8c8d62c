"""PinSage layers (pinsage/train/layers.py) on the engine's kernels.

Convolve          :7-30   fc_1 (Dense relu) → rs_weighted_mean_agg (u_mul_e/sum, copy_e/sum,
                          clip ws >= 1, divide) → concat h_dst → fc_2 (Dense relu) →
                          rs_frobenius_normalize (one norm over the whole block, :28-29)
SageNet           :33-46
FeatureProjector  :49-81  year / genre-as-{0,1}-ids mean / id embeddings (rs_embedding_fwd)
"""
from __future__ import annotations

import torch
from torch import nn

from .. import _lib as L
from ..embedding import Embedding
from ..nn import Dense
from .graph import Block, HeteroGraph


class _WeightedMeanAgg(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u: torch.Tensor, block: Block):
        L.require_device(u, "u")
        u = u.contiguous()
        n_src, H = u.shape
        dev = u.device
        nv = torch.empty(block.n_dst, H, device=dev)
        wsum = torch.empty(max(block.n_dst, 1), device=dev)
        L.call("rs_weighted_mean_agg_fwd", L.ptr(u), n_src, H, L.ptr(block.indptr),
               L.ptr(block.edge_src), L.ptr(block.edge_w), block.n_dst, L.ptr(nv), L.ptr(wsum),
               L.stream_ptr(dev))
        ctx.block = block
        ctx.n_src = n_src
        ctx.save_for_backward(wsum)
        return nv

    @staticmethod
    def backward(ctx, g):
        (wsum,) = ctx.saved_tensors
        b = ctx.block
        g = g.contiguous()
        H = g.shape[1]
        gu = torch.empty(ctx.n_src, H, device=g.device)
        L.call("rs_weighted_mean_agg_bwd", L.ptr(g), H, L.ptr(b.t_indptr), L.ptr(b.t_edge),
               L.ptr(b.edge_dst), L.ptr(b.edge_w), L.ptr(wsum), ctx.n_src, L.ptr(gu),
               L.stream_ptr(g.device))
        return gu, None


def weighted_mean_agg(u: torch.Tensor, block: Block) -> torch.Tensor:
    return _WeightedMeanAgg.apply(u, block)


class _FrobeniusNormalize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, n_rows: torch.Tensor | None):
        L.require_device(x, "x")
        x = x.contiguous()
        n = x.numel()
        y = torch.empty_like(x)
        norm = torch.empty(1, device=x.device)
        ws = torch.empty(L.lib().rs_frobenius_workspace_size(n), dtype=torch.uint8, device=x.device)
        if n_rows is None:
            L.call("rs_frobenius_normalize_fwd", L.ptr(x), n, L.ptr(y), L.ptr(norm), L.ptr(ws),
                   ws.numel(), L.stream_ptr(x.device))
        else:
            L.call("rs_frobenius_normalize_rows_fwd", L.ptr(x), x.shape[0], x.shape[1],
                   L.ptr(n_rows), L.ptr(y), L.ptr(norm), L.ptr(ws), ws.numel(),
                   L.stream_ptr(x.device))
        ctx.n_rows = n_rows
        ctx.save_for_backward(y, norm)
        return y

    @staticmethod
    def backward(ctx, g):
        y, norm = ctx.saved_tensors
        g = g.contiguous()
        n = g.numel()
        dx = torch.empty_like(g)
        ws = torch.empty(L.lib().rs_frobenius_workspace_size(n), dtype=torch.uint8, device=g.device)
        if ctx.n_rows is None:
            L.call("rs_frobenius_normalize_bwd", L.ptr(g), L.ptr(y), L.ptr(norm), n, L.ptr(dx),
                   L.ptr(ws), ws.numel(), L.stream_ptr(g.device))
        else:
            L.call("rs_frobenius_normalize_rows_bwd", L.ptr(g), L.ptr(y), L.ptr(norm), g.shape[0],
                   g.shape[1], L.ptr(ctx.n_rows), L.ptr(dx), L.ptr(ws), ws.numel(),
                   L.stream_ptr(g.device))
        return dx, None


def frobenius_normalize(x: torch.Tensor, n_rows: torch.Tensor | None = None) -> torch.Tensor:
    """y = x / ||x||_F. n_rows ([1] int32 device): only the first n_rows rows of the 2-D x are
    live (capacity-shaped batch); the rest come out 0 and take no part in the norm."""
    return _FrobeniusNormalize.apply(x, n_rows)


class Convolve(nn.Module):
    def __init__(self, conv_hidden_size: int, conv_output_size: int, in_size: int | None = None,
                 device=None, generator: torch.Generator | None = None):
        super().__init__()
        self.fc_1 = Dense(conv_hidden_size, "relu", in_features=in_size, device=device,
                          generator=generator)
        self.fc_2 = Dense(conv_output_size, "relu",
                          in_features=None if in_size is None else conv_hidden_size + in_size,
                          device=device, generator=generator)

    def forward(self, block: Block, h):
        h_src, h_dst = h
        u = self.fc_1(h_src)                              # neighbour transformation
        nv = weighted_mean_agg(u, block)                  # importance pooling
        new = self.fc_2(torch.cat([nv, h_dst], dim=-1))   # concat transformation
        return frobenius_normalize(new, block.n_dst_live)  # l2 normalisation (global)


class SageNet(nn.Module):
    def __init__(self, num_layers: int, conv_hidden_size: int, conv_output_size: int,
                 in_size: int | None = None, device=None, generator=None):
        super().__init__()
        sizes = [in_size] + [conv_output_size] * num_layers
        self.convolves = nn.ModuleList(
            Convolve(conv_hidden_size, conv_output_size, sizes[i], device, generator)
            for i in range(num_layers))
        self.fc_1 = Dense(conv_hidden_size, "relu", in_features=conv_output_size, device=device,
                          generator=generator)
        self.fc_2 = Dense(conv_output_size, None, in_features=conv_hidden_size, device=device,
                          generator=generator)

    def forward(self, blocks, h_src):
        for convolve, block in zip(self.convolves, blocks):
            h_dst = h_src[: block.num_dst_nodes()]
            h_src = convolve(block, (h_src, h_dst))
        return self.fc_2(self.fc_1(h_src))


class _MultiHotMeanFn(torch.autograd.Function):
    """table(mh[items]).mean(dim=1) for a multi-hot id matrix mh [n_items, G] (the genre
    feature): rs_multihot_mean_fwd reads each item's id row in place — no gathered [N, G] ids,
    no [N, G, D] rows, no mean pass — and the backward forms the table's dense [V, D] gradient
    in one pass (rs_multihot_mean_bwd), handed to the table as V rows (their densified sum is
    that gradient) instead of N·G gradient rows."""

    @staticmethod
    def forward(ctx, handle, table_module, mh, items):
        w = table_module.weight
        V, D = w.shape
        N, G = items.numel(), mh.shape[1]
        out = torch.empty(N, D, device=w.device)
        L.call("rs_multihot_mean_fwd", L.ptr(w), V, D, L.ptr(mh), G, mh.shape[0], L.ptr(items), N,
               L.ptr(out), L.ptr(table_module.err_flag), L.stream_ptr(w.device))
        ctx.table_module, ctx.mh, ctx.items = table_module, mh, items
        return out

    @staticmethod
    def backward(ctx, g):
        from ..functional import _lookup_backward

        tm = ctx.table_module
        V, D = tm.weight.shape
        N, G = ctx.items.numel(), ctx.mh.shape[1]
        dev = g.device
        dtable = torch.empty(V, D, device=dev)
        ws = _ws("multihot_bwd", L.lib().rs_multihot_mean_bwd_workspace_size(N, V, D), dev)
        L.call("rs_multihot_mean_bwd", L.ptr(ctx.mh), G, ctx.mh.shape[0], L.ptr(ctx.items), N,
               L.ptr(g.contiguous()), V, D, L.ptr(dtable), L.ptr(tm.err_flag), L.ptr(ws),
               ws.numel(), L.stream_ptr(dev))
        _lookup_backward(tm, _arange_i32(V, dev), dtable, None)
        return None, None, None, None


_ws_bufs: dict = {}
_aranges: dict = {}


def _ws(name, nbytes, dev):
    b = _ws_bufs.get((name, dev))
    if b is None or b.numel() < nbytes:
        b = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=dev)
        _ws_bufs[(name, dev)] = b
    return b


def _arange_i32(n, dev):
    t = _aranges.get((n, dev))
    if t is None:
        t = torch.arange(n, dtype=torch.int32, device=dev)
        _aranges[(n, dev)] = t
    return t


def multihot_mean_lookup(table_module, mh: torch.Tensor, items: torch.Tensor) -> torch.Tensor:
    """table_module(mh.index_select(0, items)).mean(dim=1), fused (_MultiHotMeanFn) when the
    shapes take it (V·D <= 256, G <= 32, no fused optimizer on the table). The table's gradient
    arrives as all V rows (0 for ids the batch never used): the same update under Keras Adam,
    whose sparse apply decays every row anyway (PinSage's optimizer, train.py:45-46)."""
    V, D = table_module.weight.shape
    if (mh.is_cuda and mh.dtype == torch.int32 and mh.is_contiguous() and mh.shape[1] <= 32
            and V * D <= 256 and D <= 64 and table_module.fused_optimizer is None
            and table_module.slot_offsets is None and items.numel() > 0):
        return _MultiHotMeanFn.apply(table_module.grad_handle, table_module, mh,
                                     items.to(torch.int64).contiguous())
    return table_module(mh.index_select(0, items)).mean(dim=1)


class FeatureProjector(nn.Module):
    def __init__(self, full_graph: HeteroGraph, itype: str, embedding_size: int, device=None,
                 generator: torch.Generator | None = None):
        super().__init__()
        self.itype = itype
        self.full_graph = full_graph
        data = full_graph.nodes[itype].data
        dev = device or full_graph.device
        self.year = data["year"].to(dev, torch.int32).contiguous()
        self.genre = data["genre"].to(dev, torch.int32).contiguous()  # multi-hot → {0,1} ids
        self.item_id = data["id"].to(dev, torch.int32).contiguous()
        year_vocab_size = int(self.year.max().item()) + 1
        genre_vocab_size = self.genre.shape[1]
        id_vocab_size = full_graph.number_of_nodes(itype)
        self.year_embedding = Embedding(year_vocab_size, embedding_size, device=dev,
                                        generator=generator)
        self.genre_embedding = Embedding(genre_vocab_size, embedding_size, device=dev,
                                         generator=generator)
        self.id_embedding = Embedding(id_vocab_size, embedding_size, device=dev,
                                      generator=generator)

    def tables(self):
        return [self.year_embedding, self.genre_embedding, self.id_embedding]

    def forward(self, induces_ids: torch.Tensor, padded: bool = False) -> torch.Tensor:
        ids = induces_ids.to(torch.int64)
        if padded:  # capacity-shaped block: padding src nodes (-1) read item 0, grad 0
            ids = ids.clamp_min(0)
        year_embedding = self.year_embedding(self.year.index_select(0, ids))
        genre_embedding = multihot_mean_lookup(self.genre_embedding, self.genre, ids)
        id_embedding = self.id_embedding(self.item_id.index_select(0, ids))
        return torch.cat([year_embedding, genre_embedding, id_embedding], dim=-1)
