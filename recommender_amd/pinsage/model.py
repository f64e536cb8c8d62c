"""PinSageModel (pinsage/train/model.py:8-39) and margin_loss (pinsage/train/train.py:17-20)."""
from __future__ import annotations

import torch
from torch import nn

from .. import _lib as L

from .graph import NID, HeteroGraph, PairGraph
from .layers import FeatureProjector, SageNet


_err_flags: dict = {}


def oob_flag(dev) -> torch.Tensor:
    """The device int32 flag the fused pair kernels set (RS_ERRBIT_OOB) for a node id past h's
    rows (the index_select they replace raised on one)."""
    f = _err_flags.get(dev)
    if f is None:
        f = torch.zeros(1, dtype=torch.int32, device=dev)
        _err_flags[dev] = f
    return f


def check_oob(dev) -> None:
    """Raise RecsysError (and clear the flag) if a fused pair kernel saw a node id past h's
    rows since the last check: the index_select they replace raised on one. Synchronises; called
    at the train loop's sync points (PinSageStep.__call__, the logging steps of main())."""
    f = _err_flags.get(dev)
    if f is not None and int(f.item()):
        f.zero_()
        raise L.RecsysError("PinSage: a node id outside the representation rows (the pair "
                            "kernels read a zero row and dropped its gradient)")


_ws_bufs: dict = {}


def _ws(name, nbytes, dev):
    b = _ws_bufs.get((name, dev))
    if b is None or b.numel() < nbytes:
        b = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=dev)
        _ws_bufs[(name, dev)] = b
    return b


class _GatherRowsFn(torch.autograd.Function):
    """h.index_select(0, idx) whose backward is a fixed-order index_add (rs_index_add_rows:
    sort + tiled segmented sum) — run-to-run identical, where index_select's backward adds
    colliding rows with float atomics in arrival order."""

    @staticmethod
    def forward(ctx, h, idx):
        ctx.save_for_backward(idx)
        ctx.n_rows = h.shape[0]
        return h.index_select(0, idx)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        g = g.contiguous()
        n, D = idx.numel(), g.shape[1]
        dev = g.device
        dh = torch.empty(ctx.n_rows, D, device=dev, dtype=g.dtype)
        ws = _ws("index_add", L.lib().rs_index_add_rows_workspace_size(n, D), dev)
        L.call("rs_index_add_rows", L.ptr(idx), L.id_dtype_code(idx), n, None, L.ptr(g), D,
               ctx.n_rows, L.ptr(dh), L.ptr(oob_flag(dev)), L.ptr(ws), ws.numel(),
               L.stream_ptr(dev))
        return dh, None


def gather_rows(h: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """h[idx] with a deterministic backward on the GPU (fp32 2-D h), index_select elsewhere."""
    if h.is_cuda and h.dim() == 2 and h.dtype == torch.float32 and h.requires_grad:
        return _GatherRowsFn.apply(h, idx.contiguous())
    return h.index_select(0, idx)


def item2item_scorer(graph: PairGraph, h: torch.Tensor) -> torch.Tensor:
    """apply_edges(u_dot_v) (model.py:14-19): score [E, 1] = h[src] · h[dst]."""
    src, dst = graph.src.to(torch.int64), graph.dst.to(torch.int64)
    if graph.valid is not None:  # capacity-shaped: padding pairs (-1) score node 0, masked later
        src, dst = src.clamp_min(0), dst.clamp_min(0)
    s = gather_rows(h, src)
    d = gather_rows(h, dst)
    return (s * d).sum(dim=-1, keepdim=True)


def margin_loss(pos_score, neg_score, delta: float = 1.0, valid=None, n_valid=None):
    """mean(max(neg - pos + delta, 0)) (train.py:17-20). valid / n_valid (capacity-shaped
    batch): the mean over the live pairs, with no host sync."""
    hinge = torch.clamp(neg_score + delta - pos_score, min=0)
    if valid is None:
        return hinge.mean()
    return (hinge.reshape(-1) * valid).sum() / n_valid.to(hinge.dtype).reshape(())


class _PairMarginFn(torch.autograd.Function):
    """item2item_scorer on both pair graphs + margin_loss in one kernel each way
    (rs_pair_margin_fwd / _bwd): the row gathers, products, sums, clamp, mask and mean were a
    dozen recorded ops forward and as many backward (a capacity-shaped static step replays every
    one of them as a graph node). The backward folds each node's pair terms in a fixed order
    (rs_index_add_rows inside rs_pair_margin_bwd): deterministic."""

    @staticmethod
    def forward(ctx, h, ps, pd, ns, nd, valid, n_valid, delta):
        h = h.contiguous()
        P, D = ps.numel(), h.shape[1]
        dev = h.device
        pos = torch.empty(P, device=dev)
        neg = torch.empty(P, device=dev)
        loss = torch.empty((), device=dev)
        ws = _ws("pair_fwd", L.lib().rs_pair_margin_workspace_size(P), dev)
        # a bool mask's bytes are the 0 / 1 flags the kernel reads
        L.call("rs_pair_margin_fwd", L.ptr(h), D, D, h.shape[0], L.ptr(ps), L.ptr(pd), L.ptr(ns),
               L.ptr(nd), P, float(delta), L.ptr(valid), L.ptr(n_valid), L.ptr(pos), L.ptr(neg),
               L.ptr(loss), L.ptr(oob_flag(dev)), L.ptr(ws), ws.numel(), L.stream_ptr(dev))
        ctx.save_for_backward(h, ps, pd, ns, nd, valid, n_valid, pos, neg)
        ctx.delta = float(delta)
        return loss

    @staticmethod
    def backward(ctx, g):
        h, ps, pd, ns, nd, valid, n_valid, pos, neg = ctx.saved_tensors
        P, D = ps.numel(), h.shape[1]
        dev = h.device
        dh = torch.empty_like(h)
        ws = _ws("pair_bwd", L.lib().rs_pair_margin_bwd_workspace_size(P, D), dev)
        L.call("rs_pair_margin_bwd", L.ptr(h), D, D, h.shape[0], L.ptr(ps), L.ptr(pd), L.ptr(ns),
               L.ptr(nd), P, ctx.delta, L.ptr(valid), L.ptr(n_valid), L.ptr(pos), L.ptr(neg),
               L.ptr(g.reshape(1).contiguous()), L.ptr(dh), L.ptr(oob_flag(dev)), L.ptr(ws),
               ws.numel(), L.stream_ptr(dev))
        return dh, None, None, None, None, None, None, None


def _i32(t):
    return t if t.dtype == torch.int32 and t.is_contiguous() else t.to(torch.int32).contiguous()


def pair_margin_loss(pos_graph: PairGraph, neg_graph: PairGraph, h: torch.Tensor,
                     delta: float = 1.0) -> torch.Tensor:
    """margin_loss(item2item_scorer(pos_graph, h), item2item_scorer(neg_graph, h), delta, valid,
    n_valid) — fused (_PairMarginFn) on the GPU for one negative per positive pair."""
    P = pos_graph.src.numel()
    if (h.is_cuda and h.dim() == 2 and h.shape[1] <= 64 and h.dtype == torch.float32
            and neg_graph.src.numel() == P and P > 0):
        valid = pos_graph.valid
        if valid is not None and valid.dtype not in (torch.bool, torch.uint8):
            valid = valid.to(torch.uint8)
        n_valid = None if pos_graph.n_valid is None else _i32(pos_graph.n_valid)
        return _PairMarginFn.apply(h, _i32(pos_graph.src), _i32(pos_graph.dst),
                                   _i32(neg_graph.src), _i32(neg_graph.dst),
                                   None if valid is None else valid.contiguous(), n_valid, delta)
    return margin_loss(item2item_scorer(pos_graph, h), item2item_scorer(neg_graph, h), delta,
                       pos_graph.valid, pos_graph.n_valid)


class PinSageModel(nn.Module):
    def __init__(self, full_graph: HeteroGraph, itype: str, num_layers: int, embedding_size: int,
                 conv_hidden_size: int, conv_output_size: int, device=None,
                 generator: torch.Generator | None = None):
        super().__init__()
        self.feature_projector = FeatureProjector(full_graph, itype, embedding_size, device,
                                                  generator)
        self.sagenet = SageNet(num_layers, conv_hidden_size, conv_output_size,
                               in_size=3 * embedding_size, device=device or full_graph.device,
                               generator=generator)

    def item2item_scorer(self, graph, h):
        return item2item_scorer(graph, h)

    def forward(self, pos_graph, neg_graph, blocks):
        hidden_repr = self.get_repr(blocks)
        return self.item2item_scorer(pos_graph, hidden_repr), self.item2item_scorer(neg_graph,
                                                                                    hidden_repr)

    call = forward

    def margin_loss(self, pos_graph, neg_graph, blocks, delta: float = 1.0):
        """the training loss of train.py:17-20 on this batch (pair_margin_loss)."""
        return pair_margin_loss(pos_graph, neg_graph, self.get_repr(blocks), delta)

    def get_repr(self, blocks):
        hidden_src = self.feature_projector(blocks[0].srcdata[NID],
                                            padded=blocks[0].n_src_live is not None)
        return self.sagenet(blocks, hidden_src)

    def tables(self):
        return self.feature_projector.tables()

    def dense_parameters(self):
        return [p for p in self.parameters() if p.numel() > 0]
