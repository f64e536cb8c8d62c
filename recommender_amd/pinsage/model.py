"""PinSageModel (pinsage/train/model.py:8-39) and margin_loss (pinsage/train/train.py:17-20)."""
from __future__ import annotations

import torch
from torch import nn

from .graph import NID, HeteroGraph, PairGraph
from .layers import FeatureProjector, SageNet


def item2item_scorer(graph: PairGraph, h: torch.Tensor) -> torch.Tensor:
    """apply_edges(u_dot_v) (model.py:14-19): score [E, 1] = h[src] · h[dst]."""
    src, dst = graph.src.to(torch.int64), graph.dst.to(torch.int64)
    if graph.valid is not None:  # capacity-shaped: padding pairs (-1) score node 0, masked later
        src, dst = src.clamp_min(0), dst.clamp_min(0)
    s = h.index_select(0, src)
    d = h.index_select(0, dst)
    return (s * d).sum(dim=-1, keepdim=True)


def margin_loss(pos_score, neg_score, delta: float = 1.0, valid=None, n_valid=None):
    """mean(max(neg - pos + delta, 0)) (train.py:17-20). valid / n_valid (capacity-shaped
    batch): the mean over the live pairs, with no host sync."""
    hinge = torch.clamp(neg_score + delta - pos_score, min=0)
    if valid is None:
        return hinge.mean()
    return (hinge.reshape(-1) * valid).sum() / n_valid.to(hinge.dtype).reshape(())


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

    def get_repr(self, blocks):
        hidden_src = self.feature_projector(blocks[0].srcdata[NID],
                                            padded=blocks[0].n_src_live is not None)
        return self.sagenet(blocks, hidden_src)

    def tables(self):
        return self.feature_projector.tables()

    def dense_parameters(self):
        return [p for p in self.parameters() if p.numel() > 0]
