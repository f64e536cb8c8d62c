"""ctr/model.py surface (reference ctr/model.py:6-58): DeepFM and DLRM over ONE shared
Embedding(vocab_size, embedding_size) for all categorical slots (ctr/model.py:10,42).

DLRM's lookup → concat(bottom MLP) → DotInteraction(False, True) → concat chain
(ctr/model.py:49-55) runs as ONE fused kernel pair (rs_dlrm_interaction_fwd/bwd): the rows are
gathered by id straight into the MFMA interaction and the top-MLP input [Z, bottom] is written
directly; `self.interaction` is kept for the reference attribute surface.
"""
from __future__ import annotations

import torch
from torch import nn

from ..embedding import Embedding, SlabEmbedding
from ..functional import COMPACT_ALIGN, dlrm_interaction, dlrm_top, fm_interaction
from .layers import MLP, DotInteraction


class DeepFM(nn.Module):
    def __init__(self, embedding_size, vocab_size, num_int_fea, num_cat_fea, mlp_units,
                 device=None, slot_cardinalities=None, generator=None):
        super().__init__()
        self.embedding_size = embedding_size
        self.num_int_fea = num_int_fea
        self.num_cat_fea = num_cat_fea
        if slot_cardinalities is None:
            self.embedding_layer = Embedding(vocab_size, embedding_size, device=device, generator=generator)
        else:
            self.embedding_layer = SlabEmbedding(slot_cardinalities, embedding_size, device=device, generator=generator)
        self.mlp = MLP(mlp_units, final_activation=None,
                       in_features=num_cat_fea * embedding_size + num_int_fea, device=device,
                       generator=generator)

    def forward(self, inputs, training=None, mask=None):
        cat_features, int_features = inputs["cat_features"], inputs["int_features"]
        int_features = int_features.reshape(-1, self.num_int_fea).float()
        cat_features = cat_features.reshape(-1, self.num_cat_fea)
        cat_embedding = self.embedding_layer(cat_features)              # [B, S, D]
        interaction = fm_interaction(cat_embedding)                     # ctr/model.py:21-23
        deep_cat_input = cat_embedding.reshape(-1, self.num_cat_fea * self.embedding_size)
        deep_input = torch.cat([deep_cat_input, int_features], dim=1)  # ctr/model.py:25-26
        dense_output = self.mlp(deep_input).squeeze(1)
        return torch.sigmoid(interaction + dense_output)                # ctr/model.py:28-30

    call = forward


class DLRM(nn.Module):
    """compact=True (default) feeds the top MLP only the F(F-1)/2 + D non-structural-zero
    inputs: the interaction writes the strict upper triangle without its zeros and the first
    top-MLP layer multiplies by the matching rows of its [F*F + D, units] kernel. The zero
    inputs contribute exactly 0 to every sum, so logits and gradients are the reference's;
    the kernel rows of the zero inputs receive an exactly-zero gradient as in the reference."""

    def __init__(self, bottom_mlp_units, top_mlp_units, embedding_size, vocab_size, num_cat_fea,
                 num_int_fea, device=None, slot_cardinalities=None, generator=None, compact=True,
                 embedding_layer=None):
        super().__init__()
        if bottom_mlp_units[-1] != embedding_size:
            raise ValueError("the last bottom-MLP width must equal embedding_size (ctr/model.py:55)")
        self.num_cat_fea = num_cat_fea
        self.num_int_fea = num_int_fea
        self.embedding_size = embedding_size
        self.bottom_mlp = MLP(bottom_mlp_units, final_activation="relu", in_features=num_int_fea,
                              device=device, generator=generator)
        F = num_cat_fea + 1
        self.top_mlp = MLP(top_mlp_units, final_activation="sigmoid",
                           in_features=F * F + embedding_size, device=device, generator=generator)
        if embedding_layer is not None:
            self.embedding_layer = embedding_layer  # e.g. a ShardedSlabEmbedding
        elif slot_cardinalities is None:
            self.embedding_layer = Embedding(vocab_size, embedding_size, device=device, generator=generator)
        else:
            self.embedding_layer = SlabEmbedding(slot_cardinalities, embedding_size, device=device, generator=generator)
        self.interaction = DotInteraction(False, True)
        self.compact = compact
        self._exchanged = None
        iu = torch.triu_indices(F, F, 1)
        rows = torch.cat([iu[0] * F + iu[1], F * F + torch.arange(embedding_size)])
        # the kernel pads the compact row to COMPACT_ALIGN columns with zeros; map the padding onto
        # structural-zero rows (lower triangle incl. diagonal) so their gradient stays 0
        pad = (rows.numel() + COMPACT_ALIGN - 1) // COMPACT_ALIGN * COMPACT_ALIGN - rows.numel()
        il = torch.tril_indices(F, F, 0)
        rows = torch.cat([rows, (il[0] * F + il[1])[:pad]])
        self.register_buffer("compact_rows", rows.to(device=self.top_mlp.mlp[0].kernel.device))

    def interact(self, cat_features, bmlp_activation, compact=False):
        """[Z, bottom] — ctr/model.py:49-55 fused into one kernel. With a row-sharded slab the
        kernel reads this step's exchanged unique rows through the inverse index."""
        if self._exchanged is not None:
            view, inv = self._exchanged
            self._exchanged = None
            return dlrm_interaction(view, inv, bmlp_activation, compact)
        return dlrm_interaction(self.embedding_layer, cat_features, bmlp_activation, compact)

    def forward(self, x, training=None, mask=None):
        cat_features, int_features = x["cat_features"], x["int_features"]
        int_features = int_features.reshape(-1, self.num_int_fea).float()
        cat_features = cat_features.reshape(-1, self.num_cat_fea)
        pending = None
        if not hasattr(self.embedding_layer, "exchange_begin"):
            # the side-stream radix sort of this step's ids is queued first: it then runs beside
            # the bottom MLP and the interaction kernels (queued after the forward kernels, the
            # side stream's wait on the main stream would put it behind them)
            self.embedding_layer.presort(cat_features)
        if hasattr(self.embedding_layer, "exchange_begin"):
            # row-sharded slab: the sort / split-size exchange is queued first (side stream), so
            # it runs beside the bottom MLP; the host waits for the split sizes only after the
            # bottom MLP is queued
            pending = self.embedding_layer.take_prefetched(cat_features.contiguous())
            if pending is None:
                pending = self.embedding_layer.exchange_begin(cat_features)
        bmlp_activation = self.bottom_mlp(int_features)
        if pending is not None:
            self._exchanged = self.embedding_layer.exchange_finish(pending)
        if not self.compact:
            tmlp_input = self.interact(cat_features, bmlp_activation)
            tmlp_input = tmlp_input.reshape(-1, (self.num_cat_fea + 1) ** 2 + self.embedding_size)
            out = self.top_mlp(tmlp_input).squeeze(1)
        else:
            layers = list(self.top_mlp.mlp)
            if (self.embedding_size == 128 and torch.is_grad_enabled()
                    and self.top_mlp.chain_ready(bmlp_activation)):
                # interaction + top MLP as one linear chain: rank-one interaction backward
                # (a row-sharded slab hands this step's exchanged unique rows + inverse index)
                table, ids = self.embedding_layer, cat_features
                if self._exchanged is not None:
                    (table, ids), self._exchanged = self._exchanged, None
                out = dlrm_top(table, ids, bmlp_activation, layers, self.compact_rows,
                               composed=self.top_mlp.composed_forward).squeeze(1)
            else:
                tmlp_input = self.interact(cat_features, bmlp_activation, compact=True)
                out = self.top_mlp(tmlp_input, rows=self.compact_rows).squeeze(1)
        return out

    call = forward
