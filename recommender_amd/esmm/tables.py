"""Per-feature embedding tables of the esmm models packed into ONE slab.

Reference: `{feat: keras.layers.Embedding(vocab_size, embedding_size)}` (esmm/esmm.py:10-11,
esmm/mmoe.py:12-13, esmm/base.py:11-12) and `compute_embedding` = per-feature lookups of
[B, 1] ids concatenated in INPUT-dict order and squeezed to [B, F*D] (esmm/esmm.py:15-19).
Here the F tables are one SlabEmbedding (one gather launch for all features) or, for the
40M-row config, a ShardedSlabEmbedding over the ranks.
"""
from __future__ import annotations

import torch
from torch import nn

from ..embedding import SlabEmbedding


class FeatureTables(nn.Module):
    def __init__(self, feat_vocab: dict, embedding_size: int, device=None, generator=None,
                 sharded_comm=None):
        super().__init__()
        self.feats = list(feat_vocab)
        self.index = {f: i for i, f in enumerate(self.feats)}
        self.embedding_size = embedding_size
        cards = [int(feat_vocab[f]) for f in self.feats]
        if sharded_comm is not None:
            from ..sharded import ShardedSlabEmbedding

            self.slab = ShardedSlabEmbedding(cards, embedding_size, sharded_comm, device=device,
                                             generator=generator)
        else:
            self.slab = SlabEmbedding(cards, embedding_size, device=device, generator=generator)

    def forward(self, inputs: dict) -> torch.Tensor:
        order = [self.index[f] for f in inputs]
        if order != list(range(len(self.feats))):
            raise ValueError("inputs must hold every feature of feat_vocab, in its order")
        ids = torch.stack([inputs[f].reshape(-1) for f in inputs], dim=1)  # [B, F]
        if getattr(self.slab, "fused_optimizer", None) is not None and torch.is_grad_enabled():
            # fused sparse optimizer: the step's sort is queued before the lookup (with the
            # deferred-decay Keras Adam its rows' skipped decay is replayed before they are read)
            self.slab.presort(ids)
        emb = self.slab(ids)                                                # [B, F, D]
        return emb.reshape(emb.shape[0], -1)                                # [B, F*D]
