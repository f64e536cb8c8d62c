"""esmm/base.py surface (reference esmm/base.py:7-19)."""
from __future__ import annotations

from torch import nn

from .layers import MLP
from .tables import FeatureTables


class BaseModel(nn.Module):
    def __init__(self, hidden_units, last_activation, feat_vocab, embedding_size, device=None,
                 generator=None, sharded_comm=None):
        super().__init__()
        self.embedding_layer = FeatureTables(feat_vocab, embedding_size, device, generator, sharded_comm)
        self.mlp = MLP(hidden_units, last_activation, in_features=len(feat_vocab) * embedding_size,
                       device=device, generator=generator)

    def forward(self, inputs, training=None, mask=None):
        return self.mlp(self.embedding_layer(inputs))

    call = forward
