"""esmm/esmm.py surface (reference esmm/esmm.py:7-44): shared embedding, CTR and CVR towers,
p_ctcvr = p_ctr * p_cvr, output [B, 2] = [p_ctr, p_ctcvr]."""
from __future__ import annotations

import torch
from torch import nn

from .layers import MLP
from .tables import FeatureTables


class ESMM(nn.Module):
    def __init__(self, mlp_units, feat_vocab, embedding_size, device=None, generator=None,
                 sharded_comm=None):
        super().__init__()
        self.embedding_layer = FeatureTables(feat_vocab, embedding_size, device, generator, sharded_comm)
        fin = len(feat_vocab) * embedding_size
        self.ctr = MLP(mlp_units, "sigmoid", in_features=fin, device=device, generator=generator)
        self.cvr = MLP(mlp_units, "sigmoid", in_features=fin, device=device, generator=generator)

    def compute_embedding(self, inputs):
        return self.embedding_layer(inputs)

    def forward(self, inputs, training=None, mask=None):
        e = self.compute_embedding(inputs)
        p_ctr = self.ctr(e)
        p_cvr = self.cvr(e)
        return torch.cat([p_ctr, p_cvr * p_ctr], dim=-1)

    call = forward

    def compute_cvr(self, inputs):
        return self.cvr(self.compute_embedding(inputs))

    def compute_ctr(self, inputs):
        return self.ctr(self.compute_embedding(inputs))

    def compute_ctcvr(self, inputs):
        e = self.compute_embedding(inputs)
        return self.cvr(e) * self.ctr(e)
