"""esmm/esmm.py surface (reference esmm/esmm.py:7-44): shared embedding, CTR and CVR towers,
p_ctcvr = p_ctr * p_cvr, output [B, 2] = [p_ctr, p_ctcvr]."""
from __future__ import annotations

import torch
from torch import nn

from ..nn import shared_input_dense
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

    def _towers(self, e):
        # both towers' first layers read e: one GEMM over their concatenated kernels
        # (shared_input_dense), the rest of each tower on its column block in place
        h_ctr, h_cvr = shared_input_dense(e, [self.ctr.mlp[0], self.cvr.mlp[0]])
        return self.ctr(h_ctr, start=1), self.cvr(h_cvr, start=1)

    def forward(self, inputs, training=None, mask=None):
        p_ctr, p_cvr = self._towers(self.compute_embedding(inputs))
        return torch.cat([p_ctr, p_cvr * p_ctr], dim=-1)

    call = forward

    def compute_cvr(self, inputs):
        return self.cvr(self.compute_embedding(inputs))

    def compute_ctr(self, inputs):
        return self.ctr(self.compute_embedding(inputs))

    def compute_ctcvr(self, inputs):
        p_ctr, p_cvr = self._towers(self.compute_embedding(inputs))
        return p_cvr * p_ctr
