"""esmm/mmoe.py surface (reference esmm/mmoe.py:8-109): shared embedding, num_experts expert
MLPs (relu last), one softmax gate Dense per task, task towers (sigmoid last),
outputs[1] = outputs[0] * outputs[1], output [B, num_tasks].

The experts keep their own parameters (`self.experts[i]`, the reference attribute surface) but
run as ONE wide GEMM for the first layer (concatenated kernels) and ONE batched GEMM per
deeper layer instead of num_experts small GEMMs; their weight gradients are split-K GEMMs
(recommender_amd.nn.wgrad / bwgrad) — hipBLASLt's K = batch kernels are 10x slower."""
from __future__ import annotations

import torch
from torch import nn

from ..eges.model import side_pool
from ..nn import Dense, batched_linear, linear
from .layers import MLP
from .tables import FeatureTables


class MMOE(nn.Module):
    def __init__(self, num_tasks, num_experts, expert_hidden_units, task_hidden_units, feat_vocab,
                 embedding_size, device=None, generator=None, sharded_comm=None):
        super().__init__()
        self.embedding_layer = FeatureTables(feat_vocab, embedding_size, device, generator, sharded_comm)
        fin = len(feat_vocab) * embedding_size
        self.num_tasks = num_tasks
        self.experts = nn.ModuleList(
            [MLP(expert_hidden_units, "relu", in_features=fin, device=device, generator=generator)
             for _ in range(num_experts)])
        self.gates = nn.ModuleList(
            [Dense(num_experts, "softmax", in_features=fin, device=device, generator=generator)
             for _ in range(num_tasks)])
        self.task_towers = nn.ModuleList(
            [MLP(task_hidden_units, "sigmoid", in_features=expert_hidden_units[-1], device=device,
                 generator=generator) for _ in range(num_tasks)])

    def compute_embedding(self, inputs):
        return self.embedding_layer(inputs)

    def experts_outputs(self, x):
        """[B, E, H]: every expert MLP (hidden relu, last relu) evaluated in batched GEMMs."""
        E = len(self.experts)
        layers = [e.mlp for e in self.experts]
        l0 = [m[0] for m in layers]
        k0 = torch.cat([l.kernel for l in l0], dim=1)             # [in, E*H0]
        b0 = torch.cat([l.bias for l in l0])
        # relu in the GEMM epilogues (and its mask with the bias gradient in one backward pass)
        h = linear(x, k0, b0, act=1).view(x.shape[0], E, -1).transpose(0, 1)  # [E,B,H0]
        h = h.contiguous()
        for j in range(1, len(layers[0])):
            k = torch.stack([m[j].kernel for m in layers])           # [E, Hin, Hout]
            b = torch.stack([m[j].bias for m in layers])[:, None, :]
            h = batched_linear(h, k, b, act=1)
        return h.transpose(0, 1)                                     # [B, E, H]

    def _towers(self, x):
        # [B, E, H] seen over the [E, B, H] expert outputs: rs_side_pool reads (and writes the
        # gradient of) that layout in place, no transpose pass either way
        ex = self.experts_outputs(x)
        outs = []
        for i in range(self.num_tasks):
            # softmax gate (Dense(E, softmax)) · experts, fused: rs_side_pool applies the
            # softmax to the gate logits and pools the expert rows in one pass (a [1,E]·[E,H]
            # matmul per example as 65 536 batched GEMMs costs ~1 ms per call)
            logits = self.gates[i].preactivation(x).unsqueeze(1)      # [B, 1, E]
            w = side_pool(ex, logits).squeeze(1)                      # [B, H]
            outs.append(self.task_towers[i](w))
        return outs

    def forward(self, inputs, training=None, mask=None):
        outs = self._towers(self.compute_embedding(inputs))
        outs[1] = outs[0] * outs[1]
        return torch.cat(outs, dim=1)

    call = forward

    def compute_cvr(self, inputs):
        return self._towers(self.compute_embedding(inputs))[1]

    def compute_ctr(self, inputs):
        return self._towers(self.compute_embedding(inputs))[0]

    def compute_ctcvr(self, inputs):
        o = self._towers(self.compute_embedding(inputs))
        return o[0] * o[1]
