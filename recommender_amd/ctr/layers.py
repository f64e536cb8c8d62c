"""ctr/layers.py surface (reference ctr/layers.py:1-43).

MLP(units, final_activation): hidden Dense layers carry NO activation (ctr/layers.py:8), only
the last one has `final_activation` (ctr/layers.py:9).
DotInteraction(self_interaction, skip_gather): X·Xᵀ with the triangle selection of
ctr/layers.py:23-43, computed by the gfx950 MFMA kernel rs_dot_interaction_fwd/bwd.
"""
from __future__ import annotations

import torch
from torch import nn

from ..functional import dot_interaction
from ..nn import Dense, linear_chain


class MLP(nn.Module):
    """factored_backward=True (default): the hidden layers are linear, so the backward runs as
    one linear chain (nn._LinearChainFn: every layer's gradient from the last layer's, no
    full-width dgrad GEMMs). False: layer-by-layer autograd.
    composed_forward=True (default, chain path only): the forward evaluates the chain as the one
    affine map it is, y = act(x·K_1···K_L + c_L) (nn.chain_forward) — the same function, one
    batch-deep GEMM instead of one per layer; False keeps the layer-by-layer forward, bit-identical
    to the layerwise path."""

    factored_backward = True
    composed_forward = True
    # below this batch the layerwise backward's few GEMMs cost less than the chain's extra
    # launches (DeepFM cfg1, B 1024: 1.20 ms layerwise vs 1.49 ms factored per step)
    factored_min_batch = 8192

    def __init__(self, units, final_activation, in_features=None, device=None, generator=None):
        super().__init__()
        layers = []
        fan_in = in_features
        for u in units[:-1]:
            layers.append(Dense(u, None, in_features=fan_in, device=device, generator=generator))
            fan_in = u if fan_in is not None else None
        layers.append(Dense(units[-1], final_activation, in_features=fan_in, device=device,
                            generator=generator))
        self.mlp = nn.ModuleList(layers)

    def chain_ready(self, x) -> bool:
        """True when the forward runs as one linear chain (factored backward)."""
        layers = list(self.mlp)
        return (self.factored_backward and x.dim() == 2 and x.is_cuda and torch.is_grad_enabled()
                and x.shape[0] >= self.factored_min_batch
                and all(l.kernel is not None and l.act_code >= 0 for l in layers)
                and all(l.act_code == 0 for l in layers[:-1]))

    def forward(self, x, rows=None):
        """rows: optional index of first-layer kernel rows the input holds (DLRM compact row)."""
        layers = list(self.mlp)
        if self.chain_ready(x):
            return linear_chain(x, layers, rows, composed=self.composed_forward)
        x = layers[0](x, rows=rows)
        for layer in layers[1:]:
            x = layer(x)
        return x


class DotInteraction(nn.Module):
    def __init__(self, self_interaction, skip_gather):
        super().__init__()
        self.self_interaction = bool(self_interaction)
        self.skip_gather = bool(skip_gather)

    def forward(self, inputs):
        """inputs [B, F, D] → [B, F*F] (skip_gather) or [B, F(F∓1)/2] (gathered)."""
        return dot_interaction(inputs, self.self_interaction, self.skip_gather)
