"""ctr/layers.py surface (reference ctr/layers.py:1-43).

MLP(units, final_activation): hidden Dense layers carry NO activation (ctr/layers.py:8), only
the last one has `final_activation` (ctr/layers.py:9).
DotInteraction(self_interaction, skip_gather): X·Xᵀ with the triangle selection of
ctr/layers.py:23-43, computed by the gfx950 MFMA kernel rs_dot_interaction_fwd/bwd.
"""
from __future__ import annotations

from torch import nn

from ..functional import dot_interaction
from ..nn import Dense


class MLP(nn.Module):
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

    def forward(self, x):
        for layer in self.mlp:
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
