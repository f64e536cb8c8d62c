"""esmm/layers.py surface (reference esmm/layers.py:4-13): MLP with relu hidden layers and
`last_activation` on the last one."""
from __future__ import annotations

from torch import nn

from ..nn import Dense


class MLP(nn.Module):
    def __init__(self, units, last_activation, in_features=None, device=None, generator=None):
        super().__init__()
        layers, fan_in = [], in_features
        for u in units[:-1]:
            layers.append(Dense(u, "relu", in_features=fan_in, device=device, generator=generator))
            fan_in = u if fan_in is not None else None
        layers.append(Dense(units[-1], last_activation, in_features=fan_in, device=device,
                            generator=generator))
        self.mlp = nn.ModuleList(layers)

    def forward(self, inputs, start=0, **kwargs):
        """start: the index of the first layer to run (the layers before it evaluated by the
        caller, e.g. ESMM's shared first-layer GEMM)."""
        for fc in list(self.mlp)[start:]:
            inputs = fc(inputs)
        return inputs
