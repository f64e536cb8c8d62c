"""Keras-semantics dense building blocks on torch (dense math stays on hipBLASLt/rocBLAS).

`Dense(units, activation)` mirrors keras.layers.Dense [3p]: kernel [in, out] (Keras layout),
glorot_uniform kernel init, zero bias, y = act(x @ kernel + bias). `in_features=None` builds
lazily on the first call like Keras; the models in this package always pass it.
"""
from __future__ import annotations

import math

import torch
from torch import nn
import torch.nn.functional as F

_ACTS = {
    None: None,
    "linear": None,
    "relu": torch.relu,
    "sigmoid": torch.sigmoid,
    "tanh": torch.tanh,
    "softmax": lambda x: torch.softmax(x, dim=-1),
}


def get_activation(act):
    if callable(act):
        return act
    if act not in _ACTS:
        raise ValueError(f"unknown activation {act!r}")
    return _ACTS[act]


def _splitk_chunks(batch: int, fan_in: int, fan_out: int) -> int:
    """Batch split for the K = batch weight-gradient GEMM: hipBLASLt's single-pass fp32 kernels
    for [in, B]·[B, out] with B = 65 536 run at 7-64 TF/s; a batched GEMM over 16-64 batch
    chunks followed by a sum runs at 90-120 TF/s (tools/probe_gemm.py, MI355X)."""
    if batch < 8192 or fan_in * fan_out > 4_000_000:
        return 1
    for c in (64, 32, 16, 8):
        if batch % c == 0:
            return c
    return 1


class _DenseFn(torch.autograd.Function):
    """y = x @ kernel + bias with a split-K weight gradient (deterministic: fixed chunking,
    torch's fixed-order sum over chunks)."""

    @staticmethod
    def forward(ctx, x, kernel, bias):
        y = torch.addmm(bias, x, kernel) if bias is not None else x @ kernel
        ctx.save_for_backward(x, kernel)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, kernel = ctx.saved_tensors
        dx = dk = db = None
        if ctx.needs_input_grad[0]:
            dx = dy @ kernel.t()
        if ctx.needs_input_grad[1]:
            B, fi = x.shape
            fo = dy.shape[1]
            c = _splitk_chunks(B, fi, fo)
            if c > 1:
                dk = torch.bmm(x.view(c, B // c, fi).transpose(1, 2), dy.view(c, B // c, fo)).sum(0)
            else:
                dk = x.t() @ dy
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.sum(0)
        return dx, dk, db


class Dense(nn.Module):
    def __init__(self, units: int, activation=None, use_bias: bool = True, in_features=None,
                 device=None, generator: torch.Generator | None = None):
        super().__init__()
        self.units = int(units)
        self.activation = get_activation(activation)
        self.use_bias = use_bias
        self._device = device
        self._generator = generator
        self.kernel = None
        self.bias = None
        if in_features is not None:
            self.build(in_features)

    def build(self, in_features: int, device=None):
        device = device or self._device or ("cuda" if torch.cuda.is_available() else "cpu")
        limit = math.sqrt(6.0 / (in_features + self.units))
        k = torch.empty(in_features, self.units, device=device)
        k.uniform_(-limit, limit, generator=self._generator)
        self.kernel = nn.Parameter(k)
        self.bias = nn.Parameter(torch.zeros(self.units, device=device)) if self.use_bias else None

    def forward(self, x, kernel=None):
        if self.kernel is None:
            self.build(x.shape[-1], x.device)
        k = self.kernel if kernel is None else kernel
        if x.dim() == 2 and x.is_cuda:
            y = _DenseFn.apply(x, k, self.bias)
        elif self.bias is not None:
            y = torch.matmul(x, k) + self.bias
        else:
            y = torch.matmul(x, k)
        return self.activation(y) if self.activation is not None else y


def binary_crossentropy(y_true, y_pred, from_logits: bool = False, epsilon: float = 1e-7):
    """keras.losses.binary_crossentropy per example [3p TF 2.2 backend]: probabilities are
    clipped to [eps, 1-eps] and -(y log(p+eps) + (1-y) log(1-p+eps)); from_logits uses the
    stable sigmoid cross-entropy."""
    if from_logits:
        return F.binary_cross_entropy_with_logits(y_pred, y_true, reduction="none")
    p = torch.clamp(y_pred, epsilon, 1.0 - epsilon)
    return -(y_true * torch.log(p + epsilon) + (1.0 - y_true) * torch.log(1.0 - p + epsilon))
