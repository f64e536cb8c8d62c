"""esmm/mmoe.py surface (reference esmm/mmoe.py:8-109): shared embedding, num_experts expert
MLPs (relu last), one softmax gate Dense per task, task towers (sigmoid last),
outputs[1] = outputs[0] * outputs[1], output [B, num_tasks].

The experts keep their own parameters (`self.experts[i]`, the reference attribute surface) but
run as ONE wide GEMM for the first layer (concatenated kernels) and ONE batched GEMM per
deeper layer instead of num_experts small GEMMs; their weight gradients are split-K GEMMs
(recommender_amd.nn.wgrad / bwgrad) — hipBLASLt's K = batch kernels are 10x slower."""
from __future__ import annotations

import ctypes as C
import os

import torch
from torch import nn

from .. import _lib as L
from ..eges.model import side_pool
from ..nn import Dense, _act_bwd, _affine, batched_linear, linear, wgrad
from .layers import MLP
from .tables import FeatureTables

# RS_MMOE_FUSED=0: the experts / gates / poolings as separate autograd nodes (A/B switch)
_FUSED = os.environ.get("RS_MMOE_FUSED", "1") != "0"


def _ptrs(ts):
    return C.cast((C.c_void_p * len(ts))(*[t.data_ptr() for t in ts]), C.c_void_p)


class _ExpertsGatesFn(torch.autograd.Function):
    """MMOE's shared-input block (esmm/mmoe.py:36-46) as one node: the E experts' first layers
    as one GEMM over their concatenated kernels (relu in its epilogue), the T gates' logits as
    one GEMM, the experts' second layers as one batched GEMM reading the first layer's output
    in place ([E, B, H0] seen with rows E·H0 apart: no transpose copy), and the T softmax
    poolings of the [E, B, H1] expert outputs in one pass (rs_side_pool_fwd_multi, which also
    adds the second layers' bias and applies their relu in place: no bias broadcast into the
    GEMM output, no relu pass).
    Backward: one pooling pass for all tasks (their expert-output gradients summed inside it),
    the second layers' relu masks and per-expert bias sums in one pass, their input gradient by
    one batched GEMM written straight into the first layer's [B, E·H0] layout, one mask pass
    over it, and the gates' logit gradients added to the input-gradient GEMM's output in place
    (K = T·E, beta 1): no transpose copies, no per-consumer add passes."""

    @staticmethod
    def forward(ctx, x, k0, b0, k1, b1, kg, bg, E, T):
        B = x.shape[0]
        H0, H1 = k0.shape[1] // E, k1.shape[2]
        x = x.contiguous()
        dev = x.device
        st = L.stream_ptr(dev)
        y1 = _affine(x, k0, b0, 1)                                  # [B, E*H0]
        zg = torch.addmm(bg, x, kg)                                 # [B, T*E]
        y1v = y1.view(B, E, H0).transpose(0, 1)                     # [E, B, H0], in place
        y2 = torch.bmm(y1v, k1)                                     # [E, B, H1] pre-activation
        hid = [torch.empty(B, H1, device=dev) for _ in range(T)]
        att = [torch.empty(B, E, device=dev) for _ in range(T)]
        # the pooling pass adds the bias and applies the relu to y2 in place, then pools
        L.call("rs_side_pool_fwd_multi", L.ptr(y2), H1, B * H1, B, E, H1, T,
               _ptrs([zg[:, t * E:] for t in range(T)]), T * E, _ptrs(hid), _ptrs(att),
               L.ptr(b1.reshape(E, H1).contiguous()), st)
        ctx.save_for_backward(x, k0, k1, kg, y1, y2, *att)
        ctx.E, ctx.T = E, T
        return tuple(hid)

    @staticmethod
    def backward(ctx, *gh):
        x, k0, k1, kg, y1, y2, *att = ctx.saved_tensors
        E, T = ctx.E, ctx.T
        B = x.shape[0]
        H0, H1 = k0.shape[1] // E, k1.shape[2]
        dev = x.device
        st = L.stream_ptr(dev)
        gh = [torch.zeros(B, H1, device=dev) if g is None else g.contiguous() for g in gh]
        dy2 = torch.empty_like(y2)
        dzg = torch.empty(B, T * E, device=dev)                     # the gates' logit gradients
        L.call("rs_side_pool_bwd_multi", L.ptr(y2), H1, B * H1, B, E, H1, T, _ptrs(att),
               _ptrs(gh), L.ptr(dy2), _ptrs([dzg[:, t * E:] for t in range(T)]), T * E, st)
        # second layers: every expert's relu mask in one pass, per-expert bias sums
        dz2 = torch.empty_like(y2)
        db1 = torch.empty(E, 1, H1, device=dev)
        if B % 512 == 0:
            ws = torch.empty(max(1, L.lib().rs_act_bwd_colsum_workspace_size(E * B, H1) // 4),
                             device=dev)
            L.call("rs_act_bwd_colsum_groups", L.ptr(dy2), L.ptr(y2), E * B, H1, 1, E, L.ptr(dz2),
                   L.ptr(db1), L.ptr(ws), ws.numel() * 4, st)
        else:
            for e in range(E):
                _act_bwd(dy2[e], y2[e], 1, True, dz=dz2[e], db=db1[e, 0])
        # their input gradient written straight into the first layer's [B, E·H0] layout
        dy1 = torch.empty(B, E * H0, device=dev)
        torch.bmm(dz2, k1.transpose(1, 2), out=dy1.view(B, E, H0).transpose(0, 1))
        dk1 = torch.stack([wgrad(y1[:, e * H0:(e + 1) * H0], dz2[e]) for e in range(E)])
        # first layers: one mask + bias pass over [B, E·H0]; the gates join the input gradient
        # as a K = T·E update of the same output (no add pass)
        dz1, db0 = _act_bwd(dy1, y1, 1, True)
        dbg = dzg.sum(0)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = dz1 @ k0.t()
            dx.addmm_(dzg, kg.t())
        return dx, wgrad(x, dz1), db0, dk1, db1, wgrad(x, dzg), dbg, None, None


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

    def _fused_ready(self, x):
        E = len(self.experts)
        mlps = [e.mlp for e in self.experts]
        return (_FUSED and x.dim() == 2 and x.is_cuda and torch.is_grad_enabled()
                and 1 <= self.num_tasks <= 4 and 2 <= E <= 16
                and all(len(m) == 2 and all(l.act_code == 1 and l.kernel is not None
                                            and l.bias is not None for l in m) for m in mlps)
                and len({(m[0].units, m[1].units) for m in mlps}) == 1
                and mlps[0][1].units % 4 == 0 and mlps[0][1].units <= 128
                and all(g.kernel is not None and g.bias is not None and g.units == E
                        for g in self.gates))

    def _towers(self, x):
        if self._fused_ready(x):
            E, T = len(self.experts), self.num_tasks
            l0 = [e.mlp[0] for e in self.experts]
            l1 = [e.mlp[1] for e in self.experts]
            pooled = _ExpertsGatesFn.apply(
                x, torch.cat([l.kernel for l in l0], 1), torch.cat([l.bias for l in l0]),
                torch.stack([l.kernel for l in l1]), torch.stack([l.bias for l in l1])[:, None, :],
                torch.cat([g.kernel for g in self.gates], 1), torch.cat([g.bias for g in self.gates]),
                E, T)
            return [self.task_towers[i](pooled[i]) for i in range(T)]
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
