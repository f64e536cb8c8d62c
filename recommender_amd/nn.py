"""Keras-semantics dense building blocks on torch (dense math stays on hipBLASLt/rocBLAS).

`Dense(units, activation)` mirrors keras.layers.Dense [3p]: kernel [in, out] (Keras layout),
glorot_uniform kernel init, zero bias, y = act(x @ kernel + bias). `in_features=None` builds
lazily on the first call like Keras; the models in this package always pass it.
"""
from __future__ import annotations

import contextlib
import math
import os
import weakref

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


# The Dense products on the bf16 matrix cores (csrc/gemm.hip rs_gemm_x3: split-bf16, six part
# products, each K-step re-accumulated on the VALU) — OFF by default, opt in with RS_GEMM_X3=1.
# Per element it is more accurate than the library fp32 GEMM (tools/gemm_bias_probe.py, B = 65 536,
# K = 324: mean |error| 5e-9 vs 2e-8 of the term magnitude, max 8e-8 vs 4e-7) and it measured
# 1.14-1.24x on the wide forwards (bias + relu epilogue) and 1.04-1.21x on the wide dgrads
# (tools/gemm_bench.py), but whole steps gain little (ESMM 2.72 -> 2.69 ms, MMOE 5.22 -> 5.12 ms)
# and the cfg4 full-size oracle check of the dense gradients (65 536-example sums, bound 1e-4 of
# the 512-chunk magnitude) fails with it by up to 6.7x (tests/test_fullsize_gpu.py), so parity
# keeps the library default.
_GEMM_X3 = os.environ.get("RS_GEMM_X3", "0") == "1"
_X3_MIN_N, _X3_MIN_K = 128, 160
# relu layers: hipBLASLt's bias + relu epilogue (torch._addmm_activation) instead of a separate
# in-place relu pass; RS_RELU_EPILOGUE=0 restores the pass
_RELU_EPILOGUE = os.environ.get("RS_RELU_EPILOGUE", "1") == "1"


def _x3_ready(*ts, n=0, k=0, batched=False):
    if not _GEMM_X3 or (not batched and (n < _X3_MIN_N or k < _X3_MIN_K)):
        return False
    return all(t is not None and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
               and t.data_ptr() % 16 == 0 and t.dim() >= 2 and t.shape[-1] % 4 == 0
               and t.shape[-2] % 4 == 0 for t in ts)


def gemm_x3(a, b, tb=False, bias=None, act=0):
    """act(a·op(b) + bias) by rs_gemm_x3: a [M, K] (or [E, M, K]), b [K, N] (tb: [N, K]) or
    batched [E, ...]; bias [N] / [E, N] or None; act 0 none, 1 relu, 2 sigmoid."""
    from . import _lib as L

    batched = a.dim() == 3
    E = a.shape[0] if batched else 1
    M, K = a.shape[-2], a.shape[-1]
    N = b.shape[-2] if tb else b.shape[-1]
    out = torch.empty(*((E,) if batched else ()), M, N, device=a.device, dtype=torch.float32)
    sA = M * K if batched else 0
    sB = b.shape[-2] * b.shape[-1] if batched else 0
    sbias = N if (bias is not None and batched) else 0
    L.call("rs_gemm_x3", 0, int(tb), M, N, K, L.ptr(a), K, sA, L.ptr(b), b.shape[-1], sB,
           L.ptr(out), N, M * N, E, L.ptr(bias), sbias, act, 1, None, 0, L.stream_ptr(a.device))
    return out


def _affine(x, k, b, act):
    """act(x·k + b) for one Dense layer (act 0 / 1 relu / 2 sigmoid): rs_gemm_x3 with the bias and
    activation in its epilogue when enabled and the shapes take it, else the library GEMM. Every
    layer-by-layer evaluation goes through here, so they stay bit-identical to each other."""
    if _x3_ready(x, k, n=k.shape[1], k=k.shape[0]) and (b is None or b.is_contiguous()):
        return gemm_x3(x, k, bias=b, act=act)
    if act == 1 and b is not None and _RELU_EPILOGUE and x.is_cuda:
        return torch._addmm_activation(b, x, k)  # relu in the library GEMM's epilogue
    z = torch.addmm(b, x, k) if b is not None else x @ k
    if act == 1:
        return torch.relu_(z)
    if act == 2:
        return torch.sigmoid_(z)
    return z


def _splitk_plan(K: int, fan_in: int, fan_out: int, batches: int = 1):
    """(chunks, rows per chunk) for a K-deep weight-gradient GEMM [in, K]·[K, out]: hipBLASLt's
    single-pass fp32 kernels for K >= 8k run at 7-64 TF/s (tiny-N tiles over a huge K); a
    batched GEMM over 8-64 K-chunks + a fixed-order sum runs at 90-120 TF/s
    (tools/probe_gemm.py, MI355X). Partials stay within ~16 MB."""
    if K < 8192 or fan_in * fan_out > 4_000_000:
        return 1, K
    target = max(8, min(64, (16 << 20) // max(1, batches * fan_in * fan_out * 4)))
    c = 64
    while c > target or K // c < 1024:
        c //= 2
    return (c, K // c) if c >= 2 else (1, K)


def _splitk_chunks(batch: int, fan_in: int, fan_out: int) -> int:
    return _splitk_plan(batch, fan_in, fan_out)[0]


def wgrad(x: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """xᵀ·g for x [K, in], g [K, out] with K the batch (split-K, deterministic: fixed chunking,
    fixed fold order; a K not divisible by the chunk count adds its tail rows last)."""
    K, fi = x.shape
    fo = g.shape[1]
    c, chunk = _splitk_plan(K, fi, fo)
    if c == 1:
        return x.t() @ g
    m = c * chunk
    out = torch.bmm(x[:m].reshape(c, chunk, fi).transpose(1, 2), g[:m].reshape(c, chunk, fo)).sum(0)
    if m < K:
        out += x[m:].t() @ g[m:]
    return out


def bwgrad(x: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """Batched xᵀ·g: x [E, K, in], g [E, K, out] → [E, in, out], split-K per batch entry."""
    E, K, fi = x.shape
    fo = g.shape[2]
    c, chunk = _splitk_plan(K, fi, fo, E)
    if c == 1:
        return torch.bmm(x.transpose(1, 2), g)
    m = c * chunk
    out = torch.bmm(x[:, :m].reshape(E * c, chunk, fi).transpose(1, 2),
                    g[:, :m].reshape(E * c, chunk, fo)).view(E, c, fi, fo).sum(1)
    if m < K:
        out += torch.bmm(x[:, m:].transpose(1, 2), g[:, m:])
    return out


def _act_bwd(g, y, act, want_db, dz=None, db=None):
    """(dz = act'(y)⊙g, Σ_rows dz or None) for act 0 / 1 (relu) / 2 (sigmoid) on [R, N] rows
    (rs_act_bwd_colsum: one pass for both); dz / db: optional contiguous outputs to write."""
    from . import _lib as L

    if act == 0:
        return g, (g.sum(0) if want_db else None)
    R, N = g.shape
    dz = torch.empty_like(g) if dz is None else dz
    db = torch.empty(N, device=g.device, dtype=torch.float32) if db is None else db
    ws = torch.empty(max(1, L.lib().rs_act_bwd_colsum_workspace_size(R, N) // 4), device=g.device)
    L.call("rs_act_bwd_colsum", L.ptr(g), L.ptr(y), R, N, act, L.ptr(dz), L.ptr(db), L.ptr(ws),
           ws.numel() * 4, L.stream_ptr(g.device))
    return dz, (db if want_db else None)


class _LinearFn(torch.autograd.Function):
    """y = act(x·k (+ b)), act 0 / 1 (relu) / 2 (sigmoid); backward with the split-K weight
    gradient (and the activation's mask with the bias gradient in one pass)."""

    @staticmethod
    def forward(ctx, x, k, b, act=0):
        x = x.contiguous()
        y = _affine(x, k, b, act)
        ctx.save_for_backward(x, k, y if act else None)
        ctx.has_b, ctx.act = b is not None, act
        return y

    @staticmethod
    def backward(ctx, g):
        x, k, y = ctx.saved_tensors
        g = g.contiguous()
        dz, db = _act_bwd(g, y, ctx.act, ctx.has_b)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (gemm_x3(dz, k, tb=True) if _x3_ready(dz, k, n=k.shape[0], k=k.shape[1])
                  else dz @ k.t())
        return dx, wgrad(x, dz), db, None


def linear(x: torch.Tensor, k: torch.Tensor, b: torch.Tensor | None = None,
           act: int = 0) -> torch.Tensor:
    return _LinearFn.apply(x, k, b, act)


class _BatchedLinearFn(torch.autograd.Function):
    """y[e] = act(x[e]·k[e] + b[e]) for x [E, B, in], k [E, in, out], b [E, 1, out]."""

    @staticmethod
    def forward(ctx, x, k, b, act=0):
        x = x.contiguous()
        if _x3_ready(x, k, batched=True) and b.is_contiguous():
            y = gemm_x3(x, k, bias=b.reshape(b.shape[0], -1), act=act)
        else:
            y = torch.baddbmm(b, x, k)
            if act == 1:
                y = torch.relu_(y)
            elif act == 2:
                y = torch.sigmoid_(y)
        ctx.save_for_backward(x, k, y if act else None)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, g):
        x, k, y = ctx.saved_tensors
        g = g.contiguous()
        E = g.shape[0]
        if ctx.act:
            # per expert: the mask and its bias-gradient column sums in one pass each, written in
            # place into the batched gradients
            dz = torch.empty_like(g)
            db = torch.empty(E, 1, g.shape[2], device=g.device, dtype=torch.float32)
            for e in range(E):
                _act_bwd(g[e], y[e], ctx.act, True, dz=dz[e], db=db[e, 0])
        else:
            dz, db = g, g.sum(1, keepdim=True)
        dx = torch.bmm(dz, k.transpose(1, 2)) if ctx.needs_input_grad[0] else None
        return dx, bwgrad(x, dz), db, None


def batched_linear(x, k, b, act: int = 0):
    return _BatchedLinearFn.apply(x, k, b, act)


_ACT_CODE = {"relu": 1, "sigmoid": 2}
# RS_SHARED_INPUT_DENSE=0: shared_input_dense runs the layers one by one (A/B switch)
_SHARED_INPUT = os.environ.get("RS_SHARED_INPUT_DENSE", "1") != "0"
_wgrad_stream: torch.cuda.Stream | None = None


class overlapped_weight_grads:
    """Context for a backward pass: Dense weight/bias gradients are computed on a second HIP
    stream and written straight into .grad, so the dX chain (and the memory-bound kernels on
    it, e.g. the interaction backward) runs beside the compute-bound weight-gradient GEMMs.
    On exit the current stream waits for that stream."""

    def __init__(self, device=None):
        self.stream = torch.cuda.Stream(device=device)

    def __enter__(self):
        global _wgrad_stream
        self._prev = _wgrad_stream
        _wgrad_stream = self.stream
        return self

    def __exit__(self, *exc):
        global _wgrad_stream
        torch.cuda.current_stream(self.stream.device).wait_stream(self.stream)
        _wgrad_stream = self._prev
        return False


def _accum_grad(param: torch.Tensor, g: torch.Tensor):
    if param.grad is None:
        param.grad = g
    else:
        param.grad.add_(g)


class _DenseFn(torch.autograd.Function):
    """y = act(x @ kernel[rows] + bias) for a Keras Dense layer (kernel [in, out]).

    backward: dz = act'(y)*dy and the bias gradient in one kernel (rs_act_bwd_colsum);
    dx = dz @ kernelᵀ; the weight gradient is a split-K batched GEMM (fixed chunking, fixed
    fold order: deterministic). Weight and bias gradients are written into .grad directly
    (on the overlapped weight-grad stream when one is active)."""

    @staticmethod
    def forward(ctx, x, handle, layer, rows, act=None):
        k = layer.kernel if rows is None else layer.kernel.index_select(0, rows)
        b = layer.bias
        act = layer.act_code if act is None else act
        # a row-strided x (a column block of a wider activation) goes to the GEMM in place
        xa = x if (x.dim() == 2 and x.stride(1) == 1 and x.stride(0) >= x.shape[1]) else x.contiguous()
        y = _affine(xa, k, b, act)
        ctx.layer, ctx.rows, ctx.act = layer, rows, act
        ctx.save_for_backward(x, k, y if act else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _lib as L

        x, k, y = ctx.saved_tensors
        layer, act = ctx.layer, ctx.act
        dy = dy.contiguous()
        B, fi = x.shape
        fo = dy.shape[1]
        main = torch.cuda.current_stream(dy.device)
        db = None
        if act or layer.bias is not None:
            dz = torch.empty_like(dy) if act else dy
            db = torch.empty(fo, device=dy.device, dtype=torch.float32)
            ws = torch.empty(max(1, L.lib().rs_act_bwd_colsum_workspace_size(B, fo) // 4),
                             device=dy.device)
            L.call("rs_act_bwd_colsum", L.ptr(dy), L.ptr(y), B, fo, act, L.ptr(dz), L.ptr(db),
                   L.ptr(ws), ws.numel() * 4, L.stream_ptr(dy.device))
        else:
            dz = dy
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (gemm_x3(dz, k.contiguous(), tb=True)
                  if _x3_ready(dz, k, n=k.shape[0], k=k.shape[1]) else dz @ k.t())
        side = _wgrad_stream
        if side is not None:
            side.wait_stream(main)
        with torch.cuda.stream(side if side is not None else main):
            dk = wgrad(x, dz)
            if ctx.rows is not None:
                full = torch.zeros_like(layer.kernel)
                full.index_copy_(0, ctx.rows, dk)
                dk = full
            _accum_grad(layer.kernel, dk)
            if db is not None and layer.bias is not None:
                _accum_grad(layer.bias, db)
        if side is not None:
            for t in (x, dz, db):
                if t is not None:
                    t.record_stream(side)
        return dx, None, None, None, None


class _SharedInputDenseFn(torch.autograd.Function):
    """act(x·k_i + b_i) for several Dense layers reading the same x — ESMM's CTR and CVR towers'
    first layers (esmm/esmm.py:27-28) — as ONE GEMM over the concatenated kernels: x is read
    once and the outputs are the column blocks of one [B, ΣN] activation (row stride ΣN, read in
    place by the next layers). Backward: each block masked from its own gradient into one dz
    with its bias gradient (rs_act_bwd_colsum_ld), one input-gradient GEMM over K = ΣN (the
    towers' contributions summed inside it: no add pass) and one split-K weight-gradient GEMM
    whose column blocks are the layers' kernel gradients (written into .grad as _DenseFn)."""

    @staticmethod
    def forward(ctx, x, act, layers, *handles):
        k = torch.cat([l.kernel for l in layers], dim=1)
        b = torch.cat([l.bias for l in layers])
        y = _affine(x.contiguous(), k, b, act)
        ctx.layers, ctx.act = layers, act
        ctx.save_for_backward(x, k, y)
        outs, o = [], 0
        for l in layers:
            outs.append(y[:, o:o + l.units])
            o += l.units
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        from . import _lib as L

        x, k, y = ctx.saved_tensors
        B, Nt = y.shape
        dz = torch.empty_like(y)
        db = torch.empty(Nt, device=y.device, dtype=torch.float32)
        o = 0
        for l, g in zip(ctx.layers, gs):
            n = l.units
            g = torch.zeros(B, n, device=y.device) if g is None else g
            if g.stride(-1) != 1:
                g = g.contiguous()
            ws = torch.empty(max(1, L.lib().rs_act_bwd_colsum_workspace_size(B, n) // 4),
                             device=y.device)
            L.call("rs_act_bwd_colsum_ld", L.ptr(g), g.stride(0), L.ptr(y[:, o:]), Nt, B, n,
                   ctx.act, L.ptr(dz[:, o:]), Nt, L.ptr(db[o:]), L.ptr(ws), ws.numel() * 4,
                   L.stream_ptr(y.device))
            o += n
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (gemm_x3(dz, k, tb=True) if _x3_ready(dz, k, n=k.shape[0], k=k.shape[1])
                  else dz @ k.t())
        main = torch.cuda.current_stream(y.device)
        side = _wgrad_stream
        if side is not None:
            side.wait_stream(main)
        with torch.cuda.stream(side if side is not None else main):
            dk = wgrad(x, dz)
            o = 0
            for l in ctx.layers:
                _accum_grad(l.kernel, dk[:, o:o + l.units].contiguous())
                _accum_grad(l.bias, db[o:o + l.units])
                o += l.units
        if side is not None:
            for t in (x, dz, db, dk):
                t.record_stream(side)
        return (dx, None, None) + (None,) * len(ctx.layers)


def shared_input_dense(x, layers):
    """[layer(x) for layer in layers] for built relu / sigmoid Dense layers with biases and one
    activation, as one GEMM (_SharedInputDenseFn); other cases run the layers one by one."""
    ok = (x.dim() == 2 and x.is_cuda and torch.is_grad_enabled() and len(layers) > 1
          and all(l.kernel is not None and l.bias is not None for l in layers)
          and len({l.act_code for l in layers}) == 1 and layers[0].act_code in (1, 2)
          and len({l.kernel.shape[0] for l in layers}) == 1 and _SHARED_INPUT)
    if not ok:
        return tuple(l(x) for l in layers)
    return _SharedInputDenseFn.apply(x, layers[0].act_code, tuple(layers),
                                     *[l._handle() for l in layers])


class _LinearChainFn(torch.autograd.Function):
    """A chain of Dense layers whose hidden layers are linear (ctr/layers.py:8: the reference's
    ctr MLP puts no activation on hidden layers): h_l = h_{l-1}·K_l + b_l, y = act(h_{L-1}·K_L
    + b_L). The forward is evaluated layer by layer exactly as the layerwise path (bit-identical
    outputs) or, composed=True, as the one affine map the chain is (chain_forward). The
    backward uses the chain's linearity twice:
      * every upstream gradient is the last layer's, G = act'(y)⊙dy, through a fixed matrix:
        g_l = G·Q_lᵀ with Q_l = K_{l+1}···K_L ([n_l, n_L]), so dK_l = (h_{l-1}ᵀ·G)·Q_lᵀ,
        db_l = s·Q_lᵀ (s = Σ_b G) and dx = G·Q_0ᵀ;
      * every hidden input is an affine map of the chain input, h_{l-1} = x·R_{l-1} + c_{l-1}
        (R_{l-1} = K_1···K_{l-1}, c_l = c_{l-1}·K_l + b_l), so h_{l-1}ᵀ·G = R_{l-1}ᵀ·(xᵀ·G) +
        c_{l-1}⊗s.
    The only batch-deep work left is A = xᵀ·G ([n_0, n_L], one split-K reduction), s, and dx;
    everything else is a product of weight-sized matrices. The same gradients in exact
    arithmetic as the layer-by-layer backward; only the fp32 summation order differs (as it does
    between any two GEMM tilings). tests/test_mlp_chain_gpu.py checks it against the float64
    layerwise oracle."""

    @staticmethod
    def forward(ctx, x, handle, layers, rows, composed=False):
        h, ks = chain_forward(x, layers, rows, composed)
        ctx.layers, ctx.rows = layers, rows
        ctx.save_for_backward(h if layers[-1].act_code else None, x, *ks)
        return h

    @staticmethod
    def backward(ctx, dy):
        layers, rows = ctx.layers, ctx.rows
        y, x, *ks = ctx.saved_tensors
        need_dx = ctx.needs_input_grad[0]
        G, A, s = chain_reduce(x, dy.contiguous(), y, layers[-1].act_code, need_g=need_dx)
        Q = chain_param_grads(layers, rows, ks, A, s, need_q0=need_dx)
        dx = G @ Q.t() if need_dx else None
        return dx, None, None, None, None


def chain_reduce(x, dy, y, act, need_g=True):
    """(G, A = xᵀ·G, s = Σ_b G) of a linear chain's last layer, G = act'(y) ⊙ dy: one fused
    deterministic pass (rs_chain_reduce) for the narrow shapes of the ctr MLPs, else the
    act_bwd_colsum kernel + a split-K reduction. G is None unless need_g (fused path)."""
    from . import _lib as L

    B, n0 = x.shape
    nl = dy.shape[1]
    vec_ok = (nl == 1 and n0 <= 1024 and n0 % 4 == 0 and x.stride(0) % 4 == 0
              and x.data_ptr() % 16 == 0)
    if x.stride(1) == 1 and (vec_ok or (nl > 1 and nl <= 256 and n0 <= 32)):
        out = torch.empty(n0 * nl + nl, device=dy.device, dtype=torch.float32)
        G = torch.empty_like(dy) if need_g else None
        nb = L.lib().rs_chain_reduce_workspace_size(B, n0, nl)
        ws = torch.empty(max(1, nb // 4), device=dy.device)
        L.call("rs_chain_reduce", L.ptr(x), x.stride(0), n0, L.ptr(dy), L.ptr(y), nl, act, B,
               L.ptr(out), L.ptr(G), L.ptr(ws), ws.numel() * 4, L.stream_ptr(dy.device))
        if G is None and act == 0 and need_g:
            G = dy
        return G, out[:n0 * nl].view(n0, nl), out[n0 * nl:]
    G = dy
    s = None
    if act:
        G = torch.empty_like(dy)
        s = torch.empty(nl, device=dy.device, dtype=torch.float32)
        ws = torch.empty(max(1, L.lib().rs_act_bwd_colsum_workspace_size(B, nl) // 4), device=dy.device)
        L.call("rs_act_bwd_colsum", L.ptr(dy), L.ptr(y), B, nl, act, L.ptr(G), L.ptr(s),
               L.ptr(ws), ws.numel() * 4, L.stream_ptr(dy.device))
    return G, wgrad(x, G), (s if s is not None else G.sum(0))


_pgrad_stream: torch.cuda.Stream | None = None


class overlapped_param_grads:
    """Context for a backward pass over linear chains: the parameter gradients (a dozen small
    products of weight-sized matrices per chain) are formed on a second HIP stream, beside the
    batch-sized kernels that follow (the interaction backward, the sparse apply); the input
    gradient's chain stays on the current stream. On exit the current stream waits for it."""

    def __init__(self, device=None):
        self.stream = torch.cuda.Stream(device=device)

    def __enter__(self):
        global _pgrad_stream
        self._prev = _pgrad_stream
        _pgrad_stream = self.stream
        return self

    def __exit__(self, *exc):
        global _pgrad_stream
        torch.cuda.current_stream(self.stream.device).wait_stream(self.stream)
        _pgrad_stream = self._prev
        return False


def chain_param_grads(layers, rows, ks, A, s, need_q0=True):
    """Accumulate every layer's kernel / bias gradient of a linear chain from A = xᵀ·G and
    s = Σ_b G (see _LinearChainFn); returns Q_0 = K_1···K_L for the input gradient G·Q_0ᵀ
    (None unless need_q0, narrow-input chains only).
    Qa[i] = K_{i+1}···K_L is formed on the current stream (the input gradient needs it); the
    rest, with h_{i}ᵀ·G = T_{i+1} + c_i⊗s where T_1 = A, T_{i+1} = K_iᵀ·T_i and
    c_i = K_iᵀ·c_{i-1} + b_i, runs on the overlapped parameter-gradient stream when one is
    active (matrix-vector chains when the output width is 1). A chain whose input is narrower
    than its output (the DLRM bottom MLP, 13 features) goes through _narrow_chain_grads."""
    n = len(layers)
    if (n == 3 and A.is_cuda and A.shape[1] == 1 and ks[2].shape[1] == 1
            and all(l.bias is not None for l in layers)):
        return _chain3_vec_grads(layers, rows, ks, A, s)
    if n > 1 and A.shape[0] < A.shape[1] and _pgrad_stream is None:
        if rows is None and narrow_chain_hip_ready(layers, A.shape[0]) and A.is_cuda:
            return _narrow_chain_grads_hip(layers, ks, A, s, need_q0)
        return _narrow_chain_grads(layers, rows, ks, A, s, need_q0)
    Qa = [None] * n  # Qa[i] = K_{i+1}···K_L (None: identity)
    for i in range(n - 2, -1, -1):
        Qa[i] = ks[i + 1] if Qa[i + 1] is None else ks[i + 1] @ Qa[i + 1]
    Q0 = ks[0] if Qa[0] is None else ks[0] @ Qa[0]
    side = _pgrad_stream if A.is_cuda else None
    if side is not None:
        side.wait_stream(torch.cuda.current_stream(A.device))
        for t in (A, s, *ks, *[q for q in Qa if q is not None]):
            t.record_stream(side)
    with (torch.cuda.stream(side) if side is not None else contextlib.nullcontext()):
        T, c = A, None
        for i in range(n):
            M = T if c is None else torch.addr(T, c, s)
            dk = M if Qa[i] is None else M @ Qa[i].t()
            layer = layers[i]
            if i == 0 and rows is not None:
                full = torch.zeros_like(layer.kernel)
                full.index_copy_(0, rows, dk)
                dk = full
            _accum_grad(layer.kernel, dk)
            if layer.bias is not None:
                _accum_grad(layer.bias, s if Qa[i] is None else Qa[i] @ s)
            if i < n - 1:
                b = layer.bias
                T = ks[i].t() @ T
                if c is None:
                    c = b if b is not None else torch.zeros(ks[i].shape[1], device=A.device)
                else:
                    c = torch.addmv(b, ks[i].t(), c) if b is not None else ks[i].t() @ c
    return Q0


def _narrow_chain_grads(layers, rows, ks, A, s, need_q0):
    """chain_param_grads for a chain whose input width n_0 is below its output width n_L: every
    batch-deep product is carried on the n_0 side. With R_i = K_1···K_i ([n_0, n_i]),
    h_iᵀ·G = R_iᵀ·A + c_i⊗s ([n_i, n_L]) and dK_{i+1} = (h_iᵀ·G)·K_Lᵀ···K_{i+2}ᵀ evaluated left
    to right, so no [n_i, n_L]-by-[n_L, n_{i+1}] chain product (K_{i+1}ᵀ·T_i, K_{i+1}···K_L) is
    ever formed: for the DLRM bottom MLP 13→512→256→128 that is ≈19 M multiply-adds instead of
    ≈51 M. Same gradients in exact arithmetic as the T-chain (tests/test_mlp_chain_cpu.py)."""
    n = len(layers)
    R = c = None
    for i in range(n):
        layer = layers[i]
        M = A if R is None else torch.addr(R.t() @ A, c, s)
        dk, db = M, s
        for j in range(n - 1, i, -1):
            dk = dk @ ks[j].t()
            db = ks[j] @ db
        if i == 0 and rows is not None:
            full = torch.zeros_like(layer.kernel)
            full.index_copy_(0, rows, dk)
            dk = full
        _accum_grad(layer.kernel, dk)
        if layer.bias is not None:
            _accum_grad(layer.bias, db)
        if i < n - 1:
            R = ks[0] if R is None else R @ ks[i]
            b = layer.bias
            if c is None:
                c = b if b is not None else torch.zeros(ks[i].shape[1], device=A.device, dtype=A.dtype)
            else:
                c = torch.addmv(b, ks[i].t(), c) if b is not None else ks[i].t() @ c
    if not need_q0:
        return None
    return R @ ks[n - 1]


_inv_cache: dict = {}


def _rows_i32(rows, n_full0):
    """(rows as int32, inverse map [n_full0] -> position or -1), cached per rows tensor."""
    if rows is None:
        return None, None
    key = (rows.data_ptr(), n_full0)
    hit = _inv_cache.get(key)
    if hit is None or hit[0] is not rows:
        r = rows.to(torch.int32).contiguous()
        inv = torch.full((n_full0,), -1, dtype=torch.int32, device=rows.device)
        inv[r.long()] = torch.arange(r.numel(), dtype=torch.int32, device=rows.device)
        hit = (rows, r, inv)
        _inv_cache[key] = hit
    return hit[1], hit[2]


def _chain3_vec_grads(layers, rows, ks, A, s):
    """chain_param_grads for a [n1, n2, 1] chain in three launches (rs_chain3_vec_grads)."""
    from . import _lib as L

    K1, K2, K3 = layers[0].kernel, layers[1].kernel, layers[2].kernel
    n_full0, n1 = K1.shape
    n2 = K2.shape[1]
    n0 = A.shape[0]
    dev = A.device
    r, inv = _rows_i32(rows, n_full0)
    dK1 = torch.empty_like(K1)
    dK2 = torch.empty_like(K2)
    dK3 = torch.empty_like(K3)
    db1 = torch.empty(n1, device=dev)
    db2 = torch.empty(n2, device=dev)
    db3 = torch.empty(1, device=dev)
    p = torch.empty(n0, 1, device=dev)
    ws = torch.empty(2 * n1 + 2 * n2, device=dev)
    L.call("rs_chain3_vec_grads", L.ptr(K1), L.ptr(r), L.ptr(inv), n_full0, n0,
           L.ptr(layers[0].bias), L.ptr(K2), L.ptr(layers[1].bias), L.ptr(K3), n1, n2,
           L.ptr(A.contiguous()), L.ptr(s.contiguous()), L.ptr(dK1), L.ptr(db1), L.ptr(dK2),
           L.ptr(db2), L.ptr(dK3), L.ptr(db3), L.ptr(p), L.ptr(ws), ws.numel() * 4,
           L.stream_ptr(dev))
    for layer, dk, db in zip(layers, (dK1, dK2, dK3), (db1, db2, db3)):
        _accum_grad(layer.kernel, dk)
        _accum_grad(layer.bias, db)
    return p


def chain_compose(layers, ks):
    """(Q_0, c_L) of a linear chain: its pre-activation output is x·Q_0 + c_L with
    Q_0 = K_1···K_L and c_L the biases carried through the later kernels. The products run in
    whichever order is cheaper (left to right for a narrow input, e.g. the DLRM bottom MLP's 13
    features; right to left for a narrow output, e.g. the top MLP's single logit); every product
    is weight-sized."""
    n = len(layers)
    n0, nl = ks[0].shape[0], ks[-1].shape[1]
    dev = ks[0].device
    if n0 <= nl:
        Q = ks[0]
        c = (layers[0].bias if layers[0].bias is not None
             else torch.zeros(ks[0].shape[1], device=dev, dtype=ks[0].dtype))
        for i in range(1, n):
            Q = Q @ ks[i]
            b = layers[i].bias
            c = torch.addmv(b, ks[i].t(), c) if b is not None else ks[i].t() @ c
        return Q, c
    Q = ks[-1]
    b = layers[-1].bias
    c = b.clone() if b is not None else torch.zeros(nl, device=dev, dtype=ks[0].dtype)
    for i in range(n - 2, -1, -1):  # Q = K_{i+1}···K_L here
        b = layers[i].bias
        if b is not None:
            c = torch.addmv(c, Q.t(), b)
        Q = ks[i] @ Q
    return Q, c


def chain_forward(x, layers, rows=None, composed=False):
    """Forward of a linear chain: (y, the kernels as used). Layer by layer (composed=False,
    bit-identical to the layerwise path) or, composed=True, as the single affine map the chain
    is, y = act(x·Q_0 + c_L) (chain_compose): one batch-deep GEMM of width n_L instead of one
    per layer. Both are the same function in exact arithmetic; they differ only in fp32
    rounding order (tests/test_mlp_chain_gpu.py bounds both against a float64 oracle)."""
    if composed and x.is_cuda:
        fast = _composed_forward_hip(x, layers, rows)
        if fast is not None:
            return fast
    ks = [layer.kernel if (i > 0 or rows is None) else layer.kernel.index_select(0, rows)
          for i, layer in enumerate(layers)]
    if composed:
        Q, c = chain_compose(layers, ks)
        h = torch.addmm(c, x, Q)
    else:
        h = x.contiguous()
        for i, (layer, k) in enumerate(zip(layers, ks)):
            last = i == len(layers) - 1
            h = _affine(h, k.contiguous(), layer.bias, layer.act_code if last else 0)
        return h, ks
    act = layers[-1].act_code
    if act == 1:
        h = torch.relu_(h)
    elif act == 2:
        h = torch.sigmoid_(h)
    return h, ks


def vec_chain_ready(layers, n0):
    """A [n1, n2, 1] chain with biases (the ctr top MLPs): the shapes rs_chain3_vec_compose and
    the rank-one backward (_chain3_vec_grads) take."""
    return (len(layers) == 3 and layers[2].kernel.shape[1] == 1 and n0 % 4 == 0 and n0 <= 1024
            and all(l.bias is not None for l in layers))


def vec_chain_compose(layers, rows, n0):
    """(q [n0], c [1]) of a [n1, n2, 1] chain: q = K1[rows]·K2·K3, c = its carried biases
    (rs_chain3_vec_compose, two launches)."""
    from . import _lib as L

    K1, K2, K3 = (l.kernel for l in layers)
    n1, n2 = K2.shape
    dev = K1.device
    r, _ = _rows_i32(rows, K1.shape[0])
    q = torch.empty(n0, device=dev)
    c = torch.empty(1, device=dev)
    ws = torch.empty(n1 + 1, device=dev)
    L.call("rs_chain3_vec_compose", L.ptr(K1), L.ptr(r), n0, L.ptr(layers[0].bias), L.ptr(K2),
           L.ptr(layers[1].bias), L.ptr(K3), L.ptr(layers[2].bias), n1, n2, L.ptr(q), L.ptr(c),
           L.ptr(ws), ws.numel() * 4, L.stream_ptr(dev))
    return q, c


_compose_cache: dict = {}


def cached_vec_chain_compose(layers, rows, n0):
    """vec_chain_compose, reusing a composition filed by store_composed (the dense tail's
    next-step product) while the layers' parameters are unchanged."""
    key = ("vec", id(layers[0].kernel), None if rows is None else rows.data_ptr(), n0)
    hit = _compose_cache.get(key)
    if hit is not None and hit[0] == _param_versions(layers) and hit[2]() is layers[0].kernel:
        return hit[1]
    return vec_chain_compose(layers, rows, n0)


def store_composed(bottom, bottom_comp, top, rows, n0, top_qc):
    """File compositions computed elsewhere (rs_dlrm_dense_tail) under the layers' current
    parameter versions: narrow_chain_compose / cached_vec_chain_compose then return them."""
    _compose_cache[id(bottom[0].kernel)] = (_param_versions(bottom), bottom_comp,
                                            weakref.ref(bottom[0].kernel))
    key = ("vec", id(top[0].kernel), None if rows is None else rows.data_ptr(), n0)
    _compose_cache[key] = (_param_versions(top), top_qc, weakref.ref(top[0].kernel))


def invalidate_compose_cache():
    """Drop every cached chain composition. Parameter updates replayed inside a HIP graph do not
    bump the tensors' version counters, so TrainStep calls this around captures and after each
    replay; eager updates invalidate entries through the version counters."""
    _compose_cache.clear()


def _param_versions(layers):
    return tuple((l.kernel.data_ptr(), l.kernel._version,
                  None if l.bias is None else (l.bias.data_ptr(), l.bias._version)) for l in layers)


def narrow_chain_compose(layers):
    """[R̃_2, ..., R̃_n] of a narrow-input chain, R̃_j = [K_1···K_j; c_j] ([n0+1, n_j]; the last
    is [Q_0; c_L]), by rs_chain_aug_product. Cached until a parameter changes (tensor version
    counters), so the backward reuses the forward's products."""
    from . import _lib as L

    key = id(layers[0].kernel)
    ver = _param_versions(layers)
    hit = _compose_cache.get(key)
    # the entry must belong to THIS kernel tensor (an id can be reused after a model is freed)
    if hit is not None and hit[0] == ver and hit[2]() is layers[0].kernel:
        return hit[1]
    ks = [l.kernel for l in layers]
    n0 = ks[0].shape[0]
    dev = ks[0].device
    st = L.stream_ptr(dev)
    outs, qa = [], None
    for i in range(1, len(layers)):
        k, nn_ = ks[i].shape
        out = torch.empty(n0 + 1, nn_, device=dev)
        M, ldm = (ks[0], ks[0].shape[1]) if qa is None else (qa, qa.shape[1])
        cin = layers[0].bias if qa is None else qa[n0]
        L.call("rs_chain_aug_product", L.ptr(M), ldm, n0, L.ptr(cin), L.ptr(ks[i]), k, nn_,
               L.ptr(layers[i].bias), L.ptr(out), st)
        outs.append(out)
        qa = out
    _compose_cache[key] = (ver, outs, weakref.ref(layers[0].kernel))
    return outs


def narrow_chain_hip_ready(layers, n0):
    """Shapes the narrow-chain HIP kernels take: n0 < 33 inputs, fp32, every width a multiple
    of 4 and (n0 + 1)·width within the LDS staging buffer."""
    ks = [l.kernel for l in layers]
    return (len(layers) >= 2 and n0 < 33 and ks[0].is_cuda
            and all(k.dtype == torch.float32 and k.is_contiguous() for k in ks)
            and all(k.shape[1] % 4 == 0 and (n0 + 1) * k.shape[0] <= 16896 for k in ks)
            and all(l.bias is None or l.bias.is_contiguous() for l in layers))


def _narrow_chain_grads_hip(layers, ks, A, s, need_q0):
    """_narrow_chain_grads on the HIP kernels (rs_chain_rt_product, rs_chain_outer): with
    Ã = [A; s], P_L = Ã and P_{j-1} = P_j·K_jᵀ, dK_j = R̃_{j-1}ᵀ·P_j and db_j = P_j[n0], where
    R̃_j = [K_1···K_j; c_j] are the forward composition's products (narrow_chain_compose) and
    R̃_0 = [I; 0]: every contraction is over n0 + 1 rows or a weight's width, ≈4 M multiply-adds
    for the DLRM bottom MLP instead of ≈19 M."""
    from . import _lib as L

    n = len(layers)
    n0, nl = A.shape
    dev = A.device
    st = L.stream_ptr(dev)
    comp = narrow_chain_compose(layers)
    P = torch.cat([A, s.reshape(1, nl)])
    for j in range(n - 1, -1, -1):
        layer = layers[j]
        n_in, n_out = ks[j].shape
        if j == 0:
            dk = P[:n0]
        else:
            if j == 1:
                R, ldr, rl = ks[0], ks[0].shape[1], layers[0].bias
            else:
                R = comp[j - 2]
                ldr, rl = R.shape[1], R[n0]
            dk = torch.empty(n_in, n_out, device=dev)
            L.call("rs_chain_outer", L.ptr(R), ldr, n0, L.ptr(rl), n_in, L.ptr(P), n_out,
                   L.ptr(dk), st)
        _accum_grad(layer.kernel, dk)
        if layer.bias is not None:
            _accum_grad(layer.bias, P[n0])
        if j > 0:
            Pn = torch.empty(n0 + 1, n_in, device=dev)
            L.call("rs_chain_rt_product", L.ptr(P), n0, L.ptr(ks[j]), n_out, n_in, L.ptr(Pn), st)
            P = Pn
    return comp[-1][:n0] if need_q0 else None


def _composed_forward_hip(x, layers, rows):
    """chain_forward(composed=True) through the HIP kernels for the two ctr chain shapes:
    a narrow input (n0 < 33, e.g. the DLRM bottom MLP's 13 features: rs_chain_aug_product
    composes [Q_0; c_L], rs_affine_narrow_fwd evaluates it) and a [n1, n2, 1] chain (the top
    MLPs: rs_chain3_vec_compose + rs_rowdot_act). None for other shapes (torch composition)."""
    from . import _lib as L

    B, n0 = x.shape
    n = len(layers)
    nl = layers[-1].kernel.shape[1]
    act = layers[-1].act_code
    dev = x.device
    f32 = x.dtype == torch.float32 and all(l.kernel.dtype == torch.float32 for l in layers)
    if not f32 or x.stride(1) != 1 or act not in (0, 1, 2):
        return None
    st = L.stream_ptr(dev)
    ks = [l.kernel for l in layers]
    if rows is None and nl <= 256 and narrow_chain_hip_ready(layers, n0):
        qa = narrow_chain_compose(layers)[-1]
        y = torch.empty(B, nl, device=dev)
        L.call("rs_affine_narrow_fwd", L.ptr(x), x.stride(0), B, n0, L.ptr(qa), nl, act,
               L.ptr(y), nl, st)
        return y, ks
    if (vec_chain_ready(layers, n0) and x.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0
            and (rows is None or rows.numel() == n0)):
        q, c = vec_chain_compose(layers, rows, n0)
        y = torch.empty(B, 1, device=dev)
        L.call("rs_rowdot_act", L.ptr(x), x.stride(0), B, n0, L.ptr(q), L.ptr(c), act, L.ptr(y), st)
        # ks[0] stays the full kernel: the backward of this shape (_chain3_vec_grads) reads the
        # layers' kernels through rows itself
        return y, ks
    return None


def linear_chain(x, layers, rows=None, handle=None, composed=False):
    """y of a Dense chain with linear hidden layers (see _LinearChainFn; composed: chain_forward)."""
    return _LinearChainFn.apply(x, handle if handle is not None else layers[-1]._handle(),
                                layers, rows, composed)


class Dense(nn.Module):
    def __init__(self, units: int, activation=None, use_bias: bool = True, in_features=None,
                 device=None, generator: torch.Generator | None = None):
        super().__init__()
        self.units = int(units)
        self.activation = get_activation(activation)
        # fused-kernel activation code: 0 linear, 1 relu, 2 sigmoid, -1 other (plain torch path)
        if activation is None or activation == "linear":
            self.act_code = 0
        elif isinstance(activation, str):
            self.act_code = _ACT_CODE.get(activation, -1)
        else:
            self.act_code = 1 if activation is torch.relu else 2 if activation is torch.sigmoid else -1
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

    def forward(self, x, rows: torch.Tensor | None = None):
        """rows: optional index of kernel rows to use (the input holds only those features;
        the other rows get an exactly-zero gradient)."""
        if self.kernel is None:
            self.build(x.shape[-1], x.device)
        if x.dim() == 2 and x.is_cuda and torch.is_grad_enabled():
            if self.act_code >= 0:
                return _DenseFn.apply(x, self._handle(), self, rows)
            # other activations (softmax, tanh, ...): fused linear + bias grad, then torch
            z = _DenseFn.apply(x, self._handle(), self, rows, 0)
            return self.activation(z) if self.activation is not None else z
        k = self.kernel if rows is None else self.kernel.index_select(0, rows)
        y = torch.matmul(x, k)
        if self.bias is not None:
            y = y + self.bias
        return self.activation(y) if self.activation is not None else y

    def preactivation(self, x):
        """x·kernel + bias without the activation (for callers that fuse it, e.g. MMOE's gate
        softmax inside rs_side_pool)."""
        if self.kernel is None:
            self.build(x.shape[-1], x.device)
        if x.dim() == 2 and x.is_cuda and torch.is_grad_enabled():
            return _DenseFn.apply(x, self._handle(), self, None, 0)
        y = torch.matmul(x, self.kernel)
        return y + self.bias if self.bias is not None else y

    def _handle(self):
        # a differentiable input so the Function is recorded whenever the params need grad
        if not hasattr(self, "_gh") or self._gh.device != self.kernel.device:
            self._gh = torch.zeros(0, device=self.kernel.device, requires_grad=True)
        return self._gh


def binary_crossentropy(y_true, y_pred, from_logits: bool = False, epsilon: float = 1e-7):
    """keras.losses.binary_crossentropy per example [3p TF 2.2 backend]: probabilities are
    clipped to [eps, 1-eps] and -(y log(p+eps) + (1-y) log(1-p+eps)); from_logits uses the
    stable sigmoid cross-entropy."""
    if from_logits:
        return F.binary_cross_entropy_with_logits(y_pred, y_true, reduction="none")
    p = torch.clamp(y_pred, epsilon, 1.0 - epsilon)
    return -(y_true * torch.log(p + epsilon) + (1.0 - y_true) * torch.log(1.0 - p + epsilon))
