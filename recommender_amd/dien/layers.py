"""dien/layers.py surface (reference dien/layers.py:1-204) on the MI355X engine.

The three recurrent pieces run in the HIP kernels of csrc/dien.hip (rs_gru_*, rs_augru_*,
rs_dien_attention_*): the kernels do the sequential part, the input projections of all steps
and every weight gradient are single GEMMs here. Parameters keep Keras layouts and
initialisers: GRU kernel [X,3H] glorot, recurrent_kernel [H,3H] orthogonal, bias [2,3H]
(input row, recurrent row; reset_after=True); AUGRUCell's three Dense layers on [h, x] /
[x, r·h]; DIENAttention kernel [H, X_target] glorot.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from .. import _lib as L
from ..nn import Dense, wgrad


def _glorot(shape, device, gen=None):
    lim = math.sqrt(6.0 / (shape[0] + shape[1]))
    on = gen.device if gen is not None else device
    return torch.empty(*shape, device=on).uniform_(-lim, lim, generator=gen).to(device)


def _mask_u8(mask, shape, device):
    if mask is None:
        return torch.ones(shape, dtype=torch.uint8, device=device)
    return mask.to(torch.uint8).contiguous()


# ---------------------------------------------------------------------------------------------
# The B·L-row products around the recurrences on the valid (mask != 0) steps only
# (csrc/dien_proj.hip): a masked step carries the state, so its input projection is never read
# and its gradient rows are exactly 0 — the library GEMMs over all B·L rows spent ≈1 ms of the
# cfg3 step on them. Widths beyond the kernels' (input > 64) keep the GEMMs.
_proj_ws: dict = {}


def _ws(name, nbytes, dev):
    key = (name, dev)
    b = _proj_ws.get(key)
    if b is None or b.numel() < nbytes:
        b = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=dev)
        _proj_ws[key] = b
    return b


def _rows_ready(X, H):
    return X <= 64 and H <= 64


def _valid_rows(mask_u8):
    """(idx [R] int32, count [1] int32) of the rows with mask != 0, in order (on the device).
    Kept on the mask tensor object with its version counter, so the layers of one forward that
    share it (the GRU and the AUGRU of DIEN) list the rows once, and a mask buffer refilled in
    place (a static step's inputs, an eval loop) is listed again."""
    got = getattr(mask_u8, "_rs_valid_rows", None)
    if got is not None and got[0] == mask_u8._version:
        return got[1]
    rows = _valid_rows_list(mask_u8)
    mask_u8._rs_valid_rows = (mask_u8._version, rows)
    return rows


def _valid_rows_list(mask_u8):
    dev, R = mask_u8.device, mask_u8.numel()
    idx = torch.empty(R, dtype=torch.int32, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)
    nb = L.lib().rs_valid_rows_workspace_size(R)
    ws = _ws("valid_rows", nb, dev)
    L.call("rs_valid_rows", L.ptr(mask_u8), R, L.ptr(idx), L.ptr(cnt), L.ptr(ws), ws.numel(),
           L.stream_ptr(dev))
    return idx, cnt


def _ld(t):
    if t.stride(-1) != 1:
        raise ValueError("row-major views only")
    return t.stride(0)


def _masked_proj(x2, W, bias, vr):
    """x2 [R, K]·W [K, N] + bias on the listed rows; other rows of the result are undefined."""
    R, K = x2.shape
    N = W.shape[1]
    y = torch.empty(R, N, device=x2.device)
    L.call("rs_masked_proj", L.ptr(x2), _ld(x2), L.ptr(W.contiguous()), L.ptr(bias), L.ptr(vr[0]),
           L.ptr(vr[1]), R, K, N, L.ptr(y), N, L.stream_ptr(x2.device))
    return y


def _masked_dx(d2, W, mask_u8, vr):
    """d2 [R, N]·Wᵀ (W [K, N]) on the listed rows (vr = _valid_rows(mask_u8)), 0 where the mask
    is 0."""
    R, N = d2.shape
    K = W.shape[0]
    dx = torch.empty(R, K, device=d2.device)
    L.call("rs_masked_dx", L.ptr(d2), _ld(d2), L.ptr(W.contiguous()), L.ptr(mask_u8),
           L.ptr(vr[0]), L.ptr(vr[1]), R, K, N, L.ptr(dx), K, L.stream_ptr(d2.device))
    return dx


def _masked_wgrad(A2, shift_L, D2, vr, sums=True):
    """(Σ_listed A_rᵀ·D_r [K, N], Σ_listed D_r [N] or None); shift_L > 0: A_r = row r - 1 within
    each length-shift_L sequence (0 at its first step)."""
    K, N = A2.shape[1], D2.shape[1]
    dev = D2.device
    C = torch.empty(K, N, device=dev)
    s = torch.empty(N, device=dev) if sums else None
    nb = L.lib().rs_masked_wgrad_workspace_size(K, N)
    ws = _ws("masked_wgrad", nb, dev)
    L.call("rs_masked_wgrad", L.ptr(A2), _ld(A2), shift_L, L.ptr(D2), _ld(D2), L.ptr(vr[0]),
           L.ptr(vr[1]), K, N, L.ptr(C), L.ptr(s), L.ptr(ws), ws.numel(), L.stream_ptr(dev))
    return C, s


# ---------------------------------------------------------------------------------------------
class _GRUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kernel, recurrent_kernel, bias, mask_u8):
        B, T, X = x.shape
        H = recurrent_kernel.shape[0]
        rows = _rows_ready(X, H)
        if rows:
            vr = _valid_rows(mask_u8)
            xw = _masked_proj(x.reshape(-1, X), kernel, bias[0], vr).view(B, T, 3 * H)
        else:
            vr = (None, None)
            xw = torch.addmm(bias[0], x.reshape(-1, X), kernel).view(B, T, 3 * H)
        out = torch.empty(B, T, H, device=x.device)
        saved = torch.empty(B, T, 4 * H, device=x.device)
        rk = recurrent_kernel.contiguous()
        L.call("rs_gru_fwd", L.ptr(xw), L.ptr(rk), L.ptr(bias[1].contiguous()), L.ptr(mask_u8), B, T,
               H, L.ptr(out), L.ptr(saved), L.stream_ptr(x.device))
        ctx.save_for_backward(x, kernel, rk, out, saved, mask_u8, *vr)
        ctx.rows = rows
        return out

    @staticmethod
    def backward(ctx, dout):
        x, kernel, rk, out, saved, mask_u8, idx, cnt = ctx.saved_tensors
        B, T, X = x.shape
        H = rk.shape[0]
        dout = dout.contiguous()
        dxw = torch.empty(B, T, 3 * H, device=x.device)
        dinner = torch.empty(B, T, 3 * H, device=x.device)
        # the valid-row kernels below read only the valid steps' rows: the masked ones stay unwritten
        skip = L.RS_DIEN_SKIP_MASKED_ROWS if ctx.rows else 0
        L.call("rs_gru_bwd", L.ptr(dout), L.ptr(out), L.ptr(saved), L.ptr(rk), L.ptr(mask_u8), B, T,
               H, L.ptr(dxw), L.ptr(dinner), skip, L.stream_ptr(x.device))
        dxw2, din2 = dxw.view(-1, 3 * H), dinner.view(-1, 3 * H)
        if ctx.rows:
            vr = (idx, cnt)
            m = mask_u8.reshape(-1)
            dx = _masked_dx(dxw2, kernel, m, vr).view(B, T, X) if ctx.needs_input_grad[0] else None
            dk, db0 = _masked_wgrad(x.reshape(-1, X), 0, dxw2, vr)
            drk, db1 = _masked_wgrad(out.view(-1, H), T, din2, vr)
            return dx, dk, drk, torch.stack([db0, db1]), None
        hp = torch.cat([torch.zeros(B, 1, H, device=x.device), out[:, :-1]], 1).reshape(-1, H)
        dx = (dxw2 @ kernel.t()).view(B, T, X) if ctx.needs_input_grad[0] else None
        dk = wgrad(x.reshape(-1, X), dxw2)
        drk = wgrad(hp, din2)
        db = torch.stack([dxw2.sum(0), din2.sum(0)])
        return dx, dk, drk, db, None


class GRU(nn.Module):
    """keras.layers.GRU(units, return_sequences=True) [3p TF 2.2: reset_after=True, sigmoid
    recurrent activation, tanh activation]; masked steps carry the state."""

    def __init__(self, units, input_dim=None, device=None, generator=None):
        super().__init__()
        self.units = units
        self._device, self._gen = device, generator
        self.kernel = None
        if input_dim is not None:
            self.build(input_dim)

    def build(self, input_dim, device=None):
        dev = device or self._device or "cuda"
        H = self.units
        self.kernel = nn.Parameter(_glorot((input_dim, 3 * H), dev, self._gen))
        rk = torch.empty(3 * H, H)
        # orthogonal init [3p keras] runs on the host (QR): a CPU generator seeded from the
        # model's generator, so two models built from equal seeds are equal (the global host RNG
        # made them differ: the round-2 "DIEN graph step" discrepancy)
        g = self._gen
        if g is not None and g.device.type != "cpu":
            seed = int(torch.randint(0, 2 ** 62, (1,), device=g.device, generator=g).item())
            g = torch.Generator().manual_seed(seed)
        nn.init.orthogonal_(rk, generator=g)
        self.recurrent_kernel = nn.Parameter(rk.t().contiguous().to(dev))
        self.bias = nn.Parameter(torch.zeros(2, 3 * H, device=dev))

    def forward(self, x, mask=None):
        if self.kernel is None:
            self.build(x.shape[-1], x.device)
        L.require_device(x, "GRU input")
        m = _mask_u8(mask, x.shape[:2], x.device)
        return _GRUFn.apply(x.contiguous(), self.kernel, self.recurrent_kernel, self.bias, m)


# ---------------------------------------------------------------------------------------------
class _AUGRUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, att, ku, bu, kr, br, kh, bh, mask_u8):
        B, T, X = x.shape
        H = ku.shape[1]
        # x parts: update/reset kernels take [h, x] (rows H: are x), candidate takes [x, r·h]
        wx = torch.cat([ku[H:], kr[H:], kh[:X]], dim=1)                 # [X, 3H]
        bx = torch.cat([bu, br, bh])
        rows = _rows_ready(X, H)
        if rows:
            vr = _valid_rows(mask_u8)
            xw = _masked_proj(x.reshape(-1, X), wx, bx, vr).view(B, T, 3 * H)
        else:
            vr = (None, None)
            xw = torch.addmm(bx, x.reshape(-1, X), wx).view(B, T, 3 * H)
        ctx.rows = rows
        kuh, krh, khr = ku[:H].contiguous(), kr[:H].contiguous(), kh[X:].contiguous()
        final = torch.empty(B, H, device=x.device)
        states = torch.empty(B, T, H, device=x.device)
        saved = torch.empty(B, T, 4 * H, device=x.device)
        a = att.reshape(B, T).contiguous()
        L.call("rs_augru_fwd", L.ptr(xw), L.ptr(a), L.ptr(kuh), L.ptr(krh), L.ptr(khr),
               L.ptr(mask_u8), B, T, H, L.ptr(final), L.ptr(states), L.ptr(saved),
               L.RS_DIEN_SKIP_MASKED_ROWS if rows else 0, L.stream_ptr(x.device))
        ctx.save_for_backward(x, a, wx, kuh, krh, khr, states, saved, mask_u8, *vr)
        ctx.att_shape = att.shape
        return final

    @staticmethod
    def backward(ctx, dfinal):
        x, a, wx, kuh, krh, khr, states, saved, mask_u8, idx, cnt = ctx.saved_tensors
        B, T, X = x.shape
        H = kuh.shape[0]
        dxw = torch.empty(B, T, 3 * H, device=x.device)
        datt = torch.empty(B, T, device=x.device)
        L.call("rs_augru_bwd", L.ptr(dfinal.contiguous()), L.ptr(a), L.ptr(states), L.ptr(saved),
               L.ptr(kuh), L.ptr(krh), L.ptr(khr), L.ptr(mask_u8), B, T, H, L.ptr(dxw),
               L.ptr(datt), L.RS_DIEN_SKIP_MASKED_ROWS if ctx.rows else 0, L.stream_ptr(x.device))
        d2 = dxw.view(-1, 3 * H)
        dpu, dpr, dph = d2[:, :H], d2[:, H:2 * H], d2[:, 2 * H:]
        x2 = x.reshape(-1, X)
        if ctx.rows:
            vr = (idx, cnt)
            dwx, sb = _masked_wgrad(x2, 0, d2, vr)                        # [X, 3H], Σ rows
            dhur, _ = _masked_wgrad(states.view(-1, H), T, d2[:, :2 * H], vr, sums=False)
            dkhr, _ = _masked_wgrad(saved.view(-1, 4 * H)[:, 3 * H:], 0, dph, vr, sums=False)
            dku = torch.cat([dhur[:, :H], dwx[:, :H]], 0)
            dkr = torch.cat([dhur[:, H:], dwx[:, H:2 * H]], 0)
            dkh = torch.cat([dwx[:, 2 * H:], dkhr], 0)
            dx = (_masked_dx(d2, wx, mask_u8.reshape(-1), vr).view(B, T, X)
                  if ctx.needs_input_grad[0] else None)
            return (dx, datt.view(ctx.att_shape), dku, sb[:H], dkr, sb[H:2 * H], dkh, sb[2 * H:],
                    None)
        hp = torch.cat([torch.zeros(B, 1, H, device=x.device), states[:, :-1]], 1).reshape(-1, H)
        rh = saved[:, :, 3 * H:].reshape(-1, H)
        dwx = wgrad(x2, d2)                                               # [X, 3H]
        dhur = wgrad(hp, d2[:, :2 * H])                                   # [H, 2H]
        dku = torch.cat([dhur[:, :H], dwx[:, :H]], 0)
        dkr = torch.cat([dhur[:, H:], dwx[:, H:2 * H]], 0)
        dkh = torch.cat([dwx[:, 2 * H:], wgrad(rh, dph)], 0)
        dx = (d2 @ wx.t()).view(B, T, X) if ctx.needs_input_grad[0] else None
        return (dx, datt.view(ctx.att_shape), dku, dpu.sum(0), dkr, dpr.sum(0), dkh, dph.sum(0),
                None)


class AUGRUCell(nn.Module):
    """dien/layers.py:161-188: update/reset gates Dense(H, sigmoid) on [h_prev, x], candidate
    Dense(H, tanh) on [x, r·h_prev]; u ← a·u; h = u·hh + (1-u)·h_prev."""

    def __init__(self, units, input_dim, device=None, generator=None):
        super().__init__()
        self.units = units
        H, X = units, input_dim
        self.update_gate = Dense(H, "sigmoid", in_features=H + X, device=device, generator=generator)
        self.reset_gate = Dense(H, "sigmoid", in_features=H + X, device=device, generator=generator)
        self.hidden_layer = Dense(H, "tanh", in_features=X + H, device=device, generator=generator)

    @property
    def state_size(self):
        return self.units


class InterestEvolve(nn.Module):
    """dien/layers.py:191-204: keras.layers.RNN(AUGRUCell) over [history_state, score], masked
    steps carry the state, returns the last state [B, H]."""

    def __init__(self, gru_units, input_dim=None, device=None, generator=None):
        super().__init__()
        self.gru_units = gru_units
        self.augru = AUGRUCell(gru_units, input_dim if input_dim is not None else gru_units, device,
                               generator)

    def forward(self, inputs, training=False, mask=None):
        history_state, attention_score = inputs
        c = self.augru
        m = _mask_u8(mask, history_state.shape[:2], history_state.device)
        return _AUGRUFn.apply(history_state.contiguous(), attention_score, c.update_gate.kernel,
                              c.update_gate.bias, c.reset_gate.kernel, c.reset_gate.bias,
                              c.hidden_layer.kernel, c.hidden_layer.bias, m)


# ---------------------------------------------------------------------------------------------
class _AttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, target, hidden, kernel, mask_u8):
        B, T, H = hidden.shape
        t2 = target.reshape(B, -1)
        q = (t2 @ kernel.t()).contiguous()                          # q = K·t  [B, H]
        a = torch.empty(B, T, device=hidden.device)
        hs = hidden.contiguous()
        L.call("rs_dien_attention_fwd", L.ptr(hs), L.ptr(q), L.ptr(mask_u8), B, T, H, L.ptr(a),
               L.stream_ptr(hidden.device))
        ctx.save_for_backward(t2, hs, kernel, q, a)
        ctx.tshape = target.shape
        return a.unsqueeze(-1)

    @staticmethod
    def backward(ctx, da):
        t2, hs, kernel, q, a = ctx.saved_tensors
        B, T, H = hs.shape
        dhs = torch.empty_like(hs)
        dq = torch.empty(B, H, device=hs.device)
        L.call("rs_dien_attention_bwd", L.ptr(hs), L.ptr(q), L.ptr(a),
               L.ptr(da.reshape(B, T).contiguous()), B, T, H, L.ptr(dhs), L.ptr(dq),
               L.stream_ptr(hs.device))
        dk = dq.t() @ t2                                              # [H, Xt]
        dt = (dq @ kernel).view(ctx.tshape)
        return dt, dhs, dk, None


class _AttentionEvolveFn(torch.autograd.Function):
    """DIENAttention then InterestEvolve (dien/model.py:71-73) as one node: the same kernels as
    _AttentionFn + _AUGRUFn; the backward runs the AUGRU recurrence, then the attention
    backward on its score gradient, and the attention's part of dL/dhidden is the addend of the
    AUGRU's input-gradient kernel (rs_masked_dx_acc) — the sum autograd would form, no add pass."""

    @staticmethod
    def forward(ctx, target, hidden, att_kernel, mask_u8, ku, bu, kr, br, kh, bh):
        B, T, H = hidden.shape
        X = H
        dev = hidden.device
        st = L.stream_ptr(dev)
        hs = hidden.contiguous()
        t2 = target.reshape(B, -1)
        q = (t2 @ att_kernel.t()).contiguous()
        a = torch.empty(B, T, device=dev)
        L.call("rs_dien_attention_fwd", L.ptr(hs), L.ptr(q), L.ptr(mask_u8), B, T, H, L.ptr(a), st)
        Hh = ku.shape[1]
        wx = torch.cat([ku[Hh:], kr[Hh:], kh[:X]], dim=1)
        bx = torch.cat([bu, br, bh])
        vr = _valid_rows(mask_u8)
        xw = _masked_proj(hs.reshape(-1, X), wx, bx, vr).view(B, T, 3 * Hh)
        kuh, krh, khr = ku[:Hh].contiguous(), kr[:Hh].contiguous(), kh[X:].contiguous()
        final = torch.empty(B, Hh, device=dev)
        states = torch.empty(B, T, Hh, device=dev)
        saved = torch.empty(B, T, 4 * Hh, device=dev)
        L.call("rs_augru_fwd", L.ptr(xw), L.ptr(a), L.ptr(kuh), L.ptr(krh), L.ptr(khr),
               L.ptr(mask_u8), B, T, Hh, L.ptr(final), L.ptr(states), L.ptr(saved),
               L.RS_DIEN_SKIP_MASKED_ROWS, st)
        ctx.save_for_backward(t2, hs, att_kernel, q, a, wx, kuh, krh, khr, states, saved, mask_u8,
                              *vr)
        ctx.tshape = target.shape
        return final

    @staticmethod
    def backward(ctx, dfinal):
        (t2, hs, att_kernel, q, a, wx, kuh, krh, khr, states, saved, mask_u8, idx,
         cnt) = ctx.saved_tensors
        B, T, X = hs.shape
        Hh = kuh.shape[0]
        dev = hs.device
        st = L.stream_ptr(dev)
        dxw = torch.empty(B, T, 3 * Hh, device=dev)
        datt = torch.empty(B, T, device=dev)
        L.call("rs_augru_bwd", L.ptr(dfinal.contiguous()), L.ptr(a), L.ptr(states), L.ptr(saved),
               L.ptr(kuh), L.ptr(krh), L.ptr(khr), L.ptr(mask_u8), B, T, Hh, L.ptr(dxw),
               L.ptr(datt), L.RS_DIEN_SKIP_MASKED_ROWS, st)
        # attention backward on the score gradient
        dhs = torch.empty_like(hs)
        dq = torch.empty(B, X, device=dev)
        L.call("rs_dien_attention_bwd", L.ptr(hs), L.ptr(q), L.ptr(a), L.ptr(datt), B, T, X,
               L.ptr(dhs), L.ptr(dq), st)
        datt_k = dq.t() @ t2
        dt = (dq @ att_kernel).view(ctx.tshape)
        d2 = dxw.view(-1, 3 * Hh)
        vr = (idx, cnt)
        x2 = hs.reshape(-1, X)
        dwx, sb = _masked_wgrad(x2, 0, d2, vr)
        dhur, _ = _masked_wgrad(states.view(-1, Hh), T, d2[:, :2 * Hh], vr, sums=False)
        dkhr, _ = _masked_wgrad(saved.view(-1, 4 * Hh)[:, 3 * Hh:], 0, d2[:, 2 * Hh:], vr,
                                sums=False)
        dku = torch.cat([dhur[:, :Hh], dwx[:, :Hh]], 0)
        dkr = torch.cat([dhur[:, Hh:], dwx[:, Hh:2 * Hh]], 0)
        dkh = torch.cat([dwx[:, 2 * Hh:], dkhr], 0)
        # dL/dhidden = the AUGRU's input gradient + the attention's (the addend)
        dx = torch.empty_like(hs)
        L.call("rs_masked_dx_acc", L.ptr(d2), _ld(d2), L.ptr(wx), L.ptr(mask_u8.reshape(-1)),
               L.ptr(idx), L.ptr(cnt), B * T, X, 3 * Hh, L.ptr(dhs), X, L.ptr(dx), X, st)
        return (dt, dx, datt_k, None, dku, sb[:Hh], dkr, sb[Hh:2 * Hh], dkh, sb[2 * Hh:])


def attention_evolve(attention, evolve, target, hidden, mask):
    """evolve((hidden, attention((target, hidden), mask=mask)), mask=mask) as one node when the
    kernels take the shapes (_AttentionEvolveFn), else the two layers."""
    c = evolve.augru
    H = hidden.shape[-1]
    if attention.kernel is None:
        attention.build(H, target.shape[-1], hidden.device)
    if (hidden.is_cuda and torch.is_grad_enabled() and c.units == H and _rows_ready(H, H)
            and attention.kernel.shape == (H, target.shape[-1])):
        m = _mask_u8(mask, hidden.shape[:2], hidden.device)
        return _AttentionEvolveFn.apply(target, hidden, attention.kernel, m,
                                        c.update_gate.kernel, c.update_gate.bias,
                                        c.reset_gate.kernel, c.reset_gate.bias,
                                        c.hidden_layer.kernel, c.hidden_layer.bias)
    score = attention((target, hidden), mask=mask)
    return evolve((hidden, score), mask=mask)


class DIENAttention(nn.Module):
    """dien/layers.py:136-158: score = softmax_L((H·K)·tᵀ + (1-mask)·(-1e9)) → [B, L, 1]."""

    def __init__(self, hidden_dim=None, target_dim=None, device=None, generator=None):
        super().__init__()
        self._device, self._gen = device, generator
        self.kernel = None
        if hidden_dim is not None and target_dim is not None:
            self.build(hidden_dim, target_dim)

    def build(self, hidden_dim, target_dim, device=None):
        self.kernel = nn.Parameter(_glorot((hidden_dim, target_dim), device or self._device or "cuda", self._gen))

    def forward(self, inputs, training=False, mask=None):
        target, hidden_state = inputs
        if self.kernel is None:
            self.build(hidden_state.shape[-1], target.shape[-1], hidden_state.device)
        m = _mask_u8(mask, hidden_state.shape[:2], hidden_state.device)
        return _AttentionFn.apply(target, hidden_state, self.kernel, m)


# ---------------------------------------------------------------------------------------------
class _BatchNormFn(torch.autograd.Function):
    """BatchNormalization on [B, C] rows in two launches per direction (csrc/batchnorm.hip:
    batch statistics, normalisation and the moving-average update in the forward; Σ dy,
    Σ dy·x̂ and dx in the backward) instead of a dozen elementwise / reduction passes each."""

    @staticmethod
    def forward(ctx, x, gamma, beta, bn, training):
        x = x.contiguous()
        B, C = x.shape
        dev = x.device
        y = torch.empty_like(x)
        mean = torch.empty(C, device=dev)
        invstd = torch.empty(C, device=dev)
        ws = _ws("batch_norm", L.lib().rs_batch_norm_workspace_size(B, C), dev)
        L.call("rs_batch_norm_fwd", L.ptr(x), B, C, L.ptr(gamma), L.ptr(beta), bn.epsilon,
               bn.momentum, int(training), L.ptr(bn.moving_mean), L.ptr(bn.moving_variance),
               L.ptr(y), L.ptr(mean), L.ptr(invstd), L.ptr(ws), ws.numel(), L.stream_ptr(dev))
        ctx.save_for_backward(x, gamma, mean, invstd)
        ctx.training = training
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, mean, invstd = ctx.saved_tensors
        B, C = x.shape
        dev = x.device
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        dgamma = torch.empty(C, device=dev)
        dbeta = torch.empty(C, device=dev)
        ws = _ws("batch_norm_bwd", L.lib().rs_batch_norm_workspace_size(B, C), dev)
        L.call("rs_batch_norm_bwd", L.ptr(dy), L.ptr(x), B, C, L.ptr(mean), L.ptr(invstd),
               L.ptr(gamma), int(ctx.training), L.ptr(dx), L.ptr(dgamma), L.ptr(dbeta), L.ptr(ws),
               ws.numel(), L.stream_ptr(dev))
        return dx, dgamma, dbeta, None, None


class BatchNormalization(nn.Module):
    """keras.layers.BatchNormalization [3p]: momentum 0.99, epsilon 1e-3; training → batch
    statistics + moving-average update; inference → moving statistics."""

    def __init__(self, dim, momentum=0.99, epsilon=1e-3, device=None):
        super().__init__()
        self.momentum, self.epsilon = momentum, epsilon
        self.gamma = nn.Parameter(torch.ones(dim, device=device))
        self.beta = nn.Parameter(torch.zeros(dim, device=device))
        self.register_buffer("moving_mean", torch.zeros(dim, device=device))
        self.register_buffer("moving_variance", torch.ones(dim, device=device))

    def forward(self, x, training=False):
        if x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and x.shape[0] > 0:
            return _BatchNormFn.apply(x, self.gamma, self.beta, self, bool(training))
        if training:
            mean = x.mean(0)
            var = x.var(0, unbiased=False)  # tf.nn.moments: the population variance
            with torch.no_grad():
                # keras _assign_moving_average: var -= (var - value) * (1 - momentum)
                decay = 1.0 - self.momentum
                self.moving_mean.sub_((self.moving_mean - mean.detach()) * decay)
                self.moving_variance.sub_((self.moving_variance - var.detach()) * decay)
        else:
            mean, var = self.moving_mean, self.moving_variance
        return (x - mean) * torch.rsqrt(var + self.epsilon) * self.gamma + self.beta


def compute_his_average(his_embedding, mask):
    """dien/layers.py:5-17: masked mean over the history (0/0 → NaN for an empty history)."""
    m = mask.unsqueeze(-1).to(his_embedding.dtype)
    return (his_embedding * m).sum(1) / m.sum(1)


class MLP(nn.Module):
    """dien/layers.py:20-31: BatchNormalization on the input, relu hidden layers."""

    def __init__(self, units, last_activation, in_features, device=None, generator=None):
        super().__init__()
        self.bn = BatchNormalization(in_features, device=device)
        layers, fin = [], in_features
        for u in units[:-1]:
            layers.append(Dense(u, "relu", in_features=fin, device=device, generator=generator))
            fin = u
        layers.append(Dense(units[-1], last_activation, in_features=fin, device=device, generator=generator))
        self.mlp = nn.ModuleList(layers)

    def forward(self, inputs, training=False):
        x = self.bn(inputs, training=training)
        for layer in self.mlp:
            x = layer(x)
        return x


class LocalActivationUnit(nn.Module):
    """dien/layers.py:34-59 (DIN): unnormalised weights Dense(80σ)→Dense(40σ)→Dense(1) on
    [t, h, t-h, t·h], masked, then weightsᵀ·H."""

    def __init__(self, dim, device=None, generator=None):
        super().__init__()
        self.layer_1 = Dense(80, "sigmoid", in_features=4 * dim, device=device, generator=generator)
        self.layer_2 = Dense(40, "sigmoid", in_features=80, device=device, generator=generator)
        self.layer_3 = Dense(1, None, in_features=40, device=device, generator=generator)

    def forward(self, inputs, mask=None):
        target, history = inputs
        B, T, D = history.shape
        t = target.expand(B, T, D)
        c = torch.cat([t, history, t - history, t * history], -1).reshape(B * T, 4 * D)
        w = self.layer_3(self.layer_2(self.layer_1(c))).view(B, T, 1)
        w = w * mask.unsqueeze(-1).to(w.dtype)
        return (w.transpose(1, 2) @ history).squeeze(1)


class AuxiliaryNet(nn.Module):
    """dien/layers.py:62-73: Dense(80σ) → Dense(40σ) → Dense(1)."""

    def __init__(self, mlp_units, in_features, device=None, generator=None):
        super().__init__()
        layers, fin = [], in_features
        for u in mlp_units[:-1]:
            layers.append(Dense(u, "sigmoid", in_features=fin, device=device, generator=generator))
            fin = u
        layers.append(Dense(mlp_units[-1], None, in_features=fin, device=device, generator=generator))
        self.layers = nn.ModuleList(layers)

    def forward(self, inputs, training=False, **kwargs):
        shp = inputs.shape
        x = inputs.reshape(-1, shp[-1])
        for layer in self.layers:
            x = layer(x)
        return x.view(*shp[:-1], -1)


class _AuxLossFn(torch.autograd.Function):
    """InterestExtract.compute_auxiliary_loss on the fused kernels (csrc/dien_aux.hip):
    the aux net is evaluated only on the 16-row tiles that hold a valid (m = 1) row and its
    [rows, 80] activations never reach HBM; the backward recomputes them."""

    @staticmethod
    def forward(ctx, hidden, pos, neg, mask_u8, W1, b1, W2, b2, W3, b3):
        B, Lh, H = hidden.shape
        E = pos.shape[-1]
        aux = torch.empty(B, device=hidden.device)
        ws = (hidden, pos, neg, mask_u8, B, Lh, H, E, W1, b1, W2, b2, W3, b3)
        L.call("rs_dien_aux_fwd", *[L.ptr(x) if isinstance(x, torch.Tensor) else x for x in ws],
               L.ptr(aux), L.stream_ptr(hidden.device))
        ctx.save_for_backward(hidden, pos, neg, mask_u8, W1, b1, W2, b2, W3, b3)
        return aux

    @staticmethod
    def backward(ctx, daux):
        hidden, pos, neg, mask_u8, W1, b1, W2, b2, W3, b3 = ctx.saved_tensors
        B, Lh, H = hidden.shape
        E = pos.shape[-1]
        dev = hidden.device
        dh = torch.empty_like(hidden)
        dp = torch.empty_like(pos)
        dn = torch.empty_like(neg)
        In, n1, n2 = H + E, W1.shape[1], W2.shape[1]
        dparams = torch.empty(In * n1 + n1 + n1 * n2 + n2 + n2 + 1, device=dev)
        ws = _aux_workspace(B, Lh, H, E, dev)
        args = (hidden, pos, neg, mask_u8, B, Lh, H, E, W1, b1, W2, b2, W3, b3,
                daux.contiguous(), dh, dp, dn, dparams, ws)
        L.call("rs_dien_aux_bwd", *[L.ptr(x) if isinstance(x, torch.Tensor) else x for x in args],
               ws.numel(), L.stream_ptr(dev))
        o = 0
        outs = []
        for shape in (W1.shape, b1.shape, W2.shape, b2.shape, W3.shape, b3.shape):
            n = int(torch.Size(shape).numel())
            outs.append(dparams[o:o + n].view(shape))
            o += n
        return (dh, dp, dn, None, *outs)


_aux_ws: dict = {}


def _aux_workspace(B, Lh, H, E, dev):
    nb = L.lib().rs_dien_aux_workspace_size(B, Lh, H, E)
    ws = _aux_ws.get(dev)
    if ws is None or ws.numel() < nb:
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        _aux_ws[dev] = ws
    return ws


class _InterestExtractFn(torch.autograd.Function):
    """InterestExtract (dien/layers.py:76-133) as one autograd node: the GRU over the positive
    history and the auxiliary loss on its states. Same kernels as _GRUFn + _AuxLossFn; the
    backward sums the two consumers' gradients inside the kernels instead of in separate passes:
    the aux loss's part of dL/dh is added in place to the upstream dL/dh (rs_dien_aux_bwd_acc: no
    zero fill, no add), and its part of dL/dpos is the addend of the GRU's input gradient
    (rs_masked_dx_acc: no add)."""

    @staticmethod
    def forward(ctx, pos, neg, mask_u8, kernel, recurrent_kernel, bias, W1, b1, W2, b2, W3, b3):
        B, T, X = pos.shape
        H = recurrent_kernel.shape[0]
        E = neg.shape[-1]
        dev = pos.device
        vr = _valid_rows(mask_u8)
        xw = _masked_proj(pos.reshape(-1, X), kernel, bias[0], vr).view(B, T, 3 * H)
        out = torch.empty(B, T, H, device=dev)
        saved = torch.empty(B, T, 4 * H, device=dev)
        rk = recurrent_kernel.contiguous()
        st = L.stream_ptr(dev)
        L.call("rs_gru_fwd", L.ptr(xw), L.ptr(rk), L.ptr(bias[1].contiguous()), L.ptr(mask_u8), B, T,
               H, L.ptr(out), L.ptr(saved), st)
        aux = torch.empty(B, device=dev)
        L.call("rs_dien_aux_fwd", L.ptr(out), L.ptr(pos), L.ptr(neg), L.ptr(mask_u8), B, T, H, E,
               L.ptr(W1), L.ptr(b1), L.ptr(W2), L.ptr(b2), L.ptr(W3), L.ptr(b3), L.ptr(aux), st)
        ctx.save_for_backward(pos, neg, kernel, rk, out, saved, mask_u8, *vr, W1, b1, W2, b2, W3, b3)
        return out, aux

    @staticmethod
    def backward(ctx, dhidden, daux):
        (pos, neg, kernel, rk, out, saved, mask_u8, idx, cnt,
         W1, b1, W2, b2, W3, b3) = ctx.saved_tensors
        B, T, X = pos.shape
        H = rk.shape[0]
        E = neg.shape[-1]
        dev = pos.device
        st = L.stream_ptr(dev)
        # dL/dh: the upstream gradient (owned by this node: summed by autograd or handed over by
        # its one consumer), the aux loss's part added in place below
        if dhidden is None:
            dh = torch.zeros(B, T, H, device=dev)
        elif dhidden.is_contiguous():
            dh = dhidden
        else:
            dh = dhidden.contiguous()
        da = torch.zeros(B, device=dev) if daux is None else daux.contiguous()
        dp_aux = torch.empty_like(pos)
        dneg = torch.empty_like(neg)
        In, n1, n2 = H + E, W1.shape[1], W2.shape[1]
        dparams = torch.empty(In * n1 + n1 + n1 * n2 + n2 + n2 + 1, device=dev)
        ws = _aux_workspace(B, T, H, E, dev)
        L.call("rs_dien_aux_bwd_acc", L.ptr(out), L.ptr(pos), L.ptr(neg), L.ptr(mask_u8), B, T, H,
               E, L.ptr(W1), L.ptr(b1), L.ptr(W2), L.ptr(b2), L.ptr(W3), L.ptr(b3), L.ptr(da),
               L.ptr(dh), 1, L.ptr(dp_aux), L.ptr(dneg), L.ptr(dparams), L.ptr(ws), ws.numel(),
               st)
        dxw = torch.empty(B, T, 3 * H, device=dev)
        dinner = torch.empty(B, T, 3 * H, device=dev)
        L.call("rs_gru_bwd", L.ptr(dh), L.ptr(out), L.ptr(saved), L.ptr(rk), L.ptr(mask_u8), B, T,
               H, L.ptr(dxw), L.ptr(dinner), L.RS_DIEN_SKIP_MASKED_ROWS, st)
        dxw2, din2 = dxw.view(-1, 3 * H), dinner.view(-1, 3 * H)
        vr = (idx, cnt)
        m = mask_u8.reshape(-1)
        dpos = torch.empty_like(pos)
        L.call("rs_masked_dx_acc", L.ptr(dxw2), _ld(dxw2), L.ptr(kernel.contiguous()), L.ptr(m),
               L.ptr(idx), L.ptr(cnt), B * T, X, 3 * H, L.ptr(dp_aux), X, L.ptr(dpos), X, st)
        dk, db0 = _masked_wgrad(pos.reshape(-1, X), 0, dxw2, vr)
        drk, db1 = _masked_wgrad(out.view(-1, H), T, din2, vr)
        o = 0
        outs = []
        for shape in (W1.shape, b1.shape, W2.shape, b2.shape, W3.shape, b3.shape):
            n = int(torch.Size(shape).numel())
            outs.append(dparams[o:o + n].view(shape))
            o += n
        return (dpos, dneg, None, dk, drk, torch.stack([db0, db1]), *outs)


def _sigmoid_ce(labels, logits):
    # tf.nn.sigmoid_cross_entropy_with_logits: max(x,0) - x*z + log(1 + exp(-|x|))
    return torch.clamp(logits, min=0) - logits * labels + torch.log1p(torch.exp(-logits.abs()))


class InterestExtract(nn.Module):
    """dien/layers.py:76-133: GRU over the positive history + auxiliary loss on
    (h_t, e_{t+1}) for positive / negative next items, masked mean over 2·Σmask[:,1:]."""

    def __init__(self, gru_units, input_dim, device=None, generator=None):
        super().__init__()
        self.gru = GRU(gru_units, input_dim, device, generator)
        self.auxiliary_net = AuxiliaryNet([80, 40, 1], gru_units + input_dim, device, generator)

    def _fused_aux_ready(self, hidden_state, pos_his):
        layers = list(self.auxiliary_net.layers)
        H, E = hidden_state.shape[-1], pos_his.shape[-1]
        return (hidden_state.is_cuda and (H, E) in ((36, 36), (16, 16))
                and hidden_state.shape[1] >= 2 and len(layers) == 3
                and [l.units for l in layers] == [80, 40, 1]
                and [l.act_code for l in layers] == [2, 2, 0]
                and all(l.kernel is not None and l.bias is not None for l in layers)
                and layers[0].kernel.shape[0] == H + E)

    def compute_auxiliary_loss(self, inputs, training=False, mask=None):
        hidden_state, pos_his, neg_his = inputs
        if self._fused_aux_ready(hidden_state, pos_his):
            l1, l2, l3 = self.auxiliary_net.layers
            m = _mask_u8(mask, hidden_state.shape[:2], hidden_state.device)
            return _AuxLossFn.apply(hidden_state.contiguous(), pos_his.contiguous(),
                                    neg_his.contiguous(), m, l1.kernel, l1.bias, l2.kernel,
                                    l2.bias, l3.kernel, l3.bias)
        h = hidden_state[:, :-1, :]
        m = mask[:, 1:].to(h.dtype)
        both = torch.cat([torch.cat([h, pos_his[:, 1:, :]], -1),
                          torch.cat([h, neg_his[:, 1:, :]], -1)], 0)     # one pass for pos + neg
        logits = self.auxiliary_net(both).squeeze(-1)
        B = h.shape[0]
        pos_loss = _sigmoid_ce(torch.ones_like(logits[:B]), logits[:B]) * m
        neg_loss = _sigmoid_ce(torch.zeros_like(logits[B:]), logits[B:]) * m
        s = torch.cat([pos_loss, neg_loss], -1).sum(-1)
        return s / (m.sum(-1) * 2.0)

    def forward(self, inputs, training=False, mask=None):
        pos_history, neg_history = inputs
        g = self.gru
        if g.kernel is None:
            g.build(pos_history.shape[-1], pos_history.device)
        H, X = g.units, pos_history.shape[-1]
        if (_rows_ready(X, H) and pos_history.is_cuda and neg_history.shape == pos_history.shape
                and pos_history.shape[1] >= 2
                and self._fused_aux_ready(pos_history.new_empty(1, 2, H), pos_history)):
            # the GRU and its aux loss as one node (_InterestExtractFn)
            l1, l2, l3 = self.auxiliary_net.layers
            m = _mask_u8(mask, pos_history.shape[:2], pos_history.device)
            return _InterestExtractFn.apply(pos_history.contiguous(), neg_history.contiguous(), m,
                                            g.kernel, g.recurrent_kernel, g.bias, l1.kernel,
                                            l1.bias, l2.kernel, l2.bias, l3.kernel, l3.bias)
        hidden_state = self.gru(pos_history, mask=mask)
        aux = self.compute_auxiliary_loss((hidden_state, pos_history, neg_history), training, mask)
        return hidden_state, aux
