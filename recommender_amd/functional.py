"""torch.autograd wrappers around the C-ABI kernels (the only callers of recommender_amd._lib).

Embedding gradients never become dense [V, D] tensors: the backward of a lookup hands its
upstream rows (position order) and ids to the owning EmbeddingTable, and the sparse optimizer
(recommender_amd.optim) sorts, segment-sums and applies them in one fused pass.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _lib as L

# compact DLRM row alignment: 479 = 351 + 128 columns → 480 (float4-aligned rows for the
# interaction kernels). The top-MLP first layer's three GEMMs (fwd, dgrad, split-K wgrad)
# measured 866 µs at K = 512 vs 768-804 µs at K = 480-496 (tools/probe_k480.py, 1x MI355X).
COMPACT_ALIGN = 16


def _ids_flat(ids: torch.Tensor) -> torch.Tensor:
    ids = ids.contiguous()
    L.require_device(ids, "ids")
    L.id_dtype_code(ids)
    return ids


def _wait_update(table_module):
    """Order this stream after a deferred sparse update of the table (Embedding.wait_update);
    table views without deferred updates (e.g. a sharded exchange's unique rows) have none."""
    w = getattr(table_module, "wait_update", None)
    if w is not None:
        w()


class _EmbeddingLookup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, handle, table_module, ids, grad_mask=None):
        _wait_update(table_module)
        w = table_module.weight
        L.require_device(w, "embedding table")
        ids = _ids_flat(ids)
        dim = w.shape[1]
        out = torch.empty(*ids.shape, dim, device=w.device, dtype=torch.float32)
        so = table_module.slot_offsets
        n_slots = 1 if so is None else so.numel() - 1
        L.call("rs_embedding_fwd", L.ptr(w), w.shape[0], dim, L.ptr(ids), L.id_dtype_code(ids),
               ids.numel(), L.ptr(so), n_slots, L.ptr(out), L.ptr(table_module.err_flag),
               L.stream_ptr(w.device))
        ctx.table_module = table_module
        ctx.ids = ids
        ctx.grad_mask = grad_mask
        return out

    @staticmethod
    def backward(ctx, grad_out):
        g = grad_out.reshape(-1, grad_out.shape[-1])
        _lookup_backward(ctx.table_module, ctx.ids, g, ctx.grad_mask)
        return None, None, None, None


def _lookup_backward(tm, ids, g, grad_mask):
    """A lookup's upstream rows g [N, dim] (possibly a strided column block) to its table."""
    if tm.fused_optimizer is not None:
        tm.fused_optimizer.apply_async(tm, ids, g.contiguous(), tm.take_presorted(ids))
    elif grad_mask is None:
        tm.accumulate_grad(ids, g)
    else:
        tm.accumulate_grad(ids, g, valid=grad_mask)


class _EmbeddingLookupConcat(torch.autograd.Function):
    """tf.concat([table_a(ids_a), table_b(ids_b)], -1) in one output: each lookup gathers into its
    column block (rs_embedding_fwd_strided), no concat pass; the backward hands each table its
    column block of the upstream gradient as strided rows (the table's take_grad concatenates
    lookups in one copy anyway)."""

    @staticmethod
    def forward(ctx, handle_a, handle_b, ta, tb, ids_a, ids_b, grad_mask=None):
        _wait_update(ta)
        _wait_update(tb)
        ids_a, ids_b = _ids_flat(ids_a), _ids_flat(ids_b)
        if ids_a.shape != ids_b.shape:
            raise ValueError("the two lookups must have the same ids shape")
        wa, wb = ta.weight, tb.weight
        L.require_device(wa, "embedding table")
        L.require_device(wb, "embedding table")
        da, db = wa.shape[1], wb.shape[1]
        out = torch.empty(*ids_a.shape, da + db, device=wa.device, dtype=torch.float32)
        st = L.stream_ptr(wa.device)
        for t, ids, col, d in ((ta, ids_a, 0, da), (tb, ids_b, da, db)):
            so = t.slot_offsets
            n_slots = 1 if so is None else so.numel() - 1
            L.call("rs_embedding_fwd_strided", L.ptr(t.weight), t.weight.shape[0], d, L.ptr(ids),
                   L.id_dtype_code(ids), ids.numel(), L.ptr(so), n_slots,
                   L.ptr(out.narrow(-1, col, d)), da + db, L.ptr(t.err_flag), st)
        ctx.tables = (ta, tb)
        ctx.ids = (ids_a, ids_b)
        ctx.grad_mask = grad_mask
        ctx.da = da
        return out

    @staticmethod
    def backward(ctx, grad_out):
        g = grad_out.reshape(-1, grad_out.shape[-1])
        da = ctx.da
        (ta, tb), (ia, ib) = ctx.tables, ctx.ids
        _lookup_backward(ta, ia, g[:, :da], ctx.grad_mask)
        _lookup_backward(tb, ib, g[:, da:], ctx.grad_mask)
        return None, None, None, None, None, None, None


def embedding_lookup_concat(table_a, ids_a, table_b, ids_b, grad_mask=None) -> torch.Tensor:
    """[table_a(ids_a) ‖ table_b(ids_b)] along the last axis (grad_mask: embedding_lookup)."""
    return _EmbeddingLookupConcat.apply(table_a.grad_handle, table_b.grad_handle, table_a,
                                        table_b, ids_a, ids_b, grad_mask)


def embedding_lookup(table_module, ids: torch.Tensor, grad_mask=None) -> torch.Tensor:
    """grad_mask (bool / uint8, ids' shape, optional): the caller's statement that the lookup's
    masked positions receive exactly zero gradient (the model skips them); the densified table
    gradient then leaves them out instead of summing their zero rows (Embedding.take_grad)."""
    return _EmbeddingLookup.apply(table_module.grad_handle, table_module, ids, grad_mask)


class _DotInteraction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, self_interaction, skip_gather):
        L.require_device(x, "x")
        x = x.contiguous().float()
        B, F, D = x.shape
        if skip_gather:
            w = F * F
        else:
            w = F * (F + 1) // 2 if self_interaction else F * (F - 1) // 2
        out = torch.empty(B, w, device=x.device, dtype=torch.float32)
        L.call("rs_dot_interaction_fwd", L.ptr(x), B, F, D, int(self_interaction),
               int(skip_gather), L.ptr(out), w, L.stream_ptr(x.device))
        ctx.save_for_backward(x)
        ctx.flags = (int(self_interaction), int(skip_gather), w)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        (x,) = ctx.saved_tensors
        si, sg, w = ctx.flags
        B, F, D = x.shape
        g = grad_out.contiguous()
        gx = torch.empty_like(x)
        L.call("rs_dot_interaction_bwd", L.ptr(x), L.ptr(g), B, F, D, si, sg, w, L.ptr(gx),
               L.stream_ptr(x.device))
        return gx, None, None


def dot_interaction(x, self_interaction: bool, skip_gather: bool):
    return _DotInteraction.apply(x, self_interaction, skip_gather)


class _DLRMInteraction(torch.autograd.Function):
    """Fused gather + DotInteraction(False, True) + concat (ctr/model.py:49-55)."""

    @staticmethod
    def forward(ctx, handle, dense, table_module, ids, compact):
        _wait_update(table_module)
        w = table_module.weight
        L.require_device(w, "embedding table")
        ids = _ids_flat(ids)
        dense = dense.contiguous()
        B, S = ids.shape
        D = w.shape[1]
        F = S + 1
        if dense.shape != (B, D):
            raise ValueError(f"bottom-MLP output must be [B, {D}], got {tuple(dense.shape)}")
        width = (F * (F - 1) // 2 if compact else F * F) + D
        if compact:  # pad to a multiple of COMPACT_ALIGN columns (top-MLP GEMM tiling)
            width = (width + COMPACT_ALIGN - 1) // COMPACT_ALIGN * COMPACT_ALIGN
        out = torch.empty(B, width, device=w.device, dtype=torch.float32)
        L.call("rs_dlrm_interaction_fwd", L.ptr(w), w.shape[0], D, L.ptr(ids),
               L.id_dtype_code(ids), S, L.ptr(table_module.slot_offsets), L.ptr(dense), B,
               int(compact), L.ptr(out), width, L.ptr(table_module.err_flag), L.stream_ptr(w.device))
        ctx.table_module = table_module
        ctx.ids = ids
        ctx.compact = int(compact)
        ctx.save_for_backward(dense)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        (dense,) = ctx.saved_tensors
        tm = ctx.table_module
        w = tm.weight
        ids = ctx.ids
        B, S = ids.shape
        D = w.shape[1]
        g = grad_out.contiguous()
        grad_emb = torch.empty(B * S, D, device=w.device, dtype=torch.float32)
        grad_dense = torch.empty(B, D, device=w.device, dtype=torch.float32)
        L.call("rs_dlrm_interaction_bwd", L.ptr(w), w.shape[0], D, L.ptr(ids),
               L.id_dtype_code(ids), S, L.ptr(tm.slot_offsets), L.ptr(dense), B, ctx.compact,
               L.ptr(g), g.shape[1], L.ptr(grad_emb), L.ptr(grad_dense), L.stream_ptr(w.device))
        if tm.fused_optimizer is not None:
            tm.fused_optimizer.apply_async(tm, ids, grad_emb, tm.take_presorted(ids))
        else:
            tm.accumulate_grad(ids, grad_emb)
        return None, grad_dense, None, None, None


def dlrm_interaction(table_module, ids, dense, compact: bool = False):
    """[Z, dense] with Z the strict-upper X·Xᵀ of X = [emb(ids), dense]: F*F wide with zeros
    (reference layout) or, compact=True, the F(F-1)/2 kept values only (row zero-padded to a
    multiple of COMPACT_ALIGN columns)."""
    return _DLRMInteraction.apply(table_module.grad_handle, dense, table_module, ids, compact)


class _DLRMTopFn(torch.autograd.Function):
    """DLRM's fused lookup + interaction (compact row) feeding the top MLP as one linear chain
    (ctr/model.py:49-57 with the ctr MLP's linear hidden layers, ctr/layers.py:8). Forward:
    rs_dlrm_interaction_fwd, then the top MLP as one chain (layer by layer, bit-identical to the
    unfused path, or composed into its single affine map, nn.chain_forward). Backward: rs_chain_reduce over the interaction row gives G = σ'(y)·dy [B], A = Zᵀ·G
    and Σ G in one pass; every top-MLP gradient follows from them (nn.chain_param_grads); the
    upstream gradient of the interaction is then the rank-one G ⊗ Q_0 (Q_0 = K_1·K_2·K_3), which
    rs_dlrm_interaction_bwd_rank1 consumes without materialising the [B, width] rows.

    Production path (composed head, D = 128): rs_dlrm_interaction_fwd_head_dx forms each
    example's UNIT interaction gradient (M + Mᵀ)·X[b] (M = the strict-upper pairs of Q_0) while
    its rows are in registers, so the backward only scales: the embedding rows' gradient is
    G[b] · unit rows, handed to the fused sparse optimizer as (unit rows, row_scale = G) and
    multiplied in its walk; the bottom-MLP gradient is G[b] · unit bottom row. No re-gather."""

    @staticmethod
    def forward(ctx, handle, dense, table_module, ids, layers, rows, composed=False):
        from .nn import chain_forward, vec_chain_compose, vec_chain_ready

        dense = dense.contiguous()
        w = table_module.weight
        D = w.shape[1]
        width = rows.numel() if rows is not None else 0
        if (composed and D == 128 and ids.shape[-1] + 1 <= 32 and vec_chain_ready(layers, width)
                and w.data_ptr() % 16 == 0 and dense.data_ptr() % 16 == 0):
            # the composed top MLP fused into the interaction kernel: y = act(row·q + c) per
            # example as the row is written (rs_dlrm_interaction_fwd_head)
            q, c = vec_chain_compose(layers, rows, width)
            _wait_update(table_module)
            L.require_device(w, "embedding table")
            ids = _ids_flat(ids)
            B, S = ids.shape
            F = S + 1
            nz = F * (F - 1) // 2 + D
            if width != (nz + COMPACT_ALIGN - 1) // COMPACT_ALIGN * COMPACT_ALIGN:
                raise ValueError(f"compact rows ({width}) do not match the interaction row")
            if dense.shape != (B, D):
                raise ValueError(f"bottom-MLP output must be [B, {D}], got {tuple(dense.shape)}")
            z = torch.empty(B, width, device=w.device, dtype=torch.float32)
            y = torch.empty(B, 1, device=w.device, dtype=torch.float32)
            # the unit interaction gradient of every example, formed while its rows are in
            # registers (rs_dlrm_interaction_fwd_head_dx): the backward scales it by G[b]
            dxu_emb = torch.empty(B * S, D, device=w.device, dtype=torch.float32)
            dxu_dense = torch.empty(B, D, device=w.device, dtype=torch.float32)
            L.call("rs_dlrm_interaction_fwd_head_dx", L.ptr(w), w.shape[0], D, L.ptr(ids),
                   L.id_dtype_code(ids), S, L.ptr(table_module.slot_offsets), L.ptr(dense), B,
                   L.ptr(z), width, L.ptr(q), L.ptr(c), layers[-1].act_code, L.ptr(y),
                   L.ptr(dxu_emb), L.ptr(dxu_dense), L.ptr(table_module.err_flag),
                   L.stream_ptr(w.device))
            ctx.table_module, ctx.ids, ctx.compact = table_module, ids, 1
            ctx.dxu = (dxu_emb, dxu_dense)
            ks = [l.kernel for l in layers]  # the backward (_chain3_vec_grads) reads rows itself
        else:
            z = _DLRMInteraction.forward(ctx, handle, dense, table_module, ids, True)
            y, ks = chain_forward(z, layers, rows, composed)
            ctx.dxu = None
        ctx.layers, ctx.rows = layers, rows
        ctx.save_for_backward(dense, z, y, *ks)
        return y

    @staticmethod
    def backward(ctx, dy):
        from .nn import chain_param_grads, chain_reduce

        dense, z, y, *ks = ctx.saved_tensors
        layers, rows = ctx.layers, ctx.rows
        G, A, s = chain_reduce(z, dy.contiguous(), y, layers[-1].act_code, need_g=True)
        Q = chain_param_grads(layers, rows, ks, A, s)
        tm = ctx.table_module
        w = tm.weight
        ids = ctx.ids
        B, S = ids.shape
        D = w.shape[1]
        if ctx.dxu is not None:
            # rank-one upstream gradient G ⊗ q: every gradient row is G[b] times the unit one
            dxu_emb, dxu_dense = ctx.dxu
            ctx.dxu = None
            grad_dense = G * dxu_dense
            if getattr(tm, "fused_optimizer", None) is not None:
                tm.fused_optimizer.apply_async(tm, ids, dxu_emb, tm.take_presorted(ids),
                                               row_scale=G.reshape(-1))
            else:
                tm.accumulate_grad(ids, (G.reshape(B, 1, 1) * dxu_emb.view(B, S, D)).view(B * S, D))
            return None, grad_dense, None, None, None, None, None
        grad_emb = torch.empty(B * S, D, device=w.device, dtype=torch.float32)
        grad_dense = torch.empty(B, D, device=w.device, dtype=torch.float32)
        p = Q[:, 0].contiguous()
        if all(t.data_ptr() % 16 == 0 for t in (w, dense, grad_emb, grad_dense)):
            L.call("rs_dlrm_interaction_bwd_rank1", L.ptr(w), w.shape[0], D, L.ptr(ids),
                   L.id_dtype_code(ids), S, L.ptr(tm.slot_offsets), L.ptr(dense), B, L.ptr(G),
                   L.ptr(p), p.numel(), L.ptr(grad_emb), L.ptr(grad_dense), L.stream_ptr(w.device))
        else:  # unaligned buffers: the same rows, materialised
            g = (G * p[None, :]).contiguous()
            L.call("rs_dlrm_interaction_bwd", L.ptr(w), w.shape[0], D, L.ptr(ids),
                   L.id_dtype_code(ids), S, L.ptr(tm.slot_offsets), L.ptr(dense), B, 1, L.ptr(g),
                   g.shape[1], L.ptr(grad_emb), L.ptr(grad_dense), L.stream_ptr(w.device))
        if getattr(tm, "fused_optimizer", None) is not None:
            tm.fused_optimizer.apply_async(tm, ids, grad_emb, tm.take_presorted(ids))
        else:
            tm.accumulate_grad(ids, grad_emb)
        return None, grad_dense, None, None, None, None, None


def dlrm_top(table_module, ids, dense, layers, rows, composed=False):
    """sigmoid-head top MLP over the compact DLRM interaction row, fused (see _DLRMTopFn)."""
    return _DLRMTopFn.apply(table_module.grad_handle, dense, table_module, ids, list(layers), rows,
                            composed)


class _FM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, emb):
        L.require_device(emb, "emb")
        emb = emb.contiguous().float()
        B, F, D = emb.shape
        out = torch.empty(B, device=emb.device, dtype=torch.float32)
        L.call("rs_fm_fwd", L.ptr(emb), B, F, D, L.ptr(out), L.stream_ptr(emb.device))
        ctx.save_for_backward(emb)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        (emb,) = ctx.saved_tensors
        B, F, D = emb.shape
        g = grad_out.contiguous()
        ge = torch.empty_like(emb)
        L.call("rs_fm_bwd", L.ptr(emb), L.ptr(g), B, F, D, L.ptr(ge), L.stream_ptr(emb.device))
        return ge


def fm_interaction(emb):
    """DeepFM second-order term 0.5*Σ_d((Σ_f e)^2 - Σ_f e^2) (ctr/model.py:21-23)."""
    return _FM.apply(emb)


_RED = {"none": 0, "sum": 1, "mean": 2}


class _BCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p, y, reduction, eps):
        L.require_device(p, "y_pred")
        p = p.contiguous().float()
        y = y.contiguous().float().reshape(p.shape)
        n = p.numel()
        red = _RED[reduction]
        out = torch.empty(p.shape if red == 0 else (), device=p.device, dtype=torch.float32)
        ws = torch.empty(max(1, L.lib().rs_bce_workspace_size(n) // 4), device=p.device)
        L.call("rs_bce_fwd", L.ptr(p), L.ptr(y), n, eps, red, L.ptr(out), L.ptr(ws),
               ws.numel() * 4, L.stream_ptr(p.device))
        ctx.save_for_backward(p, y)
        ctx.red, ctx.eps = red, eps
        return out

    @staticmethod
    def backward(ctx, g):
        p, y = ctx.saved_tensors
        g = g.contiguous().float()
        dp = torch.empty_like(p)
        L.call("rs_bce_bwd", L.ptr(p), L.ptr(y), p.numel(), ctx.eps, ctx.red, L.ptr(g), L.ptr(dp),
               L.stream_ptr(p.device))
        return dp, None, None, None


def binary_crossentropy(y_true, y_pred, reduction: str = "mean", epsilon: float = 1e-7):
    """Fused keras binary_crossentropy on probabilities (one kernel forward, one backward)."""
    return _BCE.apply(y_pred, y_true, reduction, epsilon)


TRAIN_SUMS_ATOP = 512  # rs_dlrm_train_step_fwd_unit's sums layout (include/recsys_hip.h)
# the train kernel waiting for the presort's completion (below): off for the chunked kernel
# (interleaved A/B, 3 x 100 steps: 0.695-0.699 vs 0.700-0.704 ms/step, p90 0.698-0.700 vs
# 0.704-0.707); RS_TRAIN_WAITS_SORT=1 restores the wait
_TRAIN_WAITS_SORT = os.environ.get("RS_TRAIN_WAITS_SORT", "0") != "0"


def dlrm_fused_train_forward(model, cat_features, int_features, label, reduction="mean",
                             epsilon=1e-7, sgd_lr=None, comm=None):
    """The production DLRM train step's forward + loss + backward reductions in one kernel
    (rs_dlrm_train_step_fwd_unit): the reference's DLRM.call (ctr/model.py:45-57) under the mean
    Keras BCE (ctr/train.py:85) with the SGD path's gradients (ctr/train.py:77-79).

    Runs: the side-stream radix sort of the ids; the bottom MLP as its composed affine map
    (ctr/layers.py:8: hidden layers linear); the fused kernel (gather, MFMA interaction, composed
    top MLP head, BCE, G = σ'·dL/dy, the table gradient rows, and the deterministic batch sums
    A_top, s_top, loss, A_bot, s_bot); every top / bottom MLP parameter gradient from those sums
    (nn.chain_param_grads: the factored backward's weight-sized products), accumulated into
    .grad; the segmented-sum sparse update queued on the fused optimizer's side stream.
    sgd_lr (float): also apply plain SGD to every MLP parameter and compose the next step's
    maps, all in rs_dlrm_dense_tail (bit-identical to chain_param_grads + torch.optim.SGD +
    the next forward's compositions, in six launches instead of sixteen); the caller then skips
    its dense optimizer step.
    comm (a recommender_amd.sharded.Comm with a row-sharded ShardedSlabEmbedding): the same step
    on this rank's share of a global batch of B·W examples — the exchange fetches the batch's
    unique rows from their owners (side stream, beside the bottom MLP), the kernel reads them by
    the inverse index with dL/dl_b = 1/(B·W), one all-reduce of the batch sums (≈9 KB) makes every
    rank's dense tail the global step, and the gradient rows go back to the owners' apply.
    Returns (prediction y [B] (detached), loss scalar tensor (no autograd graph))."""
    from .nn import _composed_forward_hip, chain_param_grads, cached_vec_chain_compose

    emb = model.embedding_layer
    S, n_in = model.num_cat_fea, model.num_int_fea
    ids = _ids_flat(cat_features.reshape(-1, S))
    sharded = hasattr(emb, "exchange_begin")
    world = comm.world if (sharded and comm is not None) else 1
    if sharded:
        # sort / unique / split sizes beside the bottom MLP (or queued a step ahead: prefetch)
        pending = emb.take_prefetched(ids)
        if pending is None:
            pending = emb.exchange_begin(ids)
    else:
        emb.presort(ids)  # the sort runs beside the bottom MLP and the fused kernel
    x = int_features.reshape(-1, n_in).float().contiguous()
    lab = label.reshape(-1).float().contiguous()
    B = ids.shape[0]
    bl = list(model.bottom_mlp.mlp)
    tl = list(model.top_mlp.mlp)
    rows = model.compact_rows
    width = rows.numel()
    with torch.no_grad():
        got = _composed_forward_hip(x, bl, None)
        if got is None:
            raise RuntimeError("fused DLRM step: the bottom MLP is not a narrow composed chain")
        h, bks = got
        q, c = cached_vec_chain_compose(tl, rows, width)
    if sharded:
        view, inv = emb.exchange_finish(pending)  # this step's unique rows + inverse index
        w, kid, offs, n_rows = view.weight, inv.reshape(-1, S), None, view.input_dim
        D = emb.output_dim
        dev = w.device
    else:
        w = emb.weight
        D = w.shape[1]
        dev = w.device
        _wait_update(emb)
        # the fused kernel is one round of resident blocks: launched while the sort stream's last
        # scatter still holds CU slots, some of dlrm_train_pipe's blocks were placed a round late
        # (measured: 0.42 -> 0.62 ms whenever the two overlapped), so that kernel waits for the
        # sort; the chunked kernel measured better without the wait (_TRAIN_WAITS_SORT above).
        ahead = emb._presorted[1] if getattr(emb, "_presorted", None) else None
        ready = getattr(ahead, "ready", None)
        if ready is not None and _TRAIN_WAITS_SORT:
            L.stream_wait_event(torch.cuda.current_stream(dev), ready)
        kid, offs, n_rows = ids, emb.slot_offsets, w.shape[0]
    y = torch.empty(B, device=dev, dtype=torch.float32)
    grad = torch.empty(B * S, D, device=dev, dtype=torch.float32)
    M = TRAIN_SUMS_ATOP + 2 + n_in * D + D
    sums = torch.empty(M, device=dev, dtype=torch.float32)
    ws = _train_ws(B, dev)
    n_global = B * world
    scale = 1.0 / n_global if reduction == "mean" else 1.0
    g_rows = torch.empty(B, device=dev, dtype=torch.float32)
    early = _APPLY_EARLY and not sharded
    if early:
        # the kernel alone, then the sparse update ordered after it (the rows, G and y are final
        # there), then the batch-sum fold on this stream beside the update: the update no longer
        # waits for the fold's two launches (round 6; bit-identical to the one-call form)
        L.call("rs_dlrm_train_step_fwd_unit_nofold", L.ptr(w), n_rows, D, L.ptr(kid),
               L.id_dtype_code(kid), S, L.ptr(offs), L.ptr(h), L.ptr(x), n_in, L.ptr(lab), B,
               L.ptr(q), L.ptr(c), float(epsilon), scale, L.ptr(y), L.ptr(grad), L.ptr(g_rows),
               L.ptr(ws), ws.numel(), L.ptr(emb.err_flag), L.stream_ptr(dev))
        emb.fused_optimizer.apply_async(emb, ids, grad, emb.take_presorted(ids), row_scale=g_rows)
        L.call("rs_dlrm_train_fold", L.ptr(ws), ws.numel(), B, D, L.id_dtype_code(kid),
               L.ptr(sums), L.stream_ptr(dev))
    else:
        L.call("rs_dlrm_train_step_fwd_unit", L.ptr(w), n_rows, D, L.ptr(kid),
               L.id_dtype_code(kid), S, L.ptr(offs), L.ptr(h), L.ptr(x), n_in, L.ptr(lab), B,
               L.ptr(q), L.ptr(c), float(epsilon), scale, L.ptr(y), L.ptr(grad), L.ptr(g_rows),
               L.ptr(sums), L.ptr(ws), ws.numel(), L.ptr(emb.err_flag), L.stream_ptr(dev))
    if not sharded and emb._prefetch_queue:
        emb.flush_prefetch()  # a later batch's sort, beside this step's update and dense tail
    if sharded and comm is not None and comm.collective:
        # the dense half of the global step: every MLP gradient is a linear function of these
        # batch sums, so one all-reduce of ≈9 KB replaces the all-reduce of ≈3 MB of gradients
        comm.all_reduce_(sums)
    a = TRAIN_SUMS_ATOP
    A_top, s_top = sums[:a].view(a, 1)[:width], sums[a:a + 1]
    loss_sum = sums[a + 1]
    A_bot = sums[a + 2:a + 2 + n_in * D].view(n_in, D)
    s_bot = sums[a + 2 + n_in * D:]
    if sharded:
        # the gradient rows (already of the global mean loss) go to their owners' apply
        emb.backward_exchange(grad, global_grads=True, row_scale=g_rows)
        if sgd_lr is not None:
            _dense_tail_sgd(tl, rows, bl, A_top, s_top, sums[a + 2:].view(n_in + 1, D), sgd_lr)
        else:
            chain_param_grads(tl, rows, [l.kernel for l in tl], A_top, s_top)
            chain_param_grads(bl, None, bks, A_bot, s_bot, need_q0=False)
        loss = loss_sum / n_global if reduction == "mean" else loss_sum
        return y, loss
    # the sparse update (side stream) is queued right after the kernel. With the presort on its
    # own stream this measured 0.841 vs 0.862 ms/step for queueing it after the top chain's
    # gradients (which was the better order while the presort queued behind the update on the
    # side stream: 0.907 vs 0.96); RS_APPLY_EARLY=0 restores it
    if sgd_lr is not None:
        if not early:
            emb.fused_optimizer.apply_async(emb, ids, grad, emb.take_presorted(ids), row_scale=g_rows)
        _dense_tail_sgd(tl, rows, bl, A_top, s_top, sums[a + 2:].view(n_in + 1, D), sgd_lr)
    else:
        chain_param_grads(tl, rows, [l.kernel for l in tl], A_top, s_top)
        if not early:
            emb.fused_optimizer.apply_async(emb, ids, grad, emb.take_presorted(ids), row_scale=g_rows)
        chain_param_grads(bl, None, bks, A_bot, s_bot, need_q0=False)
    loss = loss_sum / B if reduction == "mean" else loss_sum
    return y, loss


def dense_tail_ready(model, opt_dense) -> bool:
    """rs_dlrm_dense_tail applies: plain SGD (no momentum / dampening / weight decay / nesterov /
    maximize, one group) over exactly the DLRM's twelve MLP parameters, bottom chain
    [n0 < 16 -> n1 -> n2 -> n3] and top chain [n0 -> n1 -> n2 -> 1], all with biases."""
    if not isinstance(opt_dense, torch.optim.SGD) or len(opt_dense.param_groups) != 1:
        return False
    g = opt_dense.param_groups[0]
    if (g.get("momentum", 0) != 0 or g.get("weight_decay", 0) != 0 or g.get("nesterov")
            or g.get("maximize") or g.get("dampening", 0) != 0 or callable(g["lr"])):
        return False
    bl, tl = list(model.bottom_mlp.mlp), list(model.top_mlp.mlp)
    if len(bl) != 3 or len(tl) != 3 or any(l.bias is None for l in bl + tl):
        return False
    params = [t for l in tl + bl for t in (l.kernel, l.bias)]
    if {id(p) for p in g["params"]} != {id(p) for p in params} or len(g["params"]) != 12:
        return False
    n0 = bl[0].kernel.shape[0]
    return (n0 < 16 and tl[2].kernel.shape[1] == 1
            and all(p.is_contiguous() and p.dtype == torch.float32 for p in params)
            and all(l.kernel.shape[1] % 4 == 0 for l in bl)
            and all((n0 + 1) * l.kernel.shape[0] <= 16896 for l in bl))


def _dense_tail_sgd(tl, rows, bl, A_top, s_top, P_bot, lr):
    """rs_dlrm_dense_tail: gradients into fresh .grad tensors (as chain_param_grads leaves them),
    SGD on the twelve parameters, next step's compositions into the compose cache."""
    from .nn import _rows_i32, narrow_chain_compose, store_composed

    dev = A_top.device
    comp2 = narrow_chain_compose(bl)[0]  # current [K1·K2; c2] (the forward's, cached)
    n0, n1 = tl[0].kernel.shape[0], tl[0].kernel.shape[1]
    n2 = tl[1].kernel.shape[1]
    width = A_top.shape[0]
    r, inv = _rows_i32(rows, n0)
    m, b1 = bl[0].kernel.shape
    b2, b3 = bl[1].kernel.shape[1], bl[2].kernel.shape[1]
    tdk = [torch.empty_like(l.kernel) for l in tl]
    tdb = [torch.empty_like(l.bias) for l in tl]
    P2 = torch.empty(m + 1, b2, device=dev)
    P1 = torch.empty(m + 1, b1, device=dev)
    dk2 = torch.empty(b1, b2, device=dev)
    dk3 = torch.empty(b2, b3, device=dev)
    comp2n = torch.empty(m + 1, b2, device=dev)
    comp3n = torch.empty(m + 1, b3, device=dev)
    q = torch.empty(width, device=dev)
    c = torch.empty(1, device=dev)
    ws = _tail_ws(width, n1, n2, dev)
    a = L.DlrmTailArgs()
    for i in range(3):
        a.top_k[i], a.top_b[i] = tl[i].kernel.data_ptr(), tl[i].bias.data_ptr()
        a.top_dk[i], a.top_db[i] = tdk[i].data_ptr(), tdb[i].data_ptr()
        a.bot_k[i], a.bot_b[i] = bl[i].kernel.data_ptr(), bl[i].bias.data_ptr()
    a.top_rows = None if r is None else r.data_ptr()
    a.top_inv = None if inv is None else inv.data_ptr()
    a.top_n_full0, a.top_n0, a.top_n1, a.top_n2 = n0, width, n1, n2
    a.top_A, a.top_s = A_top.data_ptr(), s_top.data_ptr()
    a.top_q, a.top_c = q.data_ptr(), c.data_ptr()
    a.bot_n0, a.bot_n1, a.bot_n2, a.bot_n3 = m, b1, b2, b3
    a.bot_P, a.bot_comp2 = P_bot.data_ptr(), comp2.data_ptr()
    a.bot_dk2, a.bot_dk3, a.bot_P2, a.bot_P1 = dk2.data_ptr(), dk3.data_ptr(), P2.data_ptr(), P1.data_ptr()
    a.bot_comp2_next, a.bot_comp3_next = comp2n.data_ptr(), comp3n.data_ptr()
    a.lr = float(lr)
    L.call("rs_dlrm_dense_tail", C.byref(a), L.ptr(ws), ws.numel() * 4, L.stream_ptr(dev))
    grads = list(zip(tdk, tdb)) + [(P1[:m], P1[m]), (dk2, P2[m]), (dk3, P_bot[m])]
    for layer, (dk, db) in zip(tl + bl, grads):
        layer.kernel.grad, layer.bias.grad = dk, db
    # the kernels moved the parameters in place: bump their versions (stale caches of other
    # consumers miss), then file the next step's compositions under the new versions
    for l in tl + bl:
        torch.autograd.graph.increment_version(l.kernel)
        torch.autograd.graph.increment_version(l.bias)
    store_composed(bl, [comp2n, comp3n], tl, rows, width, (q, c))


_tail_ws_cache: dict = {}


def _tail_ws(n0, n1, n2, dev):
    n = (L.lib().rs_dlrm_dense_tail_workspace_size(n0, n1, n2) + 3) // 4
    t = _tail_ws_cache.get(dev)
    if t is None or t.numel() < n:
        t = torch.empty(n, device=dev)
        _tail_ws_cache[dev] = t
    return t


_train_ws_cache: dict = {}
_APPLY_EARLY = os.environ.get("RS_APPLY_EARLY", "1") == "1"



def _train_ws(B, dev):
    nb = L.lib().rs_dlrm_train_workspace_size(B)
    t = _train_ws_cache.get(dev)
    if t is None or t.numel() < nb:
        t = torch.empty(nb, dtype=torch.uint8, device=dev)
        _train_ws_cache[dev] = t
    return t
