"""Checker for one production DLRM SGD step against oracle/ctr.py: the touched table rows AND
the dense half (every MLP parameter gradient and update).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py; parity unpinned): called by
tests/test_northstar_gpu.py (full north-star size, cfg2) and __graft_entry__.smoke() (small
size). It drives the product path (recommender_amd TrainStep on cuda) and checks it; nothing in
the product imports this module.

The slab rows the batch references are gathered before the step and the ids are remapped onto
them monotonically, so the oracle's sort order, tiles and segmented-sum order are exactly those
of the full slab (reference semantics: ctr/model.py:45-57, ctr/train.py:77-79 SGD path).
The oracle carries its OWN MLP state across steps (pass the same `state` dict to every call):
an error in one step's MLP update then shows up in the next step's logits and gradients instead
of being absorbed by re-reading the GPU's weights. The table rows are read from the GPU before
each step (they are checked bit-exact against the oracle apply, so the two tables agree).
Checks (tolerances are the ones stated here):
  * loss within 1e-5 relative;
  * per-example logits: the pre-sigmoid value recovered from p within 1e-5 of its own value
    plus 1e-6 of its float64 magnitude bound (|row|·|K1|·|K2|·|K3| with |biases|: every fp32
    rounding of either MLP evaluation order is relative to it), plus the fp32 resolution of p;
  * grad rows [B*S, D] (position order) within 1e-5 of the oracle's, relative to each element's
    float64 magnitude bound |dZ + dZᵀ|·|X|;
  * every top / bottom MLP kernel and bias gradient within 1e-5 of its float64 magnitude bound
    (oracle.ctr.chain_grad_bounds: Σ_b |h_b|·|G_b| carried through the chain), plus the bound
    of the gradient error the logit tolerance above admits (|dG/dz| <= 1/4 per example, through
    the same chain) and, for the top chain, 1e-6 of Σ_b bound(h_b)·|G_b| over the bottom-output
    inputs (the composed bottom map's rounding: dense_half_tolerances), for the bottom
    chain, of its upstream gradient's tolerance and of the ReLU outputs whose pre-activation
    lies within rounding of 0, and with world > 1 the fp32 all-reduce of the ranks' sums;
  * every MLP parameter after the step equal to fp32(before - lr·grad) within 1 ulp (the SGD
    apply) — so it also lies within lr·(gradient tolerance) + 1 ulp of the oracle's update;
  * sorted rows / positions bit-exact;
  * touched table rows BIT-EXACT against the oracle's segmented sum + SGD fed with the kernel's
    own grad rows, and within 1e-4 of each row's |Δ| (+2 ulp of w) of the all-oracle update;
    at least a quarter of the touched elements must actually change (a vacuous update fails);
  * sampled untouched rows (including the slab's last rows) unchanged.
"""
from __future__ import annotations

import numpy as np

from .ctr import DLRMState, chain_grad_bounds, dlrm_sgd_step, magnitude_chain
from .embedding import global_rows, segment_sum_tiled


def _layers(mlp):
    return [(l.kernel.detach().cpu().numpy().copy(), l.bias.detach().cpu().numpy().copy())
            for l in mlp.mlp]


def _grads(mlp):
    out = []
    for l in mlp.mlp:
        assert l.kernel.grad is not None and l.bias.grad is not None, "an MLP gradient is missing"
        out.append((l.kernel.grad.detach().cpu().numpy().copy(),
                    l.bias.grad.detach().cpu().numpy().copy()))
    return out


def _check_chain(name, got, ref, tol):
    """got / ref: [(dk, db)]; tol: [(kernel tol, bias tol)] (float64, same shapes)."""
    worst = 0.0
    for i, ((gk, gb), (rk, rb), (tk, tb)) in enumerate(zip(got, ref, tol)):
        for what, g, r, t in (("kernel", gk, rk, tk), ("bias", gb, rb, tb)):
            err = np.abs(g.astype(np.float64) - np.asarray(r, np.float64))
            t = np.asarray(t, np.float64).reshape(err.shape) + 1e-38
            ratio = err / t
            if (ratio > 1).any():
                j = int(np.argmax(ratio))
                raise AssertionError(
                    f"{name} layer {i} {what} gradient off at flat index {j}: gpu "
                    f"{g.reshape(-1)[j]!r} oracle {np.asarray(r).reshape(-1)[j]!r} "
                    f"(err/tol {ratio.max():.3g})")
            worst = max(worst, float(ratio.max()))
    return worst


def _check_sgd(name, before, after, grads, lr):
    """after == fp32(before - lr·g) within 1 ulp (fmaf or mul-then-sub rounding)."""
    lr = np.float64(np.float32(lr))
    for i, ((k0, b0), (k1, b1), (gk, gb)) in enumerate(zip(before, after, grads)):
        for what, p0, p1, g in (("kernel", k0, k1, gk), ("bias", b0, b1, gb)):
            exact = p0.astype(np.float64) - lr * g.astype(np.float64)
            err = np.abs(p1.astype(np.float64) - exact)
            ok = err <= np.spacing(np.abs(p1).astype(np.float32)).astype(np.float64)
            assert ok.all(), (f"{name} layer {i} {what}: SGD update is not before - lr*grad "
                              f"({int((~ok).sum())} elements)")


def dense_half_tolerances(det, n_examples, mean=True, world=1):
    """Per-element tolerances of the top / bottom chains' parameter gradients (see the module
    docstring). Returns (top [(tk, tb)], bottom [(tk, tb)]).

    Top chain. Every top gradient is linear in A_top = Σ_b z_b·G_b (z_b the top input: the pair
    values and the bottom output). Against the oracle's float64 sum of ITS fp32 z_b, G_b:
      * G_b differs by 1e-5·|G_b| plus what the logit tolerance admits (|dG/dz| <= 1/4);
      * z_b differs by the roundings of two fp32 evaluations. For the pair values (dot products
        of the same table rows: split-bf16 MFMA vs numpy) those roundings change sign from
        example to example and stay inside the 1e-5·|z_b|·|G_b| term. The bottom output is
        different: the kernel evaluates the bottom MLP as ONE composed affine map
        (x·(K1·K2·K3) + c, ctr/layers.py:8 hidden layers linear) and the oracle layer by layer,
        so each output column carries the composed matrix's own rounding, the SAME for every
        example — over non-negative dense features it adds up across the batch instead of
        cancelling, and it is relative to the column's magnitude bound (|x|·|K1|·|K2|·|K3| +
        |biases|, det["top_in_bound"]'s last D columns), not to |h_b|. Round 5 left this term
        out, and a world-4 case (4 096 examples) exceeded its bound 2.45× on exactly such a row
        (top kernel 0, input 825 = bottom output 96: 3.5065e-08 vs 3.5104e-08). It enters at
        1e-6 of the bound, as in the logit check, on the kernels only;
      * the sum's own roundings (the kernel's per-wave, per-block and two-level folds) are
        within 1e-5 of Σ|z_b|·|G_b| at these depths (≤ a few hundred additions, random-walk);
      * world > 1: the fp32 all-reduce of the W per-rank partial sums adds at most (W-1)·u of
        Σ_r |partial_r| <= Σ_b |z_b|·|G_b| (u = 2^-24), stated as its own term below; the
        per-rank partials themselves are bit-identical to the one-GPU kernel on the rank's
        examples (tests/test_sharded_gpu.py checks that), so sharding adds nothing else.
    So the tolerance is 1e-5 of Σ|z_b|·|G_b| carried through the chain (the G and summation
    terms), plus 1e-6 of Σ bound(h_b)·|G_b| over the bottom-output inputs (the composed map's
    rounding), plus the all-reduce term."""
    scale = 1.0 / n_examples if mean else 1.0
    z = det["logit"].astype(np.float64)
    ztol = 1e-5 * np.abs(z) + 1e-6 * det["logit_bound"]
    tG = np.abs(det["top_G"]).astype(np.float64)                      # [B, 1]
    dG = 0.25 * ztol[:, None] * scale                                  # |dG/dz| <= 1/4
    top_tol, _ = chain_grad_bounds(det["top_in"], det["top_layers"], 1e-5 * tG + dG)
    if "top_in_bound" in det:
        # the bottom output's composition rounding, 1e-6 of its bound (as for the logit), summed
        # coherently over the batch; it moves h_l = z·R + c by δz·R only, so the kernels carry
        # it and the biases (Σ_b g_l) do not
        zb = np.zeros_like(det["top_in_bound"])
        nD = det["bottom_dout"].shape[1]
        # an output the ReLU clamps (pre-activation below -its rounding) is exactly 0 in both
        pb = magnitude_chain(np.abs(det["bottom_in"]), det["bottom_layers"])
        live = det["bottom_pre"] > -1e-5 * pb
        zb[:, -nD:] = 1e-6 * det["top_in_bound"][:, -nD:] * live
        nob = [(k, np.zeros_like(b)) for k, b in det["top_layers"]]
        ib, _ = chain_grad_bounds(zb, nob, tG + dG)
        top_tol = [(tk + ak, tb) for (tk, tb), (ak, _) in zip(top_tol, ib)]
    if world > 1:
        u = 2.0 ** -24
        ar, _ = chain_grad_bounds(det["top_in"], det["top_layers"], (world - 1) * u * tG)
        top_tol = [(tk + ak, tb + ab) for (tk, tb), (ak, ab) in zip(top_tol, ar)]
    # bottom chain upstream gradient dbot = (interaction part) + G·Q0[F²:]: its tolerance
    F2 = det["top_in"].shape[1] - det["bottom_dout"].shape[1]
    qtail = det["top_Q"][F2:][None, :]
    ddbot = 1e-5 * det["dbot_interaction_bound"] + (1e-5 * tG + dG) * qtail
    # ReLU outputs whose pre-activation is within rounding of 0 may go either way
    pre_bound = magnitude_chain(np.abs(det["bottom_in"]), det["bottom_layers"])
    amb = np.abs(det["bottom_pre"]) <= 1e-5 * pre_bound
    bG = np.abs(det["bottom_G"]).astype(np.float64)
    dGb = ddbot + amb * (np.abs(det["bottom_dout"]) + ddbot)
    bot_tol, _ = chain_grad_bounds(det["bottom_in"], det["bottom_layers"], 1e-5 * bG + dGb)
    if world > 1:  # the all-reduce of A_bot / s_bot, as for the top chain
        ar, _ = chain_grad_bounds(det["bottom_in"], det["bottom_layers"],
                                  (world - 1) * 2.0 ** -24 * (bG + dGb))
        bot_tol = [(tk + ak, tb + ab) for (tk, tb), (ak, ab) in zip(bot_tol, ar)]
    return top_tol, bot_tol


def checked_dlrm_sgd_step(model, step, cat, dn, lb, lr, state=None) -> dict:
    """Run `step` (a recommender_amd.ctr.train.TrainStep with a fused SparseSGD) on one batch and
    check it against the oracle; raises AssertionError on a mismatch, returns a summary.
    state: a dict reused across consecutive calls; it carries the oracle's own MLP layers."""
    import torch

    emb = model.embedding_layer
    W = emb.weight
    dev = W.device
    V, D = W.shape
    B, S = cat.shape
    so = emb.slot_offsets.cpu().numpy() if emb.slot_offsets is not None else None
    rows = global_rows(cat, V, so).reshape(B, S)
    assert (rows >= 0).all(), "the checker expects in-range ids"
    uniq = np.unique(rows)
    compact = np.searchsorted(uniq, rows).astype(np.int64)  # monotone: same sort order
    ut = torch.from_numpy(uniq).to(dev)
    emb.wait_update()
    torch.cuda.synchronize()
    before = W[ut].cpu().numpy()
    probe = np.setdiff1d(np.r_[np.arange(0, V, max(V // 41, 1)), V - 1, V - 2], uniq)
    pt = torch.from_numpy(probe).to(dev)
    probe_before = W[pt].cpu().numpy()
    top0, bot0 = _layers(model.top_mlp), _layers(model.bottom_mlp)
    if state is None:
        state = {}
    if "top" not in state:
        state["top"] = [(k.copy(), b.copy()) for k, b in top0]
        state["bottom"] = [(k.copy(), b.copy()) for k, b in bot0]
    st = DLRMState(before.copy(), None, state["bottom"], state["top"])

    captured = {}
    opt = step.opt_sparse
    apply = opt.apply  # the side-stream and the current-stream (apply_now) update both call it

    def spy(table, ids, grad_rows, params, sorted_ids=None, row_scale=None):
        captured["grad_rows"], captured["sorted"] = grad_rows, sorted_ids
        captured["row_scale"] = row_scale
        return apply(table, ids, grad_rows, params, sorted_ids=sorted_ids, row_scale=row_scale)

    opt.apply = spy
    try:
        batch = (torch.from_numpy(cat).to(dev), torch.from_numpy(dn).to(dev),
                 torch.from_numpy(lb).to(dev))
        loss = float(step(batch).detach())
    finally:
        del opt.apply
    emb.wait_update()
    torch.cuda.synchronize()
    assert "grad_rows" in captured, "the fused sparse apply did not run"
    p_gpu = step.last_pred.cpu().numpy().astype(np.float64)
    after = W[ut].cpu().numpy()
    g_gpu = captured["grad_rows"].cpu().numpy().reshape(B * S, D)
    if captured["row_scale"] is not None:
        # the fused step hands unit rows + G[b]: the apply's row is their one fp32 product
        sc = captured["row_scale"].cpu().numpy().astype(np.float32)
        g_gpu = (np.repeat(sc, S)[:, None] * g_gpu).astype(np.float32)
    s_rows = captured["sorted"].rows.cpu().numpy().view(np.uint32).astype(np.int64)
    s_pos = captured["sorted"].pos.cpu().numpy()
    assert np.array_equal(W[pt].cpu().numpy(), probe_before), "an untouched row changed"
    tgrad_gpu, bgrad_gpu = _grads(model.top_mlp), _grads(model.bottom_mlp)
    top1, bot1 = _layers(model.top_mlp), _layers(model.bottom_mlp)

    det: dict = {}
    ref_loss = dlrm_sgd_step(st, compact, dn, lb, lr, det)
    state["top"], state["bottom"] = st.top, st.bottom
    assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss), f"loss {loss} vs oracle {ref_loss}"

    z_ref = det["logit"].astype(np.float64)
    pc = np.clip(p_gpu, 1e-30, 1 - 1e-7)
    z_gpu = np.log(pc) - np.log1p(-pc)
    res = 2 * np.spacing(p_gpu.astype(np.float32)).astype(np.float64) / (pc * (1 - pc))
    ztol = 1e-5 * np.abs(z_ref) + 1e-6 * det["logit_bound"] + res
    zerr = np.abs(z_gpu - z_ref)
    assert (zerr <= ztol).all(), (
        f"logit off at example {int(np.argmax(zerr / ztol))}: max err/tol {(zerr / ztol).max():.3g}")

    # the dense half: twelve parameter gradients against the oracle, then the SGD apply
    mean = getattr(step, "loss_reduction", "mean") == "mean"
    top_tol, bot_tol = dense_half_tolerances(det, B, mean)
    top_ratio = _check_chain("top MLP", tgrad_gpu, det["top_grads"], top_tol)
    bot_ratio = _check_chain("bottom MLP", bgrad_gpu, det["bottom_grads"], bot_tol)
    _check_sgd("top MLP", top0, top1, tgrad_gpu, lr)
    _check_sgd("bottom MLP", bot0, bot1, bgrad_gpu, lr)

    assert np.array_equal(uniq[det["sorted_rows"].astype(np.int64)], s_rows), "sorted rows differ"
    assert np.array_equal(det["sorted_pos"], s_pos), "sorted positions differ"

    gerr = np.abs(g_gpu.astype(np.float64) - det["dx"])
    gtol = 1e-5 * det["dx_bound"] + 1e-38
    assert (gerr <= gtol).all(), f"grad rows: max err/bound {(gerr / gtol).max():.3g}"

    ur, ug = segment_sum_tiled(det["sorted_rows"], det["sorted_pos"], g_gpu, uniq.size)
    assert np.array_equal(ur.astype(np.int64), np.arange(uniq.size))
    expect = before - np.float32(lr) * ug
    bad = (after != expect).any(1)
    assert not bad.any(), f"{int(bad.sum())} of {uniq.size} touched rows differ from the oracle apply"
    changed = float((after != before).mean())
    assert changed >= 0.25, f"only {changed:.2%} of touched elements changed: vacuous check"
    d_gpu = after.astype(np.float64) - before
    d_ref = st.table.astype(np.float64) - before
    row_scale = np.abs(d_ref).max(1, keepdims=True)
    assert (np.abs(d_gpu - d_ref) <= 1e-4 * row_scale + 2 * np.spacing(np.abs(before))).all(), \
        "table update differs from the all-oracle step beyond 1e-4 of the row's |delta|"
    return {"loss": loss, "oracle_loss": ref_loss, "touched_rows": int(uniq.size),
            "max_row": int(uniq.max()), "rows_beyond_2^32_elems": int((uniq * D >= (1 << 32)).sum()),
            "logit_err_over_tol": float((zerr / ztol).max()),
            "grad_err_over_bound": float((gerr / gtol).max()),
            "top_mlp_grad_err_over_tol": top_ratio, "bottom_mlp_grad_err_over_tol": bot_ratio,
            "frac_elements_changed": changed}


def checked_dlrm_keras_step(model, step, cat, dn, lb, state) -> dict:
    """One production DLRM step with the reference's active optimizer, Keras Adam on every
    variable (ctr/train.py:80,84: tf.keras.optimizers.Adam(); the table's IndexedSlices through
    _resource_apply_sparse, i.e. dense m / v decay and a dense var update [3p TF 2.2]), checked
    against the oracle. `step`: a TrainStep(model, "keras_adam", ...) with a fused SparseAdam,
    deferred decay or not; `state`: a dict reused across consecutive calls.

    Checks: loss, logits, the table gradient rows and the twelve MLP gradients as
    checked_dlrm_sgd_step; every MLP parameter = Keras Adam of its own gradient from its own
    m / v, bit for bit; the table, m and v — after SparseAdam.materialize(), on every row any
    checked step touched (the only rows with non-zero m / v, so the only rows Keras moves) —
    BIT-EXACT against the oracle's tiled dedup of the kernel's gradient rows + Keras sparse
    apply, the oracle carrying those rows' w / m / v across the steps itself."""
    import torch

    from .embedding import apply_keras_adam, keras_adam_coefficients
    from .models import keras_adam_torch

    emb = model.embedding_layer
    opt = step.opt_sparse
    W = emb.weight
    dev = W.device
    V, D = W.shape
    B, S = cat.shape
    so = emb.slot_offsets.cpu().numpy() if emb.slot_offsets is not None else None
    rows = global_rows(cat, V, so).reshape(B, S)
    assert (rows >= 0).all(), "the checker expects in-range ids"
    opt.materialize()
    emb.wait_update_raw()
    torch.cuda.synchronize()
    m_t, v_t, _ = opt._slots(emb)
    union = state.get("rows", np.zeros(0, np.int64))
    new = np.setdiff1d(np.unique(rows), union)
    nt = torch.from_numpy(new).to(dev)
    w_new = W[nt].cpu().numpy()
    assert not m_t[nt].any() and not v_t[nt].any(), "an unchecked row has Adam state"
    allr = np.union1d(union, new)
    wu = np.empty((allr.size, D), np.float32)
    mu = np.zeros((allr.size, D), np.float32)
    vu = np.zeros((allr.size, D), np.float32)
    if union.size:
        at = np.searchsorted(allr, union)
        wu[at], mu[at], vu[at] = state["w"], state["m"], state["v"]
    wu[np.searchsorted(allr, new)] = w_new
    compact = np.searchsorted(allr, rows).astype(np.int64)
    dense = [p for l in list(model.top_mlp.mlp) + list(model.bottom_mlp.mlp) for p in (l.kernel, l.bias)]
    d0 = [p.detach().clone() for p in dense]
    s0 = [{k: v.detach().clone() for k, v in step.opt_dense.state[p].items()} for p in dense]
    top0, bot0 = _layers(model.top_mlp), _layers(model.bottom_mlp)

    captured = {}
    apply = opt.apply

    def spy(table, ids, grad_rows, params, sorted_ids=None, row_scale=None):
        captured["grad_rows"], captured["sorted"] = grad_rows, sorted_ids
        captured["row_scale"] = row_scale
        return apply(table, ids, grad_rows, params, sorted_ids=sorted_ids, row_scale=row_scale)

    opt.apply = spy
    try:
        batch = (torch.from_numpy(cat).to(dev), torch.from_numpy(dn).to(dev),
                 torch.from_numpy(lb).to(dev))
        loss = float(step(batch).detach())
    finally:
        del opt.apply
    opt.materialize()
    emb.wait_update_raw()
    torch.cuda.synchronize()
    assert "grad_rows" in captured, "the fused sparse apply did not run"
    g_gpu = captured["grad_rows"].cpu().numpy().reshape(B * S, D)
    if captured["row_scale"] is not None:  # unit rows + G[b]: the apply's row is their product
        sc = captured["row_scale"].cpu().numpy().astype(np.float32)
        g_gpu = (np.repeat(sc, S)[:, None] * g_gpu).astype(np.float32)
    p_gpu = step.last_pred.cpu().numpy().astype(np.float64)

    st = DLRMState(wu.copy(), None, [(k.copy(), b.copy()) for k, b in bot0],
                   [(k.copy(), b.copy()) for k, b in top0])
    det: dict = {}
    ref_loss = dlrm_sgd_step(st, compact, dn, lb, 0.0, det)  # lr 0: the step's gradients only
    assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss), f"loss {loss} vs oracle {ref_loss}"
    z_ref = det["logit"].astype(np.float64)
    pc = np.clip(p_gpu, 1e-30, 1 - 1e-7)
    z_gpu = np.log(pc) - np.log1p(-pc)
    res = 2 * np.spacing(p_gpu.astype(np.float32)).astype(np.float64) / (pc * (1 - pc))
    ztol = 1e-5 * np.abs(z_ref) + 1e-6 * det["logit_bound"] + res
    assert (np.abs(z_gpu - z_ref) <= ztol).all(), "logits"
    gerr = np.abs(g_gpu.astype(np.float64) - det["dx"])
    assert (gerr <= 1e-5 * det["dx_bound"] + 1e-38).all(), "grad rows"
    top_tol, bot_tol = dense_half_tolerances(det, B, step.loss_reduction == "mean")
    _check_chain("top MLP", _grads(model.top_mlp), det["top_grads"], top_tol)
    _check_chain("bottom MLP", _grads(model.bottom_mlp), det["bottom_grads"], bot_tol)
    it = step.opt_dense.iterations
    c = {k: float(x) for k, x in keras_adam_coefficients(it, step.opt_dense.param_groups[0]["lr"]).items()}
    for i, (p, p0, sd) in enumerate(zip(dense, d0, s0)):
        want, _, _ = keras_adam_torch(p0, sd.get("m", torch.zeros_like(p0)),
                                      sd.get("v", torch.zeros_like(p0)), p.grad, c)
        assert torch.equal(p.detach(), want), f"MLP parameter {i} is not Keras Adam of its gradient"

    ur, ug = segment_sum_tiled(det["sorted_rows"], det["sorted_pos"], g_gpu, allr.size)
    co = keras_adam_coefficients(opt.iterations, opt.lr)
    w2, m2, v2 = apply_keras_adam(wu, mu, vu, ur.astype(np.int64), ug, co)
    at = torch.from_numpy(allr).to(dev)
    for name, got, want in (("table", W[at], w2), ("m", m_t[at], m2), ("v", v_t[at], v2)):
        g = got.cpu().numpy()
        bad = (g != want).any(1)
        assert not bad.any(), f"{name}: {int(bad.sum())} of {allr.size} rows differ from the oracle"
    state.update(rows=allr, w=w2, m=m2, v=v2)
    return {"loss": loss, "oracle_loss": ref_loss, "rows_checked": int(allr.size),
            "step": int(opt.iterations), "rows_beyond_2^32_elems": int((allr * D >= (1 << 32)).sum())}
