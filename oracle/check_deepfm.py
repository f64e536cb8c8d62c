"""Checker for one DeepFM Keras-Adam train step (SURVEY cfg1) against oracle/ctr.py.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py; parity unpinned): called by
tests/test_deepfm_gpu.py. It drives the product path (recommender_amd TrainStep on cuda: gather,
FM kernel, MLP, fused BCE, sparse Keras Adam on the shared table, dense KerasAdam) and checks it
from the same pre-step state (reference: ctr/model.py:6-31, ctr/train.py:81-85).
Checks (tolerances stated here):
  * loss within 1e-5 relative;
  * per-example logits (recovered from p) within 1e-5 of their own value plus 1e-6 of their
    float64 magnitude bound (FM: 0.5·Σ((Σ|e|)² + Σ e²); chain: |x|·|K1|·|K2|·|K3| + |biases|);
  * table gradient rows within 1e-5 of their float64 magnitude bound;
  * table, m, v over ALL rows (Keras Adam is dense) BIT-EXACT against the oracle's tiled
    segmented sum + Keras apply fed with the kernel's own gradient rows;
  * dense kernels / biases within 1e-6 + 1e-4·|update| of the all-oracle Keras Adam step.
"""
from __future__ import annotations

import numpy as np

from .ctr import deepfm_keras_adam_step


def _np(t):
    return t.detach().cpu().numpy().copy()


def checked_deepfm_adam_step(model, step, cat, dn, lb) -> dict:
    import torch

    emb = model.embedding_layer
    W = emb.weight
    dev = W.device
    B, S = cat.shape
    D = W.shape[1]
    opt = step.opt_sparse
    m_t, v_t, _ = opt._slots(emb)
    emb.wait_update()
    torch.cuda.synchronize()
    so = emb.slot_offsets.cpu().numpy() if emb.slot_offsets is not None else None
    table0, m0, v0 = _np(W), _np(m_t), _np(v_t)
    layers0 = [(_np(l.kernel), _np(l.bias)) for l in model.mlp.mlp]

    def dstate(p, key):
        st = step.opt_dense.state.get(p, {})
        return _np(st[key]) if key in st else np.zeros(tuple(p.shape), np.float32)

    dm0 = [(dstate(l.kernel, "m"), dstate(l.bias, "m")) for l in model.mlp.mlp]
    dv0 = [(dstate(l.kernel, "v"), dstate(l.bias, "v")) for l in model.mlp.mlp]
    it = opt.iterations + 1

    captured = {}
    apply = opt.apply  # both the fused (side-stream) and the step()-time apply go through it

    def spy(table, ids, grad_rows, params, sorted_ids=None, row_scale=None):
        captured["grad_rows"], captured["sorted"] = grad_rows, sorted_ids
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
    assert "grad_rows" in captured, "the sparse apply did not run"
    g_gpu = captured["grad_rows"].cpu().numpy().reshape(B * S, D).astype(np.float32)
    p_gpu = step.last_pred.cpu().numpy().astype(np.float64)

    ref_loss, ref, det = deepfm_keras_adam_step(table0, m0, v0, layers0, dm0, dv0, cat, dn, lb,
                                                it, slot_offsets=so)
    assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss), f"loss {loss} vs oracle {ref_loss}"
    z_ref = det["logit"].astype(np.float64)
    pc = np.clip(p_gpu, 1e-30, 1 - 1e-7)
    z_gpu = np.log(pc) - np.log1p(-pc)
    res = 2 * np.spacing(p_gpu.astype(np.float32)).astype(np.float64) / (pc * (1 - pc))
    ztol = 1e-5 * np.abs(z_ref) + 1e-6 * det["logit_bound"] + res
    zerr = np.abs(z_gpu - z_ref)
    assert (zerr <= ztol).all(), f"logits: max err/tol {(zerr / ztol).max():.3g}"
    if captured["sorted"] is not None:  # the fused path's side-stream radix sort
        s_rows = captured["sorted"].rows.cpu().numpy().view(np.uint32).astype(np.int64)
        s_pos = captured["sorted"].pos.cpu().numpy()
        assert np.array_equal(det["sorted_rows"].astype(np.int64), s_rows), "sorted rows differ"
        assert np.array_equal(det["sorted_pos"], s_pos), "sorted positions differ"
    gerr = np.abs(g_gpu.astype(np.float64) - det["dx"])
    gtol = 1e-5 * det["dx_bound"] + 1e-38
    assert (gerr <= gtol).all(), f"grad rows: max err/bound {(gerr / gtol).max():.3g}"

    # the apply, bit for bit, from the kernel's own gradient rows
    _, pinned, _ = deepfm_keras_adam_step(table0, m0, v0, layers0, dm0, dv0, cat, dn, lb, it,
                                          slot_offsets=so, grad_rows=g_gpu)
    for name, got, want in (("table", _np(W), pinned["table"]), ("m", _np(m_t), pinned["m"]),
                            ("v", _np(v_t), pinned["v"])):
        bad = got != want
        assert not bad.any(), f"{name}: {int(bad.sum())} of {bad.size} elements differ from the oracle apply"
    moved = _np(W) != table0
    touched = np.unique(det["sorted_rows"].astype(np.int64))
    changed = float(moved[touched].mean())
    assert changed >= 0.25, f"only {changed:.2%} of touched elements changed: vacuous check"
    # the dense half: every row with momentum from earlier steps moves, touched or not
    carried = (m0 != 0).any(1)
    if carried.any():
        frac = float(moved[carried].any(1).mean())
        assert frac > 0.99, f"Keras Adam's dense update moved only {frac:.2%} of rows with momentum"
    derr = 0.0
    for l, (k0, b0), (k1, b1) in zip(model.mlp.mlp, layers0, ref["layers"]):
        for got, before, want in ((_np(l.kernel), k0, k1), (_np(l.bias), b0, b1)):
            tol = 1e-6 + 1e-4 * np.abs(want - before)
            e = np.abs(got - want)
            assert (e <= tol).all(), f"dense parameter off: max err/tol {(e / tol).max():.3g}"
            derr = max(derr, float((e / tol).max()))
    return {"loss": loss, "oracle_loss": ref_loss, "logit_err_over_tol": float((zerr / ztol).max()),
            "grad_err_over_bound": float((gerr / gtol).max()), "dense_err_over_tol": derr,
            "touched_elements_changed": changed,
            "rows_with_momentum": int((m0 != 0).any(1).sum())}
