"""The whole DIEN train step (dien/train.py:14-22: mean Keras BCE + mean auxiliary loss, Keras
Adam on every variable, the mask_zero tables included) against oracle/dien.py dien_step, in both
head BatchNormalization modes (recommender_amd/dien/model.py: "propagate", TF 2.2's training
propagation, and "inference"), and the graph-capturable step against the eager one.

Per step, from the GPU's pre-step state (Adam's normalisation turns the sign of a near-zero
gradient into a full lr-sized move, so two trajectories rounded differently separate by design;
each step is therefore checked from the same state, and the update itself bit for bit):
  * loss within 1e-5 relative of the float64 oracle, predictions per element;
  * every dense gradient and every table gradient row per element against the float64 oracle:
    1e-5 relative + 4x the fp32 oracle's own error there (sampled over three batch orders) +
    for the dense gradients 1e-5 of the element's float64 batch-reduction magnitude (Σ over 32
    batch chunks of |chunk contribution|), for the rows 1e-6 of the tensor's largest;
  * every dense parameter = Keras Adam of its own gradient from its own m / v, bit for bit;
  * both tables and their m / v, all rows (Keras' sparse Adam is dense), bit-exact against the
    oracle's tiled dedup + Keras apply of the kernel's own gradient rows;
  * the head BN's moving averages ("propagate") within 1e-5 of the float64 oracle's.
"""
import numpy as np
import pytest
import torch

from oracle import dien as OD
from oracle import embedding as OE
from oracle.models import keras_adam_torch
from tests.conftest import assert_close_f64 as _close64

pytestmark = pytest.mark.gpu


def assert_close_f64(got, r64, r32, msg, mag=None):
    """mag (dense gradients): the float64 magnitude of the batch reduction, Σ over 32 chunks of
    the batch of |chunk contribution| (oracle.dien.dien_grad_magnitude); 1e-5 of it per element
    (≈ 170 fp32 ulps of the summed magnitude; each chunk still cancels over its 8 examples x L
    steps) covers any fp32 summation order over the batch —
    the GPU reduces the B·L terms in another structure than the oracle samples. Without it (the
    per-position table gradient rows, each a chain through up to L recurrent steps): 1e-6 of the
    tensor's largest."""
    if mag is None:
        _close64(got, r64, r32, msg, floor=1e-6)
        return
    g = got.detach().double().cpu().numpy()
    r = r64.detach().double().cpu().numpy()
    spread = np.max([np.abs(x.detach().double().cpu().numpy() - r) for x in r32], axis=0)
    tol = 1e-5 * np.abs(r) + 4 * spread + 1e-5 * mag.detach().double().cpu().numpy()
    err = np.abs(g - r)
    bad = ~(err <= tol)
    assert not bad.any(), (f"{msg}: {int(bad.sum())} / {bad.size} off; max err/tol "
                           f"{float((err / np.maximum(tol, 1e-300)).max()):.3g}")


DEV = "cuda"
IV, CV = 3001, 81


def _model(mode, seed=2):
    from recommender_amd.dien import DIEN

    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    return DIEN(36, 36, head_bn_mode=mode, item_vocab_size=IV, item_embedding_size=18,
                cat_vocab_size=CV, cat_embedding_size=18, mlp_units=[200, 80, 1], device=DEV,
                generator=g)


def _batches(n, B=256, L=50, seed=5):
    from recommender_amd.dien.train import synthetic_batch

    r = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        f, lab = synthetic_batch(r, B, L, IV, CV)
        out.append(({k: torch.from_numpy(v).to(DEV) for k, v in f.items()},
                    torch.from_numpy(lab).to(DEV)))
    return out


def _checked_step(model, step, feats, label):
    """One eager DIENStep checked against the oracle; returns the loss."""
    tables = {"item": model.item_embedding, "cat": model.cat_embedding}
    snap = {k: (t.weight.detach().clone(),) + tuple(x.detach().clone() for x in
                                                     step.opt_sparse._slots(t)[:2])
            for k, t in tables.items()}
    dense = {n: p for n, p in model.named_parameters() if not n.endswith("grad_handle")}
    d0 = {n: p.detach().clone() for n, p in dense.items()}
    st0 = {n: {k: v.detach().clone() for k, v in step.opt_dense.state[p].items()}
           for n, p in dense.items()}
    bn0 = (model.mlp.bn.moving_mean.clone(), model.mlp.bn.moving_variance.clone())
    ref64 = OD.dien_step(model, feats, label, torch.float64)
    mag = OD.dien_grad_magnitude(model, feats, label, chunks=32, bn_stats=ref64["bn_batch"])
    B = label.shape[0]
    gp = torch.Generator(device=DEV).manual_seed(1)
    perms = [None, torch.arange(B - 1, -1, -1, device=DEV),
             torch.randperm(B, device=DEV, generator=gp)]
    r32 = [OD.dien_step(model, feats, label, torch.float32, perm=p) for p in perms]
    ref32 = {"prob": [r["prob"] for r in r32],
             "grads": {n: [r["grads"][n] for r in r32] for n in ref64["grads"]},
             "rows": {k: [r["rows"][k] for r in r32] for k in ref64["rows"]},
             "stats": ([r["stats"][0] for r in r32], [r["stats"][1] for r in r32])
             if ref64["stats"] is not None else None}

    # the lookups' gradient chunks in the order the tables receive them, and the applies
    order = {k: [] for k in tables}
    acc = {k: t.accumulate_grad for k, t in tables.items()}
    cap = {}
    apply = step.opt_sparse.apply
    for k, t in tables.items():
        def rec(ids, grad_rows, valid=None, _k=k, _f=acc[k]):
            order[_k].append(ids.reshape(-1).clone())
            return _f(ids, grad_rows, valid=valid)
        t.accumulate_grad = rec

    def spy(table, ids, grad_rows, params, sorted_ids=None, row_scale=None, valid=None):
        name = "item" if table is tables["item"] else "cat"
        cap[name] = (ids.clone(), grad_rows.clone(), None if valid is None else valid.clone())
        return apply(table, ids, grad_rows, params, sorted_ids=sorted_ids, row_scale=row_scale,
                     valid=valid)

    step.opt_sparse.apply = spy
    try:
        total, _ = step(feats, label)
    finally:
        del step.opt_sparse.apply
        for t in tables.values():
            del t.accumulate_grad
    torch.cuda.synchronize()
    loss = float(total)
    assert abs(loss - ref64["loss"]) <= 1e-5 * abs(ref64["loss"]), (loss, ref64["loss"])
    assert_close_f64(step.last_pred, ref64["prob"], ref32["prob"], "prediction")

    # dense: gradients vs the oracle, update = Keras Adam of the GPU's own gradient
    it = step.opt_dense.iterations
    co = OE.keras_adam_coefficients(it, step.opt_dense.param_groups[0]["lr"])
    c = {k: float(v) for k, v in co.items()}
    for n, p in dense.items():
        assert p.grad is not None, f"{n}: no gradient"
        assert_close_f64(p.grad, ref64["grads"][n], ref32["grads"][n], f"grad {n}", mag[n])
        m0 = st0[n].get("m", torch.zeros_like(p))
        v0 = st0[n].get("v", torch.zeros_like(p))
        want, _, _ = keras_adam_torch(d0[n], m0, v0, p.grad, c)
        assert torch.equal(p.detach(), want), f"{n} is not Keras Adam of its own gradient"

    # tables: the kernel's rows vs the oracle's per lookup, then the apply bit for bit
    keys = {"item": ("target_item", "pos_his_item", "neg_his_item"),
            "cat": ("target_cat", "pos_his_cat", "neg_his_cat")}
    for name, t in tables.items():
        ids, rows, valid = cap[name]
        o = 0
        for chunk in order[name]:
            key = [k for k in keys[name] if torch.equal(chunk.long(), feats[k].reshape(-1).long())]
            assert len(key) == 1, "cannot tell the lookup of a gradient chunk"
            n = chunk.numel()
            assert_close_f64(rows[o:o + n], ref64["rows"][key[0]], ref32["rows"][key[0]],
                             f"{key[0]} gradient rows")
            o += n
        assert o == ids.numel()
        w0, m0, v0 = (x.cpu().numpy() for x in snap[name])
        # the history steps the model masks carry no gradient and are left out of the sums
        # (Embedding grad_mask): the oracle sorts them as out-of-range ids
        kept = ids.cpu().numpy()
        if valid is not None:
            assert bool((rows[valid == 0] == 0).all()), "a left-out position had a gradient"
            kept = np.where(valid.cpu().numpy() != 0, kept, -1)
        sr, sp, _ = OE.sort_ids(kept, t.input_dim)
        ur, ug = OE.segment_sum_tiled(sr, sp, rows.cpu().numpy(), t.input_dim)
        cot = OE.keras_adam_coefficients(step.opt_sparse.iterations, step.opt_sparse.lr)
        w2, m2, v2 = OE.apply_keras_adam(w0, m0, v0, ur.astype(np.int64), ug, cot)
        m_t, v_t, _ = step.opt_sparse._slots(t)
        np.testing.assert_array_equal(t.weight.cpu().numpy(), w2, err_msg=f"{name} table")
        np.testing.assert_array_equal(m_t.cpu().numpy(), m2, err_msg=f"{name} m")
        np.testing.assert_array_equal(v_t.cpu().numpy(), v2, err_msg=f"{name} v")

    bn = model.mlp.bn
    if model.head_bn_mode == "propagate":
        for got, r, r3, nm in ((bn.moving_mean, ref64["stats"][0], ref32["stats"][0], "moving mean"),
                               (bn.moving_variance, ref64["stats"][1], ref32["stats"][1],
                                "moving variance")):
            assert_close_f64(got, r, r3, nm)
        assert not torch.equal(bn.moving_mean, bn0[0])
    else:
        assert torch.equal(bn.moving_mean, bn0[0]) and torch.equal(bn.moving_variance, bn0[1])
    return loss


@pytest.mark.parametrize("mode", ["propagate", "inference"])
def test_dien_train_step_vs_oracle(mode):
    from recommender_amd.dien.train import DIENStep

    model = _model(mode)
    step = DIENStep(model, lr=1e-3)
    for feats, label in _batches(2):
        _checked_step(model, step, feats, label)


def test_dien_static_and_graph_step_equal_eager():
    """DIENStep.static_step (tables densified, Keras Adam with lr_t from device memory) equals the
    eager KerasAdam + SparseAdam(keras) step bit for bit over 3 steps (same gradients, same
    summation order of duplicate rows, same Keras roundings), and the step captured into a HIP
    graph and replayed on refilled input buffers equals the eager static steps bit for bit."""
    from recommender_amd.dien.train import DIENStep

    batches = _batches(3, B=128, L=50)

    def run(mode):
        m = _model("propagate")
        step = DIENStep(m, lr=1e-2)
        st_f = {k: torch.empty_like(v) for k, v in batches[0][0].items()}
        st_l = torch.empty_like(batches[0][1])
        replay, losses = None, []
        for i, (f, lab) in enumerate(batches):
            if mode == "eager":
                losses.append(float(step(f, lab)[0]))
            elif mode == "static" or i == 0:
                losses.append(float(step.static_step(f, lab)[0]))
            else:
                for k, v in f.items():
                    st_f[k].copy_(v)
                st_l.copy_(lab)
                replay = replay or step.capture(st_f, st_l)
                losses.append(float(replay()[0]))
        torch.cuda.synchronize()
        params = {n: p.detach().cpu().numpy().copy() for n, p in m.named_parameters()}
        params["item"] = m.item_embedding.weight.cpu().numpy().copy()
        params["cat"] = m.cat_embedding.weight.cpu().numpy().copy()
        params["bn_mean"] = m.mlp.bn.moving_mean.cpu().numpy().copy()
        return losses, params

    (le, pe), (ls, ps), (lg, pg) = run("eager"), run("static"), run("graph")
    assert le == ls, (le, ls)
    for n in pe:
        np.testing.assert_array_equal(ps[n], pe[n], err_msg=f"static vs eager: {n}")
    # the library GEMMs may pick another algorithm under capture: 1e-5 from the static run
    np.testing.assert_allclose(lg, ls, rtol=1e-5)
    for n in ps:
        np.testing.assert_allclose(pg[n], ps[n], rtol=1e-5, atol=1e-7, err_msg=f"graph: {n}")


def test_graph_keras_adam_skips_a_variable_without_gradient():
    """Keras apply_gradients skips a variable whose gradient is None (no m / v decay, no move);
    a zero gradient still moves a variable with non-zero m. GraphKerasAdam must do the former."""
    from recommender_amd.optim import GraphKerasAdam, KerasAdam

    g = torch.Generator(device=DEV).manual_seed(1)
    a = [torch.randn(37, device=DEV, generator=g), torch.randn(5, 3, device=DEV, generator=g),
         torch.randn(8, device=DEV, generator=g)]
    b = [t.clone() for t in a]
    pa = [torch.nn.Parameter(t) for t in a]
    ka, gk = KerasAdam(pa, lr=1e-2), GraphKerasAdam(b, lr=1e-2)
    grads = [[torch.randn_like(t, generator=None) for t in a] for _ in range(3)]
    grads[1][1] = None  # the middle tensor gets no gradient on step 2
    grads[2][0] = None
    for gs in grads:
        for p, gr in zip(pa, gs):
            p.grad = gr
        ka.step()
        gk.prepare()
        gk.iterations += 1
        gk.apply(gs)
    torch.cuda.synchronize()
    for p, q in zip(pa, b):
        assert torch.equal(p.detach(), q), "GraphKerasAdam differs from KerasAdam (None grads)"
    moved = b[1].clone()
    gk.prepare()
    gk.iterations += 1
    gk.apply([torch.zeros_like(b[0]), torch.zeros_like(b[1]), None])
    assert not torch.equal(b[1], moved), "a zero gradient must still move a variable (m != 0)"
