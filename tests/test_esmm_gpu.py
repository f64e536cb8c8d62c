"""GPU parity: ESMM / MMOE / BASE (esmm/*.py surfaces) vs the same model in plain torch fp32
ops (table lookups by indexing, Keras Dense math), and one optimizer step."""
import numpy as np
import pytest
import torch

from recommender_amd.esmm import FEAT_VOCAB
from recommender_amd.esmm.train import MultiTaskStep, build
from recommender_amd.synthetic import aliccp_batch
from tests.conftest import assert_close_f64, assert_close_rel

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_mlp(mlp, x):
    for l in mlp.mlp:
        x = x @ l.kernel + l.bias
        x = l.activation(x) if l.activation is not None else x
    return x


def _ref_forward(model, feats):
    slab = model.embedding_layer.slab
    w, so = slab.weight, slab.slot_offsets
    e = torch.cat([w[so[i] + feats[f].reshape(-1).long()] for i, f in enumerate(feats)], 1)
    kind = type(model).__name__
    if kind == "ESMM":
        c, v = _ref_mlp(model.ctr, e), _ref_mlp(model.cvr, e)
        return torch.cat([c, c * v], 1)
    if kind == "BaseModel":
        return _ref_mlp(model.mlp, e)
    ex = torch.stack([_ref_mlp(x, e) for x in model.experts], 1)
    outs = []
    for g, t in zip(model.gates, model.task_towers):
        gw = torch.softmax(e @ g.kernel + g.bias, -1)
        outs.append(_ref_mlp(t, (gw.unsqueeze(1) @ ex).squeeze(1)))
    outs[1] = outs[0] * outs[1]
    return torch.cat(outs, 1)


@pytest.mark.parametrize("kind", ["ESMM", "MMOE", "BASE"])
def test_esmm_family_forward(kind):
    vocab = {k: min(v, 5000) for k, v in FEAT_VOCAB.items()}
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    model = build(kind, vocab, 18, DEV, g)
    rng = np.random.default_rng(5)
    f, lab = aliccp_batch(rng, 512, vocab)
    feats = {k: torch.from_numpy(v).to(DEV) for k, v in f.items()}
    with torch.no_grad():
        y = model(feats)
        ref = _ref_forward(model, feats)
    assert y.shape == ref.shape
    assert_close_rel(y.cpu().numpy(), ref.cpu().numpy(), 1e-5, 1e-4, "logits")


def _tol_check(got, ref, rtol, msg, floor=1e-3):
    got, ref = got.detach().cpu().numpy(), ref.detach().cpu().numpy()
    assert_close_rel(got, ref, rtol, np.abs(ref).max() * floor + 1e-30, msg)


@pytest.mark.parametrize("kind", ["ESMM", "MMOE", "BASE"])
def test_esmm_family_keras_adam_step_vs_oracle(kind):
    """One MultiTaskStep (esmm/train.py:97-106, Keras Adam) against oracle/models.py from the
    same pre-step state, evaluated in float64: loss 1e-5; outputs, dense gradients and the
    per-position table gradient rows per element within 1e-5 relative + 4x the fp32 oracle's own
    error there (three batch orders) + 1e-7 of the tensor's largest (1e-6 for the table rows;
    tests/conftest.py assert_close_f64); dense parameters = Keras Adam of the step's own gradients, bit for bit;
    table / m / v (all rows: Keras Adam is dense) bit-exact vs the oracle's tiled dedup + Keras
    apply of the kernel's gradient rows."""
    from oracle import embedding as OE
    from oracle.models import esmm_family_step, keras_adam_torch

    vocab = {k: min(v, 5000) for k, v in FEAT_VOCAB.items()}
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    model = build(kind, vocab, 18, DEV, g)
    step = MultiTaskStep(model, "keras_adam")
    slab = model.embedding_layer.slab
    rng = np.random.default_rng(5)
    f, lab = aliccp_batch(rng, 512, vocab)
    feats = {k: torch.from_numpy(v).to(DEV) for k, v in f.items()}
    lab_t = torch.from_numpy(lab[:, :1] if kind == "BASE" else lab).to(DEV)
    table0 = slab.weight.detach().clone()
    m_t, v_t, _ = step.opt_sparse._slots(slab)
    m0, v0 = m_t.detach().cpu().numpy().copy(), v_t.detach().cpu().numpy().copy()
    dense0 = [p.detach().clone() for p in step.dense]
    ref_loss, ref_y, ref_dg, ref_rows = esmm_family_step(model, table0, slab.slot_offsets, feats,
                                                         lab_t, dtype=torch.float64)
    # fp32 evaluations in three batch orders: their spread is the rounding noise per element
    g = torch.Generator(device="cpu").manual_seed(3)
    perms = [None] + [torch.randperm(512, generator=g).to(DEV) for _ in range(2)]
    r32 = [esmm_family_step(model, table0, slab.slot_offsets, feats, lab_t, perm=p) for p in perms]

    cap = {}
    apply = step.opt_sparse.apply

    def spy(table, ids, grad_rows, params, sorted_ids=None, row_scale=None):
        cap["ids"], cap["rows"] = ids, grad_rows
        return apply(table, ids, grad_rows, params, sorted_ids=sorted_ids, row_scale=row_scale)

    step.opt_sparse.apply = spy
    loss = float(step(feats, lab_t))
    torch.cuda.synchronize()
    assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss)
    assert_close_f64(step.last_pred, ref_y, [r[1] for r in r32], "outputs")
    co = OE.keras_adam_coefficients(1)
    c = {k: float(v) for k, v in co.items()}
    for i, (p, p0, rg) in enumerate(zip(step.dense, dense0, ref_dg)):
        assert_close_f64(p.grad, rg, [r[2][i] for r in r32], f"dense grad {i}")
        want, _, _ = keras_adam_torch(p0, torch.zeros_like(p0), torch.zeros_like(p0), p.grad, c)
        assert torch.equal(p.detach(), want), f"dense parameter {i} is not Keras Adam of its gradient"
    rows_gpu = cap["rows"].reshape(-1, 18)
    # rows run back through every tower layer (relu masks, cancellations): a small element's
    # rounding follows the size of the terms that cancelled there, so its floor is 1e-6 of the
    # largest row element (was 1e-2)
    assert_close_f64(rows_gpu, ref_rows, [r[3] for r in r32], "table gradient rows", floor=1e-6)
    so = slab.slot_offsets.cpu().numpy()
    ids = cap["ids"].cpu().numpy()
    sr, sp, _ = OE.sort_ids(ids, slab.input_dim, so)
    ur, ug = OE.segment_sum_tiled(sr, sp, rows_gpu.cpu().numpy(), slab.input_dim)
    t2, m2, v2 = OE.apply_keras_adam(table0.cpu().numpy(), m0, v0, ur.astype(np.int64), ug, co)
    np.testing.assert_array_equal(slab.weight.cpu().numpy(), t2)
    np.testing.assert_array_equal(m_t.cpu().numpy(), m2)
    np.testing.assert_array_equal(v_t.cpu().numpy(), v2)


@pytest.mark.parametrize("kind", ["ESMM", "MMOE"])
def test_keras_adam_deferred_decay_equals_dense_sweep(kind):
    """cfg4's timed optimizer: MultiTaskStep("keras_adam_deferred") — the reference's Keras Adam
    with each slab row's decay replayed when the row is next read (fused sparse optimizer, no
    per-step dense sweep) — equals MultiTaskStep("keras_adam") (the dense m / v sweep every
    step) after materialize(): table, m, v and every dense parameter bit for bit over 4 steps,
    losses equal."""
    vocab = {k: min(v, 5000) for k, v in FEAT_VOCAB.items()}
    rng = np.random.default_rng(8)
    batches = []
    for _ in range(4):
        f, lab = aliccp_batch(rng, 512, vocab)
        batches.append(({k: torch.from_numpy(v).to(DEV) for k, v in f.items()},
                        torch.from_numpy(lab).to(DEV)))
    res = []
    for opt in ("keras_adam", "keras_adam_deferred"):
        g = torch.Generator(device=DEV)
        g.manual_seed(3)
        model = build(kind, vocab, 18, DEV, g)
        step = MultiTaskStep(model, opt)
        losses = [float(step(f, lab)) for f, lab in batches]
        step.materialize()
        torch.cuda.synchronize()
        slab = model.embedding_layer.slab
        m, v, _ = step.opt_sparse._slots(slab)
        res.append((losses, slab.weight.detach().clone(), m.clone(), v.clone(),
                    [p.detach().clone() for p in step.dense]))
    (la, wa, ma, va, da), (lb, wb, mb, vb, db) = res
    assert la == lb
    assert torch.equal(wa, wb) and torch.equal(ma, mb) and torch.equal(va, vb)
    for x, y in zip(da, db):
        assert torch.equal(x, y)


def _copy_into_sharded(m1, m2, rank=0, world=1):
    sd = {k: v for k, v in m1.state_dict().items() if not k.startswith("embedding_layer")}
    m2.load_state_dict(sd, strict=False)
    full = m1.embedding_layer.slab.weight
    m2.embedding_layer.slab.shard.weight.copy_(full[rank::world])


@pytest.mark.parametrize("opt", ["keras_adam", "lazy_adam"])
@pytest.mark.parametrize("kind", ["ESMM", "MMOE"])
def test_world1_sharded_esmm_equals_unsharded(kind, opt):
    """cfg4's FeatureTables(sharded_comm=...) path at world 1 (owner-major sort, unique / inverse,
    exchange, owner apply) is bit-identical to the one-slab model over two Adam steps."""
    from recommender_amd.sharded import Comm

    vocab = {k: min(v, 5000) for k, v in FEAT_VOCAB.items()}
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    m1 = build(kind, vocab, 18, DEV, g)
    m2 = build(kind, vocab, 18, DEV, torch.Generator(device=DEV).manual_seed(9), sharded_comm=Comm())
    _copy_into_sharded(m1, m2)
    s1, s2 = MultiTaskStep(m1, opt), MultiTaskStep(m2, opt, comm=Comm())
    rng = np.random.default_rng(5)
    for _ in range(2):
        f, lab = aliccp_batch(rng, 512, vocab)
        feats = {k: torch.from_numpy(v).to(DEV) for k, v in f.items()}
        lab_t = torch.from_numpy(lab).to(DEV)
        l1, l2 = float(s1(feats, lab_t)), float(s2(feats, lab_t))
        assert l1 == l2
    torch.cuda.synchronize()
    assert torch.equal(m2.embedding_layer.slab.full_weight(), m1.embedding_layer.slab.weight)
    p2 = dict(m2.named_parameters())
    for n, a in m1.named_parameters():
        if not n.endswith("grad_handle"):
            assert torch.equal(a, p2[n]), n


def _esmm_world2_worker(rank, world, port, q, kind, opt):
    import os

    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import embedding as OE
        from oracle import sharded as OS
        from oracle.models import esmm_family_step, keras_adam_torch
        from recommender_amd.sharded import Comm

        vocab = {k: min(v, 3000) for k, v in FEAT_VOCAB.items()}
        ref = build(kind, vocab, 18, DEV, torch.Generator(device=DEV).manual_seed(3))
        model = build(kind, vocab, 18, DEV, torch.Generator(device=DEV).manual_seed(9),
                      sharded_comm=Comm())
        _copy_into_sharded(ref, model, rank, world)
        step = MultiTaskStep(model, opt, comm=Comm())
        slab = model.embedding_layer.slab
        so_t = slab.slot_offsets
        so = so_t.cpu().numpy()
        table = ref.embedding_layer.slab.weight.detach().clone()   # full slab, oracle state
        t_np = table.cpu().numpy()
        V, D = t_np.shape
        m_np = np.zeros((V, D), np.float32)
        v_np = np.zeros((V, D), np.float32)
        cap = {}
        bex = slab.backward_exchange

        def spy(grad_rows):
            cap["rows"] = grad_rows.detach().cpu().numpy().copy()
            return bex(grad_rows)

        slab.backward_exchange = spy
        rng = np.random.default_rng(5)
        for it in range(2):
            f, lab = aliccp_batch(rng, 512, vocab)            # the global batch; rank r: half r
            half = {k: v[rank * 256:(rank + 1) * 256] for k, v in f.items()}
            feats = {k: torch.from_numpy(v).to(DEV) for k, v in half.items()}
            lab_t = torch.from_numpy(lab[rank * 256:(rank + 1) * 256]).to(DEV)
            dense0 = [p.detach().clone() for p in step.dense]
            st0 = [dict(step.opt_dense.state.get(p, {})) for p in step.dense]
            st0 = [(s["m"].clone(), s["v"].clone()) if s else None for s in st0]
            # oracle dense gradients: each half through oracle/models.py, averaged
            tcur = torch.from_numpy(t_np).to(DEV)
            gs = []
            for r in range(world):
                fr = {k: torch.from_numpy(v[r * 256:(r + 1) * 256]).to(DEV) for k, v in f.items()}
                lr_ = torch.from_numpy(lab[r * 256:(r + 1) * 256]).to(DEV)
                gs.append(esmm_family_step(model, tcur, so_t, fr, lr_)[2])
            step(feats, lab_t)
            torch.cuda.synchronize()
            c = {k: float(v) for k, v in OE.keras_adam_coefficients(it + 1).items()}
            for i, p in enumerate(step.dense):
                want_g = (gs[0][i] + gs[1][i]) * 0.5
                _tol_check(p.grad, want_g, 1e-4, f"all-reduced dense grad {i}")
                m0, v0 = st0[i] if st0[i] is not None else (torch.zeros_like(p), torch.zeros_like(p))
                want, _, _ = keras_adam_torch(dense0[i], m0, v0, p.grad, c)
                assert torch.equal(p.detach(), want), f"dense parameter {i}"
            # sparse: the oracle's sharded Adam from every rank's own gradient rows
            ids = np.stack([half[k].reshape(-1) for k in half], 1).astype(np.int64)
            all_ids = [None] * world
            all_rows = [None] * world
            dist.all_gather_object(all_ids, ids)
            dist.all_gather_object(all_rows, cap["rows"].reshape(-1, D))
            t_np, m_np, v_np = OS.sharded_adam_step(t_np, m_np, v_np, all_ids, all_rows, world,
                                                    it + 1, "keras" if opt == "keras_adam" else "lazy",
                                                    1e-3, so)
            full = slab.full_weight().cpu().numpy()
            np.testing.assert_array_equal(full, t_np)
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("opt", ["keras_adam", "lazy_adam"])
def test_world2_sharded_esmm_matches_oracle(opt):
    """SURVEY cfg4 on two ranks sharing the one GPU (gloo, exchange staged through the host):
    two MultiTaskStep(comm=...) steps of a row-sharded ESMM. The all-reduced dense gradients
    match the mean of oracle/models.py's half-batch gradients (1e-4), the dense parameters are
    Keras Adam of them bit for bit, and the sharded slab equals oracle/sharded.py's sharded Adam
    of the ranks' own gradient rows bit for bit."""
    import os

    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29300 + (os.getpid() % 500) + (7 if opt == "lazy_adam" else 0)
    ps = [ctx.Process(target=_esmm_world2_worker, args=(r, world, port, q, "ESMM", opt))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(60)
    assert all(v == "ok" for v in res.values()), res


def test_shared_input_dense_matches_float64():
    """shared_input_dense (ESMM's two first tower layers as one GEMM over concatenated kernels,
    each output a column block of one activation): outputs equal the layers run one by one
    within fp32 GEMM rounding, and the input / kernel / bias gradients equal a float64
    evaluation under the same relu mask (the mask taken from the outputs, so a pre-activation
    within rounding of 0 cannot flip between the two sides)."""
    from recommender_amd.nn import Dense, shared_input_dense

    g = torch.Generator(device=DEV).manual_seed(3)
    B, fi = 3000, 324
    layers = [Dense(360, "relu", in_features=fi, device=DEV, generator=g),
              Dense(200, "relu", in_features=fi, device=DEV, generator=g)]
    for l in layers:
        l.bias.data.uniform_(-0.1, 0.1, generator=g)
    x = torch.randn(B, fi, device=DEV, generator=g, requires_grad=True)
    ups = [torch.randn(B, l.units, device=DEV, generator=g) for l in layers]
    outs = shared_input_dense(x, layers)
    assert [tuple(o.shape) for o in outs] == [(B, 360), (B, 200)]
    assert outs[0].grad_fn is not None
    with torch.no_grad():
        for o, l in zip(outs, layers):
            sep = torch.relu(x @ l.kernel + l.bias)
            assert_close_rel(o.cpu(), sep.cpu(), rtol=1e-5,
                             scale=float((x.abs() @ l.kernel.abs()).max()) * 1e-2)
    sum((o * u).sum() for o, u in zip(outs, ups)).backward()
    x64 = x.detach().double()
    dx64 = torch.zeros_like(x64)
    mag_dx = torch.zeros_like(x64)
    for o, u, l in zip(outs, ups, layers):
        dz = (o.detach() > 0).double() * u.double()
        k64 = l.kernel.detach().double()
        dx64 += dz @ k64.t()
        mag_dx += dz.abs() @ k64.abs().t()
        assert_close_rel(l.kernel.grad.cpu(), (x64.t() @ dz).cpu(), rtol=1e-5,
                         scale=float((x64.abs().t() @ dz.abs()).max()) * 1e-2, msg="kernel grad")
        assert_close_rel(l.bias.grad.cpu(), dz.sum(0).cpu(), rtol=1e-5,
                         scale=float(dz.abs().sum(0).max()) * 1e-2, msg="bias grad")
    assert_close_rel(x.grad.cpu(), dx64.cpu(), rtol=1e-5, scale=float(mag_dx.max()) * 1e-2,
                     msg="input grad")


def test_side_pool_multi_equals_single_task_poolings():
    """rs_side_pool_fwd_multi / rs_side_pool_bwd_multi (MMOE's T gate poolings over the same
    [E, B, H] expert outputs in one pass) equal T rs_side_pool calls bit for bit: pooled rows,
    softmax weights, logit gradients, and the side gradient as the sum of the T side gradients
    (task order)."""
    from recommender_amd import _lib as L
    from recommender_amd.eges.model import side_pool
    from recommender_amd.esmm.mmoe import _ptrs

    g = torch.Generator(device=DEV).manual_seed(9)
    E, B, H, T = 8, 1000, 80, 3
    y = torch.randn(E, B, H, device=DEV, generator=g)
    z = torch.randn(B, T * E + 3, device=DEV, generator=g)  # logit rows wider than T·E
    ups = [torch.randn(B, H, device=DEV, generator=g) for _ in range(T)]
    st = L.stream_ptr(torch.device(DEV))
    hid = [torch.empty(B, H, device=DEV) for _ in range(T)]
    att = [torch.empty(B, E, device=DEV) for _ in range(T)]
    L.call("rs_side_pool_fwd_multi", L.ptr(y), H, B * H, B, E, H, T,
           _ptrs([z[:, t * E:] for t in range(T)]), z.shape[1], _ptrs(hid), _ptrs(att), None, st)
    dy = torch.empty_like(y)
    dz = torch.full_like(z, 7.0)
    L.call("rs_side_pool_bwd_multi", L.ptr(y), H, B * H, B, E, H, T, _ptrs(att), _ptrs(ups),
           L.ptr(dy), _ptrs([dz[:, t * E:] for t in range(T)]), z.shape[1], st)
    side = y.transpose(0, 1)
    gsum = None
    for t in range(T):
        logit = z[:, t * E:(t + 1) * E].clone().requires_grad_()
        s = side.detach().requires_grad_()
        out = side_pool(s, logit.unsqueeze(1)).squeeze(1)
        assert torch.equal(out.detach(), hid[t])
        out.backward(ups[t])
        assert torch.equal(logit.grad, dz[:, t * E:(t + 1) * E])
        gsum = s.grad.clone() if gsum is None else gsum + s.grad
    assert torch.equal(gsum.transpose(0, 1).contiguous(), dy)
    assert bool((dz[:, T * E:] == 7.0).all())  # columns past the tasks' blocks untouched
    # with side_bias: the rows become relu(z + bias) in place, then pool as before
    bias = torch.randn(E, H, device=DEV, generator=g)
    zz = torch.randn(E, B, H, device=DEV, generator=g)
    want = torch.relu(zz + bias[:, None, :])
    hid2 = [torch.empty(B, H, device=DEV) for _ in range(T)]
    att2 = [torch.empty(B, E, device=DEV) for _ in range(T)]
    L.call("rs_side_pool_fwd_multi", L.ptr(zz), H, B * H, B, E, H, T,
           _ptrs([z[:, t * E:] for t in range(T)]), z.shape[1], _ptrs(hid2), _ptrs(att2),
           L.ptr(bias), st)
    assert torch.equal(zz, want)
    for t in range(T):
        ref = side_pool(want.transpose(0, 1), z[:, t * E:(t + 1) * E].unsqueeze(1)).squeeze(1)
        assert torch.equal(hid2[t], ref)


def test_mmoe_fused_block_matches_separate_nodes(monkeypatch):
    """MMOE's experts / gates / poolings as one node (_ExpertsGatesFn) against the same model run
    through the separate nodes: outputs and every parameter and input gradient equal within
    fp32 GEMM rounding (the two paths reach the library GEMMs with different shapes)."""
    from recommender_amd.esmm import mmoe as M

    vocab = {k: 500 for k in FEAT_VOCAB}
    res = []
    for fused in (True, False):
        monkeypatch.setattr(M, "_FUSED", fused)
        gen = torch.Generator(device=DEV).manual_seed(4)
        model = build("MMOE", vocab, 18, DEV, gen)
        x = torch.randn(4096, len(vocab) * 18, device=DEV,
                        generator=torch.Generator(device=DEV).manual_seed(5)).requires_grad_()
        outs = model._towers(x)
        up = torch.Generator(device=DEV).manual_seed(6)
        loss = sum((o * torch.randn(o.shape, device=DEV, generator=up)).sum() for o in outs)
        loss.backward()
        grads = [x.grad] + [p.grad for n, p in model.named_parameters()
                            if p.grad is not None and "embedding" not in n]
        res.append(([o.detach() for o in outs], grads))
    (o1, g1), (o2, g2) = res
    assert len(g1) == len(g2)
    for a, b in zip(o1, o2):
        assert_close_rel(a.cpu(), b.cpu(), rtol=1e-5)
    for i, (a, b) in enumerate(zip(g1, g2)):
        # each element within 1e-5 of the tensor's largest: the input gradient is a sum over
        # K = E·H0 + T·E = 1616 terms (one GEMM) against the same sum split over three GEMMs and
        # two adds — near-cancelling elements differ by fp32 rounding of the largest terms
        assert_close_rel(a.cpu(), b.cpu(), rtol=1e-4, scale=float(b.abs().max()) * 1e-1,
                         msg=f"grad {i}")
