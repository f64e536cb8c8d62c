"""Composed linear-chain forward kernels (nn.chain_forward composed=True; the reference's ctr MLP
hidden layers are linear, ctr/layers.py:8, so each MLP is y = act(x·Q_0 + c_L)):
rs_chain_aug_product / rs_affine_narrow_fwd (narrow input, the DLRM bottom MLP),
rs_chain3_vec_compose / rs_rowdot_act (the [n1, n2, 1] top MLPs) and the top MLP fused into the
interaction kernel (rs_dlrm_interaction_fwd_head). Checked against the float64 layer-by-layer
forward (oracle/ctr.py mlp_forward order) within 1e-5 relative to |x|·|K_1|···|K_L| + |c|, the
magnitude bound of both evaluation orders; the interaction row itself bit-identical to
rs_dlrm_interaction_fwd."""
import numpy as np
import pytest
import torch

from recommender_amd import _lib as L
from recommender_amd import nn as N
from tests.conftest import assert_close_rel

pytestmark = pytest.mark.gpu
DEV = "cuda"


class _Layer:
    def __init__(self, k, b, act=0):
        self.kernel, self.bias, self.act_code = k, b, act


def _chain(dims, bias, act, seed):
    g = np.random.default_rng(seed)
    ks = [g.standard_normal((dims[i], dims[i + 1])) / np.sqrt(dims[i]) for i in range(len(dims) - 1)]
    bs = [g.uniform(-0.1, 0.1, dims[i + 1]) if bias else None for i in range(len(dims) - 1)]
    layers = [_Layer(torch.tensor(k, dtype=torch.float32, device=DEV),
                     None if b is None else torch.tensor(b, dtype=torch.float32, device=DEV))
              for k, b in zip(ks, bs)]
    layers[-1].act_code = act
    return ks, bs, layers


def _ref(x, ks, bs, act, rows=None):
    """float64 layer-by-layer forward and the magnitude bound of the composed product."""
    h = x.astype(np.float64)
    bound = np.abs(h)
    for i, (k, b) in enumerate(zip(ks, bs)):
        k = k if (i > 0 or rows is None) else k[rows]
        h = h @ k + (b if b is not None else 0.0)
        bound = bound @ np.abs(k) + (np.abs(b) if b is not None else 0.0)
    if act == 1:
        h = np.maximum(h, 0.0)
    elif act == 2:
        h = 1.0 / (1.0 + np.exp(-h))
    return h, bound


@pytest.mark.parametrize("dims,bias,act,B", [
    ([13, 512, 256, 128], True, 1, 4099),   # DLRM bottom MLP (north star)
    ([13, 64, 16], False, 0, 257),          # no biases
    ([5, 7, 12], True, 2, 33),              # n % 64 != 0, 3 float4 columns per row
    ([32, 40, 200], True, 1, 1000),         # widest input; 50 lanes per row (5 rows per pass)
    ([1, 4, 8], True, 0, 3),                # one feature
])
def test_narrow_chain_forward(dims, bias, act, B):
    ks, bs, layers = _chain(dims, bias, act, sum(dims))
    x = np.random.default_rng(B).standard_normal((B, dims[0])).astype(np.float32)
    xt = torch.from_numpy(x).to(DEV)
    y, used = N.chain_forward(xt, layers, None, composed=True)
    assert all(u is l.kernel for u, l in zip(used, layers))
    ref, bound = _ref(x, ks, bs, act)
    if act == 2:
        bound = np.full_like(bound, 1.0)
    assert_close_rel(y.cpu().numpy(), ref, 1e-5, bound, "y")
    # deterministic: a second evaluation is bit-identical
    y2, _ = N.chain_forward(xt, layers, None, composed=True)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("n0,n1,n2,B,act,with_rows", [
    (480, 512, 256, 4097, 2, True),   # DLRM top MLP on the compact row
    (428, 512, 256, 1024, 0, False),  # DeepFM-shaped input, linear head
    (16, 8, 4, 5, 1, False),
    (1024, 64, 32, 130, 2, False),    # widest rs_rowdot_act row
])
def test_vec_chain_forward(n0, n1, n2, B, act, with_rows):
    full = n0 + 37 if with_rows else n0
    ks, bs, layers = _chain([full, n1, n2, 1], True, act, n0 + B)
    rows = np.random.default_rng(1).permutation(full)[:n0] if with_rows else None
    x = np.random.default_rng(B).standard_normal((B, n0)).astype(np.float32)
    rt = torch.from_numpy(rows).to(DEV) if with_rows else None
    y, _ = N.chain_forward(torch.from_numpy(x).to(DEV), layers, rt, composed=True)
    assert y.shape == (B, 1)
    ref, bound = _ref(x, ks, bs, act, rows)
    if act == 2:
        bound = np.full_like(bound, 1.0)
    assert_close_rel(y.cpu().numpy(), ref, 1e-5, bound, "y")


def test_vec_compose_values():
    """q = K1[rows]·K2·K3 and c = b3 + K3ᵀ·b2 + (K2·K3)ᵀ·b1 against float64."""
    ks, bs, layers = _chain([300, 96, 40, 1], True, 0, 7)
    rows = np.arange(0, 300, 3)
    q, c = N.vec_chain_compose(layers, torch.from_numpy(rows).to(DEV), rows.size)
    q1 = ks[1] @ ks[2]
    qref = (ks[0][rows] @ q1)[:, 0]
    cref = bs[2][0] + ks[2][:, 0] @ bs[1] + q1[:, 0] @ bs[0]
    qb = (np.abs(ks[0][rows]) @ np.abs(ks[1]) @ np.abs(ks[2]))[:, 0]
    assert_close_rel(q.cpu().numpy(), qref, 1e-5, qb, "q")
    assert abs(float(c) - cref) <= 1e-5 * (abs(bs[2][0]) + np.abs(ks[2][:, 0]) @ np.abs(bs[1])
                                          + np.abs(q1[:, 0]) @ np.abs(bs[0]))


@pytest.mark.parametrize("id64,oob", [(True, False), (False, False), (True, True)])
def test_interaction_head(id64, oob):
    """rs_dlrm_interaction_fwd_head: the row bit-identical to rs_dlrm_interaction_fwd, y within
    1e-5 of act(row·q + c) in float64; an out-of-range id still sets the error flag."""
    S, D, B, V = 26, 128, 1031, 5000
    F = S + 1
    width = 480
    g = np.random.default_rng(11)
    table = torch.from_numpy(g.standard_normal((V, D)).astype(np.float32) * 0.1).to(DEV)
    ids_np = g.integers(0, V, (B, S))
    if oob:
        ids_np[7, 3] = V + 5
    ids = torch.from_numpy(ids_np.astype(np.int64 if id64 else np.int32)).to(DEV)
    dense = torch.from_numpy(g.standard_normal((B, D)).astype(np.float32)).to(DEV)
    q = torch.from_numpy(g.standard_normal(width).astype(np.float32) * 0.05).to(DEV)
    c = torch.tensor([0.3], device=DEV)
    st = L.stream_ptr(DEV)
    z0 = torch.empty(B, width, device=DEV)
    z1 = torch.empty(B, width, device=DEV)
    y = torch.empty(B, 1, device=DEV)
    f0 = torch.zeros(1, dtype=torch.int32, device=DEV)
    f1 = torch.zeros(1, dtype=torch.int32, device=DEV)
    code = L.RS_ID_I64 if id64 else L.RS_ID_I32
    L.call("rs_dlrm_interaction_fwd", L.ptr(table), V, D, L.ptr(ids), code, S, None, L.ptr(dense),
           B, 1, L.ptr(z0), width, L.ptr(f0), st)
    L.call("rs_dlrm_interaction_fwd_head", L.ptr(table), V, D, L.ptr(ids), code, S, None,
           L.ptr(dense), B, L.ptr(z1), width, L.ptr(q), L.ptr(c), 2, L.ptr(y), L.ptr(f1), st)
    assert torch.equal(z0, z1)
    assert int(f0) == int(f1) == (1 if oob else 0)
    zz = z1.cpu().numpy().astype(np.float64)
    ref = 1.0 / (1.0 + np.exp(-(zz @ q.cpu().numpy().astype(np.float64) + 0.3)))
    assert_close_rel(y.cpu().numpy()[:, 0], ref, 1e-5, np.ones_like(ref), "y")
    assert F * (F - 1) // 2 + D <= width


@pytest.mark.parametrize("id64,oob,slots", [(True, False, 26), (False, False, 26), (True, True, 26),
                                            (True, False, 13), (True, False, 31)])
def test_interaction_head_dx(id64, oob, slots):
    """rs_dlrm_interaction_fwd_head_dx: row and y bit-identical to rs_dlrm_interaction_fwd_head;
    the unit gradient U = (M + Mᵀ)·X (M = strict-upper pairs of q) within 1e-5 of float64,
    relative to |M + Mᵀ|·|X|; the bottom row carries q's dense part; rows are zero for OOB ids;
    G[b]·U equals the rank-one backward's rows within the same bound."""
    S, D, B, V = slots, 128, 517, 5000
    F = S + 1
    nzc = F * (F - 1) // 2
    width = (nzc + D + 15) // 16 * 16
    g = np.random.default_rng(13)
    table = torch.from_numpy(g.standard_normal((V, D)).astype(np.float32) * 0.1).to(DEV)
    ids_np = g.integers(0, V, (B, S))
    if oob:
        ids_np[7, 3] = V + 5
        ids_np[100, 0] = -1
    ids = torch.from_numpy(ids_np.astype(np.int64 if id64 else np.int32)).to(DEV)
    dense = torch.from_numpy(g.standard_normal((B, D)).astype(np.float32)).to(DEV)
    q = torch.from_numpy(g.standard_normal(width).astype(np.float32) * 0.05).to(DEV)
    c = torch.tensor([0.3], device=DEV)
    st = L.stream_ptr(DEV)
    code = L.RS_ID_I64 if id64 else L.RS_ID_I32
    z0, z1 = torch.empty(B, width, device=DEV), torch.empty(B, width, device=DEV)
    y0, y1 = torch.empty(B, 1, device=DEV), torch.empty(B, 1, device=DEV)
    f0, f1 = torch.zeros(1, dtype=torch.int32, device=DEV), torch.zeros(1, dtype=torch.int32, device=DEV)
    ue = torch.full((B * S, D), float("nan"), device=DEV)
    ud = torch.full((B, D), float("nan"), device=DEV)
    L.call("rs_dlrm_interaction_fwd_head", L.ptr(table), V, D, L.ptr(ids), code, S, None,
           L.ptr(dense), B, L.ptr(z0), width, L.ptr(q), L.ptr(c), 2, L.ptr(y0), L.ptr(f0), st)
    L.call("rs_dlrm_interaction_fwd_head_dx", L.ptr(table), V, D, L.ptr(ids), code, S, None,
           L.ptr(dense), B, L.ptr(z1), width, L.ptr(q), L.ptr(c), 2, L.ptr(y1), L.ptr(ue),
           L.ptr(ud), L.ptr(f1), st)
    assert torch.equal(z0, z1) and torch.equal(y0, y1)
    assert int(f0) == int(f1) == (1 if oob else 0)
    # float64 reference
    tb = table.cpu().numpy().astype(np.float64)
    ok = (ids_np >= 0) & (ids_np < V)
    X = np.zeros((B, F, D))
    X[:, :S][ok] = tb[ids_np[ok]]
    X[:, S] = dense.cpu().numpy()
    qn = q.cpu().numpy().astype(np.float64)
    Msym = np.zeros((F, F))
    iu = np.triu_indices(F, 1)
    Msym[iu] = qn[:nzc]
    Msym = Msym + Msym.T
    U = np.einsum("ik,bkd->bid", Msym, X)
    Ub = np.einsum("ik,bkd->bid", np.abs(Msym), np.abs(X))
    U[:, S] += qn[nzc:nzc + D]
    Ub[:, S] += np.abs(qn[nzc:nzc + D])
    got_e = ue.cpu().numpy().reshape(B, S, D)
    got_d = ud.cpu().numpy()
    assert np.isfinite(got_e).all() and np.isfinite(got_d).all()
    assert_close_rel(got_e, U[:, :S], 1e-5, Ub[:, :S], "unit emb grad")
    assert_close_rel(got_d, U[:, S], 1e-5, Ub[:, S], "unit dense grad")
    if S == 26 and not oob:
        # the rank-one backward's rows (G ⊗ q materialised) vs G[b] * U
        G = torch.from_numpy(g.standard_normal(B).astype(np.float32)).to(DEV)
        ge, gd = torch.empty(B * S, D, device=DEV), torch.empty(B, D, device=DEV)
        L.call("rs_dlrm_interaction_bwd_rank1", L.ptr(table), V, D, L.ptr(ids), code, S, None,
               L.ptr(dense), B, L.ptr(G), L.ptr(q), width, L.ptr(ge), L.ptr(gd), st)
        Gn = np.abs(G.cpu().numpy().astype(np.float64))
        scaled = (G.reshape(B, 1, 1) * ue.view(B, S, D)).cpu().numpy()
        assert_close_rel(scaled, ge.cpu().numpy().reshape(B, S, D), 2e-5,
                         Gn[:, None, None] * Ub[:, :S], "G * unit vs rank-one rows")


@pytest.mark.parametrize("dims,bias", [([13, 512, 256, 128], True), ([13, 64, 32, 16, 8], False),
                                       ([7, 12, 20], True), ([32, 40, 24], True)])
def test_narrow_chain_backward(dims, bias):
    """_narrow_chain_grads_hip (P-chain + outer products over n0 + 1 rows) against float64
    autograd of the layer-by-layer chain, 1e-5 relative to the magnitude of the products."""
    ks, bs, layers = _chain(dims, bias, 1, 3 * sum(dims))
    B = 2000
    g = np.random.default_rng(5)
    x = g.standard_normal((B, dims[0]))
    G = g.standard_normal((B, dims[-1]))
    A = torch.tensor((x.T @ G), dtype=torch.float32, device=DEV)
    s = torch.tensor(G.sum(0), dtype=torch.float32, device=DEV)
    for l in layers:
        l.kernel.grad = None
        if l.bias is not None:
            l.bias.grad = None
    N.chain_forward(torch.tensor(x, dtype=torch.float32, device=DEV), layers, None, composed=True)
    assert N.narrow_chain_hip_ready(layers, dims[0])
    q0 = N._narrow_chain_grads_hip(layers, [l.kernel for l in layers], A, s, need_q0=True)
    # float64 reference
    kt = [torch.tensor(k, requires_grad=True) for k in ks]
    bt = [torch.tensor(b, requires_grad=True) if b is not None else None for b in bs]
    h = torch.tensor(x)
    for k, b in zip(kt, bt):
        h = h @ k + (b if b is not None else 0.0)
    h.backward(torch.tensor(G))
    absx, absG = np.abs(x), np.abs(G)
    # magnitude bound: |h_{j-1}|ᵀ·|G|·|Q_j|ᵀ
    hb = absx
    for j, l in enumerate(layers):
        Qb = np.eye(dims[-1])
        for k in reversed(ks[j + 1:]):
            Qb = np.abs(k) @ Qb
        kb = hb.T @ absG @ Qb.T
        assert_close_rel(l.kernel.grad.cpu().numpy(), kt[j].grad.numpy(), 1e-5, kb, f"dK{j}")
        if l.bias is not None:
            assert_close_rel(l.bias.grad.cpu().numpy(), bt[j].grad.numpy(), 1e-5,
                             absG.sum(0) @ Qb.T, f"db{j}")
        hb = hb @ np.abs(ks[j]) + (np.abs(bs[j]) if bs[j] is not None else 0.0)
    Q, Qb = ks[0], np.abs(ks[0])
    for k in ks[1:]:
        Q, Qb = Q @ k, Qb @ np.abs(k)
    assert_close_rel(q0.cpu().numpy(), Q, 1e-5, Qb, "Q0")


def test_compose_cache_follows_parameter_updates():
    """The forward's composition is cached per parameter version: an in-place update (as the
    optimizer step does) makes the next forward recompose."""
    dims = [13, 64, 32]
    ks, bs, layers = _chain(dims, True, 0, 99)
    x = np.random.default_rng(2).standard_normal((100, 13)).astype(np.float32)
    xt = torch.from_numpy(x).to(DEV)
    y1, _ = N.chain_forward(xt, layers, None, composed=True)
    with torch.no_grad():
        layers[1].kernel.mul_(0.5)
        layers[0].bias.add_(1.0)
    ks[1] = ks[1] * 0.5
    bs[0] = bs[0] + 1.0
    y2, _ = N.chain_forward(xt, layers, None, composed=True)
    ref, bound = _ref(x, ks, bs, 0)
    assert_close_rel(y2.cpu().numpy(), ref, 1e-5, bound, "y after update")
    assert not torch.equal(y1, y2)


def test_graph_replay_then_eager_matches_eager_only():
    """A HIP-graph replay updates the parameters in place without bumping their version
    counters: eager steps after replays must recompose the chains (nn.invalidate_compose_cache).
    capture + replay / eager / forward-only / replay / eager equals the same steps run eagerly,
    bit for bit (without the invalidation the last eager step reuses the forward-only pass's
    compositions, made before the second replay's update)."""
    from recommender_amd.ctr.layers import MLP
    from recommender_amd.ctr.train import TrainStep, build_model
    from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

    old = MLP.factored_min_batch
    MLP.factored_min_batch = 0
    try:
        cards = criteo_cardinalities(100_000, 26)
        rng = np.random.default_rng(3)
        bs = []
        for _ in range(2):
            cat, dn, lb = criteo_batch(rng, 512, cards)
            bs.append(tuple(torch.from_numpy(x).to(DEV) for x in (cat, dn, lb)))
        models = []
        for mode in ("graph", "eager"):
            g = torch.Generator(device=DEV).manual_seed(5)
            m = build_model("DLRM", 128, sum(cards), 26, 13, torch.device(DEV), slot_cardinalities=cards,
                            bottom=[64, 128], top=[64, 32, 1], generator=g)
            st = TrainStep(m, "sgd", lr=0.05, fused=True, defer_sparse_join=True)
            def peek():  # an eager forward with no update: caches the current compositions
                m({"cat_features": bs[1][0], "int_features": bs[1][1]})

            if mode == "graph":
                replay = st.capture(bs[0], warmup=3)       # 3 eager warm-up steps on bs[0]
                replay(); st(bs[1]); peek(); replay(); st(bs[1])
            else:
                for b in (bs[0],) * 3 + (bs[0], bs[1]):
                    st(b)
                peek()
                st(bs[0]); st(bs[1])
            m.embedding_layer.wait_update()
            torch.cuda.synchronize()
            models.append(m)
        pa, pb = dict(models[0].named_parameters()), dict(models[1].named_parameters())
        for n in pa:
            assert torch.equal(pa[n], pb[n]), n
        assert torch.equal(models[0].embedding_layer.weight, models[1].embedding_layer.weight)
    finally:
        MLP.factored_min_batch = old


@pytest.mark.parametrize("D", [128, 64])
def test_graph_sequence_matches_eager_fused_step(D):
    """The graph modes of benchmarks/bench_models.py --cfg2-graph: a pool of fused DLRM steps
    captured as ONE graph (TrainStep.capture_sequence: each step's sparse update on its side
    stream overlaps the next step's bottom MLP inside the graph) and replayed twice leaves the
    slab and every MLP parameter bit-identical to the same steps run eagerly, at D = 128 (the
    north star) and D = 64 (cfg2)."""
    from recommender_amd.ctr.layers import MLP
    from recommender_amd.ctr.train import TrainStep, build_model
    from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

    old = MLP.factored_min_batch
    MLP.factored_min_batch = 0
    try:
        cards = criteo_cardinalities(100_000, 26)
        rng = np.random.default_rng(11)
        bs = []
        for _ in range(3):
            cat, dn, lb = criteo_batch(rng, 1024, cards)
            bs.append(tuple(torch.from_numpy(x).to(DEV) for x in (cat, dn, lb)))
        models = []
        for mode in ("graph", "eager"):
            g = torch.Generator(device=DEV).manual_seed(7)
            m = build_model("DLRM", D, sum(cards), 26, 13, torch.device(DEV), slot_cardinalities=cards,
                            bottom=[64, D], top=[64, 32, 1], generator=g)
            st = TrainStep(m, "sgd", lr=0.05, fused=True, defer_sparse_join=True)
            assert st.fused_step_ready(bs[0])
            if mode == "graph":
                replay = st.capture_sequence(bs, warmup=1)   # 1 eager pass over the pool
                replay()
                replay()
            else:
                for b in bs * 3:
                    st(b)
            m.embedding_layer.wait_update()
            torch.cuda.synchronize()
            models.append(m)
        pa, pb = dict(models[0].named_parameters()), dict(models[1].named_parameters())
        for n in pa:
            assert torch.equal(pa[n], pb[n]), n
        assert torch.equal(models[0].embedding_layer.weight, models[1].embedding_layer.weight)
    finally:
        MLP.factored_min_batch = old
