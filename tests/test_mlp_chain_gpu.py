"""The ctr MLP's factored backward (nn._LinearChainFn; the reference's hidden Dense layers are
linear, ctr/layers.py:8) against the layer-by-layer float64 oracle (oracle/ctr.py mlp_backward):
forward bit-identical to the layerwise path (or, composed, within 1e-5 of the oracle); kernel / bias / input gradients within 1e-5 of the
oracle relative to the magnitude bound of the factored products, (|R|ᵀ|x|ᵀ|G| + |c|⊗Σ|G|)·|Q|ᵀ,
which bounds both evaluation orders."""
import numpy as np
import pytest
import torch

from oracle.ctr import mlp_backward, mlp_forward
from recommender_amd.ctr.layers import MLP
from tests.conftest import assert_close_rel, chain_grad_bounds

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _factored_at_any_batch():
    """The production path factors from batch 8192 up; these tests use small batches."""
    old = MLP.factored_min_batch
    MLP.factored_min_batch = 0
    yield
    MLP.factored_min_batch = old


def _make(units, act, fin, seed):
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    m = MLP(units, act, in_features=fin, device=DEV, generator=g)
    for l in m.mlp:
        with torch.no_grad():
            l.bias.uniform_(-0.1, 0.1, generator=g)
    return m


@pytest.mark.parametrize("units,act,fin,B,rows", [
    ([512, 256, 1], "sigmoid", 480, 2048, None),
    ([64, 32, 1], "sigmoid", 100, 1000, 48),   # compact-row first layer (DLRM top MLP)
    ([128, 64, 16], "relu", 13, 3000, None),   # DLRM bottom MLP shape
    ([32, 1], None, 40, 700, None),            # DeepFM head (linear final)
    ([8], "relu", 5, 333, None),               # single layer
])
@pytest.mark.parametrize("composed", [False, True])
def test_factored_backward_matches_oracle(units, act, fin, B, rows, composed, rng):
    m_f = _make(units, act, fin, 1)
    m_l = _make(units, act, fin, 1)
    m_f.composed_forward = composed
    m_l.factored_backward = False
    ridx = None
    width = fin
    if rows is not None:
        ridx = torch.from_numpy(np.sort(rng.choice(fin, rows, replace=False))).to(DEV)
        width = rows
    x = rng.standard_normal((B, width)).astype(np.float32)
    xf = torch.from_numpy(x).to(DEV).requires_grad_(True)
    xl = torch.from_numpy(x).to(DEV).requires_grad_(True)
    yf, yl = m_f(xf, rows=ridx), m_l(xl, rows=ridx)
    if not composed:
        assert torch.equal(yf, yl)  # the forward is layerwise in both
    dy = rng.standard_normal(yf.shape).astype(np.float32)
    yf.backward(torch.from_numpy(dy).to(DEV))
    yl.backward(torch.from_numpy(dy).to(DEV))

    # float64 oracle on the layers as the input sees them
    layers = []
    for i, l in enumerate(m_f.mlp):
        k = l.kernel.detach().cpu().numpy().astype(np.float64)
        if i == 0 and ridx is not None:
            k = k[ridx.cpu().numpy()]
        layers.append((k, l.bias.detach().cpu().numpy().astype(np.float64)))
    out, cache = mlp_forward(x.astype(np.float64), layers, act)
    dx, grads = mlp_backward(dy.astype(np.float64), layers, cache, act)
    G = dy.astype(np.float64)
    if act == "sigmoid":
        G = G * out * (1 - out)
    elif act == "relu":
        G = G * (out > 0)
    # magnitude bounds of the factored products: h_{l-1} = x·R + c, so
    # |h_{l-1}ᵀ·G| <= |R|ᵀ·(|x|ᵀ·|G|) + |c|⊗Σ|G|  (>= |h_{l-1}|ᵀ·|G|, the layerwise bound)
    aG = np.abs(G)
    base = np.abs(x.astype(np.float64)).T @ aG
    Mb, absR, absc = [], None, None
    for i, (k, b) in enumerate(layers):
        Mb.append(base if i == 0 else absR.T @ base + np.outer(absc, aG.sum(0)))
        absR = np.abs(k) if absR is None else absR @ np.abs(k)
        absc = np.abs(b) if absc is None else np.abs(k).T @ absc + np.abs(b)
    absQ = None
    bounds = {}
    for i in range(len(layers) - 1, -1, -1):
        bound, bscale = Mb[i], aG.sum(0)
        if absQ is not None:
            bound, bscale = bound @ absQ.T, bscale @ absQ.T
        bounds[i] = bound
        got = m_f.mlp[i].kernel.grad.cpu().numpy()
        if i == 0 and ridx is not None:
            r = ridx.cpu().numpy()
            assert (np.delete(got, r, axis=0) == 0).all()
            got = got[r]
        assert_close_rel(got, grads[i][0], 1e-5, bound, f"dK{i}")
        assert_close_rel(m_f.mlp[i].bias.grad.cpu().numpy(), grads[i][1], 1e-5, bscale, f"db{i}")
        absQ = np.abs(layers[i][0]) if absQ is None else np.abs(layers[i][0]) @ absQ
    assert_close_rel(xf.grad.cpu().numpy(), dx, 1e-5, np.abs(G) @ absQ.T, "dx")
    # the output (composed: x·K_1···K_L + c_L; layerwise: layer by layer) within 1e-5 of the
    # oracle relative to |x|·|K_1|···|K_L| + |c_L|, which bounds both evaluation orders
    ybound = np.abs(x.astype(np.float64)) @ absR + absc
    assert_close_rel(yf.detach().cpu().numpy(), out, 1e-5, ybound, "y")
    # and the layerwise GPU path against the same oracle (the reference's evaluation order)
    for i in range(len(layers)):
        ref = grads[i][0]
        got = m_l.mlp[i].kernel.grad.cpu().numpy()
        if i == 0 and ridx is not None:
            got = got[ridx.cpu().numpy()]
        assert_close_rel(got, ref, 1e-5, bounds[i], f"layerwise dK{i}")


def test_rank1_interaction_bwd_bit_identical(rng):
    """rs_dlrm_interaction_bwd_rank1(G, p) == rs_dlrm_interaction_bwd on the materialised G ⊗ p."""
    from recommender_amd import _lib as L
    from recommender_amd.functional import COMPACT_ALIGN

    S, D, B, V = 26, 128, 777, 20000
    F = S + 1
    width = (F * (F - 1) // 2 + D + COMPACT_ALIGN - 1) // COMPACT_ALIGN * COMPACT_ALIGN
    table = torch.from_numpy(rng.standard_normal((V, D)).astype(np.float32)).to(DEV)
    ids = torch.from_numpy(rng.integers(0, V, (B, S))).to(DEV)
    dense = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(DEV)
    G = torch.from_numpy(rng.standard_normal(B).astype(np.float32)).to(DEV)
    p = torch.from_numpy(rng.standard_normal(width).astype(np.float32)).to(DEV)
    gmat = (G[:, None] * p[None, :]).contiguous()
    st = L.stream_ptr(torch.device(DEV))
    outs = []
    for rank1 in (False, True):
        ge = torch.empty(B * S, D, device=DEV)
        gd = torch.empty(B, D, device=DEV)
        if rank1:
            L.call("rs_dlrm_interaction_bwd_rank1", L.ptr(table), V, D, L.ptr(ids), 1, S, None,
                   L.ptr(dense), B, L.ptr(G), L.ptr(p), width, L.ptr(ge), L.ptr(gd), st)
        else:
            L.call("rs_dlrm_interaction_bwd", L.ptr(table), V, D, L.ptr(ids), 1, S, None,
                   L.ptr(dense), B, 1, L.ptr(gmat), width, L.ptr(ge), L.ptr(gd), st)
        outs.append((ge, gd))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("composed", [False, True])
def test_dlrm_fused_top_matches_layerwise(composed, rng, monkeypatch):
    """DLRM at D = 128 (the fused interaction + top-MLP chain with the rank-one backward)
    against the same model with the layer-by-layer MLP backward: logits bit-identical (layerwise
    chain forward) or within 1e-5 (composed chain forward), every gradient within 1e-5 relative
    to its magnitude."""
    from recommender_amd.ctr.model import DLRM

    monkeypatch.setattr(MLP, "composed_forward", composed)
    S, D, B, V = 26, 128, 1024, 50000
    models = []
    for _ in range(2):
        g = torch.Generator(device=DEV)
        g.manual_seed(3)
        models.append(DLRM([64, D], [64, 32, 1], D, V, S, 13, device=DEV, generator=g))
    x = {"cat_features": torch.from_numpy(rng.integers(0, V, (B, S))).to(DEV),
         "int_features": torch.from_numpy(rng.standard_normal((B, 13)).astype(np.float32)).to(DEV)}
    # the layerwise model's chain inputs / outputs, for the gradients' magnitude bounds
    seen = {}

    def grab(name):
        def hook(mod, args, kwargs, out):
            seen[name] = (args[0].detach(), out)
            out.register_hook(lambda g: seen.__setitem__(name + "_dy", g.detach()))
        return hook

    hs = [models[1].bottom_mlp.register_forward_hook(grab("bottom"), with_kwargs=True),
          models[1].top_mlp.register_forward_hook(grab("top"), with_kwargs=True)]
    MLP.factored_backward = True
    p1 = models[0](x)
    MLP.factored_backward = False
    try:
        p2 = models[1](x)
    finally:
        MLP.factored_backward = True
    if composed:
        # per example, relative to p itself (no absolute floor)
        assert_close_rel(p1.detach().cpu().numpy(), p2.detach().cpu().numpy(), 1e-5, 0.0, "p")
    else:
        assert torch.equal(p1, p2)
    gy = torch.from_numpy(rng.standard_normal(B).astype(np.float32)).to(DEV)
    p1.backward(gy)
    MLP.factored_backward = False
    try:
        p2.backward(gy)
    finally:
        MLP.factored_backward = True
    for h in hs:
        h.remove()
    bounds = {}
    for name, act in (("bottom", "relu"), ("top", "sigmoid")):
        xin, y = seen[name]
        y = y.detach().cpu().numpy().astype(np.float64)
        G = seen[name + "_dy"].cpu().numpy().astype(np.float64)
        G = G * (y > 0) if act == "relu" else G * y * (1 - y)
        mlp = getattr(models[1], name + "_mlp")
        lay = []
        for i, l in enumerate(mlp.mlp):
            k = l.kernel.detach().cpu().numpy().astype(np.float64)
            if i == 0 and name == "top":
                k = k[models[1].compact_rows.cpu().numpy()]
            lay.append((k, l.bias.detach().cpu().numpy().astype(np.float64)))
        kb, dxb = chain_grad_bounds(xin.cpu().numpy(), lay, G)
        bounds[name + "_dx"] = dxb
        for i, (kbound, bbound) in enumerate(kb):
            if i == 0 and name == "top":  # scatter back onto the full [F*F + D, units] kernel
                full = np.zeros(mlp.mlp[0].kernel.shape)
                full[models[1].compact_rows.cpu().numpy()] = kbound
                kbound = full
            bounds[f"{name}_mlp.mlp.{i}.kernel"] = kbound
            bounds[f"{name}_mlp.mlp.{i}.bias"] = bbound
    for (n1, a), (_, b) in zip(models[0].named_parameters(), models[1].named_parameters()):
        if a.grad is None and b.grad is None:
            continue
        ga, gb = a.grad.cpu().numpy(), b.grad.cpu().numpy()
        # per element, relative to the magnitude bound of the products both orders sum
        assert_close_rel(ga, gb, 1e-5, bounds[n1], n1)
    (i1, r1), (i2, r2) = models[0].embedding_layer.take_grad(), models[1].embedding_layer.take_grad()
    assert torch.equal(i1, i2)
    r2n = r2.cpu().numpy()
    # grad rows dX = (M + Mᵀ)·X per example, M the strict-upper dZ: bound |M_b + M_bᵀ|·|X|
    F = S + 1
    iu = np.triu_indices(F, 1)
    mb = np.zeros((B, F, F))
    mb[:, iu[0], iu[1]] = bounds["top_dx"][:, : iu[0].size]
    X = np.concatenate([models[1].embedding_layer.weight.cpu().numpy()[x["cat_features"].cpu().numpy()],
                        seen["bottom"][1].detach().cpu().numpy()[:, None, :]], axis=1)
    xb = np.matmul(mb + mb.transpose(0, 2, 1), np.abs(X.astype(np.float64)))
    assert_close_rel(r1.cpu().numpy(), r2n, 1e-5, xb[:, :S].reshape(B * S, D), "emb grad rows")
