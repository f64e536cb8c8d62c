"""The ctr MLP's factored backward (nn._LinearChainFn; the reference's hidden Dense layers are
linear, ctr/layers.py:8) against the layer-by-layer float64 oracle (oracle/ctr.py mlp_backward):
forward bit-identical to the layerwise path; kernel / bias / input gradients within 1e-5 of the
oracle relative to the magnitude bound of the factored products, (|R|ᵀ|x|ᵀ|G| + |c|⊗Σ|G|)·|Q|ᵀ,
which bounds both evaluation orders."""
import numpy as np
import pytest
import torch

from oracle.ctr import mlp_backward, mlp_forward
from recommender_amd.ctr.layers import MLP
from tests.conftest import assert_close_rel

pytestmark = pytest.mark.gpu
DEV = "cuda"


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
def test_factored_backward_matches_oracle(units, act, fin, B, rows, rng):
    m_f = _make(units, act, fin, 1)
    m_l = _make(units, act, fin, 1)
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
    # and the layerwise GPU path against the same oracle (the reference's evaluation order)
    for i in range(len(layers)):
        ref = grads[i][0]
        got = m_l.mlp[i].kernel.grad.cpu().numpy()
        if i == 0 and ridx is not None:
            got = got[ridx.cpu().numpy()]
        assert_close_rel(got, ref, 1e-5, bounds[i], f"layerwise dK{i}")
