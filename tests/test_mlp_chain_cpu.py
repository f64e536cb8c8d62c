"""CPU checks of the factored linear-chain MLP backward algebra (recommender_amd/nn.py
chain_param_grads) against float64 autograd on the layer-by-layer chain: the
kernel / bias gradients from A = xᵀ·G and Σ G, and the input-gradient factor Q_0."""
import pytest
import torch

from recommender_amd import nn as N


class _Layer:
    def __init__(self, k, b):
        self.kernel = torch.nn.Parameter(k.clone())
        self.bias = torch.nn.Parameter(b.clone()) if b is not None else None
        self.act_code = 0


@pytest.mark.parametrize("dims,bias", [([7, 9, 5, 3], True), ([6, 8, 4, 1], True), ([5, 2], True),
                                       ([4, 6, 3], False), ([13, 32, 16, 8], True),
                                       # narrow input (n_0 < n_L): _narrow_chain_grads
                                       ([13, 64, 32, 16], True), ([2, 6, 4, 5], False), ([3, 7], True)])
def test_chain_param_grads_match_autograd(dims, bias):
    g = torch.Generator().manual_seed(len(dims) * 10 + dims[0])
    B = 64
    ks = [torch.randn(dims[i], dims[i + 1], dtype=torch.float64, generator=g) for i in range(len(dims) - 1)]
    bs = [torch.randn(dims[i + 1], dtype=torch.float64, generator=g) if bias else None
          for i in range(len(dims) - 1)]
    x = torch.randn(B, dims[0], dtype=torch.float64, generator=g)
    G = torch.randn(B, dims[-1], dtype=torch.float64, generator=g)
    kk = [k.clone().requires_grad_() for k in ks]
    bb = [b.clone().requires_grad_() if b is not None else None for b in bs]
    xr = x.clone().requires_grad_()
    h = xr
    for k, b in zip(kk, bb):
        h = h @ k + (b if b is not None else 0)
    (h * G).sum().backward()
    layers = [_Layer(k, b) for k, b in zip(ks, bs)]
    Q0 = N.chain_param_grads(layers, None, ks, x.t() @ G, G.sum(0))
    for l, k, b in zip(layers, kk, bb):
        torch.testing.assert_close(l.kernel.grad, k.grad, rtol=1e-10, atol=1e-10)
        if b is not None:
            torch.testing.assert_close(l.bias.grad, b.grad, rtol=1e-10, atol=1e-10)
    torch.testing.assert_close(G @ Q0.t(), xr.grad, rtol=1e-10, atol=1e-10)


def test_chain_param_grads_compact_rows():
    """A first layer that reads only some kernel rows (DLRM's compact interaction row): the
    other rows get exactly zero gradient."""
    g = torch.Generator().manual_seed(7)
    rows = torch.tensor([0, 2, 5, 6])
    k1 = torch.randn(8, 5, dtype=torch.float64, generator=g)
    k2 = torch.randn(5, 1, dtype=torch.float64, generator=g)
    b1 = torch.randn(5, dtype=torch.float64, generator=g)
    b2 = torch.randn(1, dtype=torch.float64, generator=g)
    x = torch.randn(16, 4, dtype=torch.float64, generator=g)
    G = torch.randn(16, 1, dtype=torch.float64, generator=g)
    layers = [_Layer(k1, b1), _Layer(k2, b2)]
    N.chain_param_grads(layers, rows, [k1[rows], k2], x.t() @ G, G.sum(0))
    ref = torch.zeros_like(k1)
    ref[rows] = x.t() @ (G @ k2.t())
    torch.testing.assert_close(layers[0].kernel.grad, ref, rtol=1e-10, atol=1e-10)
    assert (layers[0].kernel.grad[[1, 3, 4, 7]] == 0).all()


@pytest.mark.parametrize("dims,bias,act", [([7, 9, 5, 3], True, 0), ([480, 64, 32, 1], True, 2),
                                           ([13, 64, 32, 16], True, 1), ([4, 6, 3], False, 0),
                                           ([5, 2], True, 2)])
def test_composed_forward_matches_layerwise(dims, bias, act):
    """chain_forward(composed=True), y = act(x·K_1···K_L + c_L), in either product order
    (narrow input: left to right; narrow output: right to left), equals the layer-by-layer
    forward in float64, with first-layer rows selected as DLRM's compact row does."""
    g = torch.Generator().manual_seed(dims[0] * 7 + len(dims))
    B = 32
    ks = [torch.randn(dims[i], dims[i + 1], dtype=torch.float64, generator=g) / dims[i] ** 0.5
          for i in range(len(dims) - 1)]
    bs = [torch.randn(dims[i + 1], dtype=torch.float64, generator=g) if bias else None
          for i in range(len(dims) - 1)]
    layers = [_Layer(k, b) for k, b in zip(ks, bs)]
    layers[-1].act_code = act
    for rows in (None, torch.arange(0, dims[0], 2)):
        width = dims[0] if rows is None else rows.numel()
        x = torch.randn(B, width, dtype=torch.float64, generator=g)
        with torch.no_grad():
            yc, ksc = N.chain_forward(x, layers, rows, composed=True)
            yl, ksl = N.chain_forward(x, layers, rows, composed=False)
        torch.testing.assert_close(yc, yl, rtol=1e-12, atol=1e-12)
        assert all(torch.equal(a, b) for a, b in zip(ksc, ksl))
