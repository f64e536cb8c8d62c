"""GPU parity: DotInteraction (all four self/skip_gather modes), the fused DLRM gather +
interaction, and the FM term vs the float64 oracle, within the north-star 1e-5 relative
tolerance (scaled by the Cauchy-Schwarz bound of each dot product)."""
import numpy as np
import pytest
import torch

from oracle import embedding as OE
from oracle import interaction as O
from recommender_amd.embedding import Embedding, SlabEmbedding
from recommender_amd.functional import COMPACT_ALIGN, dlrm_interaction, dot_interaction, fm_interaction
from tests.conftest import assert_close_rel

pytestmark = pytest.mark.gpu
DEV = "cuda"
RTOL = 1e-5


def _pair_scale(x, self_i, skip):
    n = np.sqrt((np.asarray(x, np.float64) ** 2).sum(-1))  # [B, F]
    s = n[:, :, None] * n[:, None, :]
    keep = O.kept_mask(x.shape[1], self_i)
    return s.reshape(x.shape[0], -1) if skip else s[:, keep]


@pytest.mark.parametrize("F,D", [(27, 128), (27, 64), (27, 16), (5, 32), (32, 128), (2, 16), (27, 18), (33, 16), (17, 100)])
@pytest.mark.parametrize("self_i,skip", [(False, True), (False, False), (True, False), (True, True)])
def test_dot_interaction(F, D, self_i, skip, rng):
    B = 67
    x = rng.standard_normal((B, F, D)).astype(np.float32)
    xt = torch.from_numpy(x).to(DEV).requires_grad_(True)
    out = dot_interaction(xt, self_i, skip)
    ref = O.dot_interaction(x, self_i, skip)
    assert out.shape == ref.shape
    assert_close_rel(out.detach().cpu().numpy(), ref, RTOL, _pair_scale(x, self_i, skip), "fwd")
    g = rng.standard_normal(ref.shape).astype(np.float32)
    out.backward(torch.from_numpy(g).to(DEV))
    gref = O.dot_interaction_bwd(x, g, self_i, skip)
    gscale = np.abs(g).max() * np.sqrt((x.astype(np.float64) ** 2).sum(-1)).max() * 2
    assert_close_rel(xt.grad.cpu().numpy(), gref, RTOL, gscale, "bwd")


def test_dot_interaction_known_answer():
    # X = [[1,2],[3,4],[5,6]]: Z = [[5,11,17],[11,25,39],[17,39,61]]
    x = torch.tensor([[[1., 2.], [3., 4.], [5., 6.]]], device=DEV)
    np.testing.assert_array_equal(dot_interaction(x, False, False).cpu().numpy(), [[11, 17, 39]])
    np.testing.assert_array_equal(dot_interaction(x, True, False).cpu().numpy(), [[5, 11, 25, 17, 39, 61]])
    np.testing.assert_array_equal(dot_interaction(x, False, True).cpu().numpy(),
                                  [[0, 11, 17, 0, 0, 39, 0, 0, 0]])


@pytest.mark.parametrize("D", [128, 64, 16, 24])
@pytest.mark.parametrize("slab", [False, True])
@pytest.mark.parametrize("compact", [False, True])
def test_dlrm_fused(D, slab, compact, rng):
    B, S, V = 300, 26, 10_000
    if slab:
        card = rng.integers(1, 800, S)
        t = SlabEmbedding(card, D, device=DEV)
        so = np.concatenate([[0], np.cumsum(card)])
        ids = np.stack([rng.integers(0, c, B) for c in card], 1).astype(np.int64)
    else:
        t = Embedding(V, D, device=DEV)
        so = None
        ids = rng.integers(0, V, (B, S)).astype(np.int32)
    w = t.weight.cpu().numpy()
    dense = rng.standard_normal((B, D)).astype(np.float32)
    dt = torch.from_numpy(dense).to(DEV).requires_grad_(True)
    out = dlrm_interaction(t, torch.from_numpy(ids).to(DEV), dt, compact)
    ref = O.dlrm_interaction(w, ids, dense, so)
    F = S + 1
    keep_cols = np.r_[np.flatnonzero(np.triu(np.ones((F, F), bool), 1).reshape(-1)), F * F + np.arange(D)]
    if compact:
        ref = ref[:, keep_cols]
        pad = (ref.shape[1] + COMPACT_ALIGN - 1) // COMPACT_ALIGN * COMPACT_ALIGN - ref.shape[1]
        got_pad = out.detach()[:, ref.shape[1]:].cpu().numpy()
        assert got_pad.shape[1] == pad and (got_pad == 0).all()
        out = out[:, : ref.shape[1]]
    emb = OE.embedding_lookup(w, ids, so)
    x = np.concatenate([emb, dense[:, None]], 1)
    scale = np.concatenate([_pair_scale(x, False, True), np.abs(dense)], 1)
    if compact:
        scale = scale[:, keep_cols]
    assert_close_rel(out.detach().cpu().numpy(), ref, RTOL, scale, "fwd")
    g = rng.standard_normal(ref.shape).astype(np.float32)
    out.backward(torch.from_numpy(g).to(DEV))
    if compact:
        gfull = np.zeros((B, F * F + D), np.float32)
        gfull[:, keep_cols] = g
        g = gfull
    ge_ref, gd_ref = O.dlrm_interaction_bwd(w, ids, dense, g, so)
    got_ids, got_rows = t.take_grad()
    np.testing.assert_array_equal(got_ids.cpu().numpy(), ids.reshape(-1))
    gscale = np.abs(g).max() * np.sqrt((x.astype(np.float64) ** 2).sum(-1)).max() * 2
    assert_close_rel(got_rows.cpu().numpy(), ge_ref, RTOL, gscale, "grad_emb")
    assert_close_rel(dt.grad.cpu().numpy(), gd_ref, RTOL, gscale, "grad_dense")


@pytest.mark.parametrize("F,D", [(26, 16), (3, 7), (26, 128)])
def test_fm(F, D, rng):
    B = 129
    e = rng.standard_normal((B, F, D)).astype(np.float32)
    et = torch.from_numpy(e).to(DEV).requires_grad_(True)
    out = fm_interaction(et)
    scale = (np.abs(e).sum(1) ** 2).sum(-1)
    assert_close_rel(out.detach().cpu().numpy(), O.fm(e), RTOL, scale, "fm fwd")
    g = rng.standard_normal(B).astype(np.float32)
    out.backward(torch.from_numpy(g).to(DEV))
    gscale = np.abs(g)[:, None, None] * np.abs(e).sum(1, keepdims=True)
    assert_close_rel(et.grad.cpu().numpy(), O.fm_bwd(e, g), RTOL, gscale, "fm bwd")


def test_dlrm_model_compact_equals_reference_layout(rng):
    from recommender_amd.ctr.model import DLRM

    S, D, B, V = 26, 32, 256, 5000
    g = torch.Generator(device=DEV)
    g.manual_seed(0)
    m1 = DLRM([64, D], [64, 1], D, V, S, 13, device=DEV, generator=g, compact=False)
    m2 = DLRM([64, D], [64, 1], D, V, S, 13, device=DEV, compact=True)
    m2.load_state_dict(m1.state_dict())
    m2.embedding_layer.weight.copy_(m1.embedding_layer.weight)
    x = {"cat_features": torch.from_numpy(rng.integers(0, V, (B, S))).to(DEV),
         "int_features": torch.from_numpy(rng.standard_normal((B, 13)).astype(np.float32)).to(DEV)}
    p1, p2 = m1(x), m2(x)
    assert_close_rel(p2.detach().cpu().numpy(), p1.detach().cpu().numpy(), 1e-5, 1e-3, "logits")
    p1.sum().backward()
    p2.sum().backward()
    k1 = m1.top_mlp.mlp[0].kernel.grad.cpu().numpy()
    k2 = m2.top_mlp.mlp[0].kernel.grad.cpu().numpy()
    assert_close_rel(k2, k1, 1e-5, np.abs(k1).max() * 1e-2, "top kernel grad")
    F = S + 1
    zero_rows = np.setdiff1d(np.arange(F * F + D), m2.compact_rows.cpu().numpy())
    assert (k2[zero_rows] == 0).all() and (k1[zero_rows] == 0).all()
    (i1, r1), (i2, r2) = m1.embedding_layer.take_grad(), m2.embedding_layer.take_grad()
    assert_close_rel(r2.cpu().numpy(), r1.cpu().numpy(), 1e-5, np.abs(r1.cpu().numpy()).max() * 1e-2, "emb grad")


@pytest.mark.parametrize("reduction", ["none", "sum", "mean"])
def test_bce_fused(reduction, rng):
    from oracle.ctr import bce, bce_grad
    from recommender_amd.functional import binary_crossentropy

    n = 10_007
    p = rng.random(n).astype(np.float32)
    p[:5] = [0.0, 1.0, 1e-9, 1 - 1e-9, 0.5]
    y = (rng.random(n) < 0.3).astype(np.float32)
    pt = torch.from_numpy(p).to(DEV).requires_grad_(True)
    out = binary_crossentropy(torch.from_numpy(y).to(DEV), pt, reduction=reduction)
    ref = bce(y, p).astype(np.float64)
    ref = {"none": ref, "sum": ref.sum(), "mean": ref.mean()}[reduction]
    assert_close_rel(out.detach().cpu().numpy(), ref, 1e-5, 0.0, "bce")
    g = torch.ones_like(out)
    out.backward(g)
    gref = bce_grad(y, p).astype(np.float64) * y.size  # oracle is for the mean
    if reduction == "mean":
        gref = gref / n
    assert_close_rel(pt.grad.cpu().numpy(), gref, 1e-5, 0.0, "bce grad")


@pytest.mark.parametrize("act", [None, "relu", "sigmoid"])
@pytest.mark.parametrize("overlap", [False, True])
def test_dense_layer_grads(act, overlap, rng):
    """Dense (Keras layout) forward/backward with the fused activation+bias epilogue and the
    split-K weight gradient vs torch fp32 autograd."""
    from recommender_amd.nn import Dense, overlapped_weight_grads

    B, fi, fo = 16384, 96, 40
    layer = Dense(fo, act, in_features=fi, device=DEV)
    x = torch.from_numpy(rng.standard_normal((B, fi)).astype(np.float32)).to(DEV).requires_grad_(True)
    k_ref = layer.kernel.detach().clone().requires_grad_(True)
    b_ref = layer.bias.detach().clone().requires_grad_(True)
    x_ref = x.detach().clone().requires_grad_(True)
    z = x_ref @ k_ref + b_ref
    y_ref = {None: z, "relu": torch.relu(z), "sigmoid": torch.sigmoid(z)}[act]
    g = torch.from_numpy(rng.standard_normal((B, fo)).astype(np.float32)).to(DEV)
    y_ref.backward(g)
    if overlap:
        with overlapped_weight_grads():
            y = layer(x)
            y.backward(g)
    else:
        y = layer(x)
        y.backward(g)
    torch.cuda.synchronize()
    for got, ref, name in ((y, y_ref, "y"), (x.grad, x_ref.grad, "dx"), (layer.kernel.grad, k_ref.grad, "dk"),
                           (layer.bias.grad, b_ref.grad, "db")):
        r = ref.detach().cpu().numpy()
        assert_close_rel(got.detach().cpu().numpy(), r, 1e-4, np.abs(r).max(), name)
