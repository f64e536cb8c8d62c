"""GPU parity: DIEN recurrent kernels (GRU reset_after, AUGRU, attention) forward AND backward
vs a plain-torch fp32 reference with explicit time loops (autograd for the gradients), with
right-padded masks like dien/data_loader.py:44,48; then the whole DIEN model forward."""
import numpy as np
import pytest
import torch

from oracle import dien as OD
from recommender_amd.dien.layers import GRU, DIENAttention, InterestEvolve
from tests.conftest import assert_close_rel

pytestmark = pytest.mark.gpu
DEV = "cuda"
RTOL = 2e-5


ref_gru, ref_augru, ref_att = OD.gru, OD.augru, OD.attention


def make_mask(rng, B, T):
    lens = np.clip(2 + rng.geometric(0.1, B), 2, T)
    return torch.from_numpy(np.arange(T)[None, :] < lens[:, None]).to(DEV)


def _close(got, ref, name):
    r = ref.detach().cpu().numpy()
    assert_close_rel(got.detach().cpu().numpy(), r, RTOL, np.abs(r).max() + 1e-30, name)


@pytest.mark.parametrize("H,X,B,T", [(36, 36, 96, 23), (16, 8, 96, 23), (64, 20, 96, 23),
                                     (36, 36, 512, 100)])
def test_gru_fwd_bwd(H, X, B, T, rng):
    g = torch.Generator(device="cpu")
    g.manual_seed(0)
    gru = GRU(H, X, device=DEV, generator=g)
    with torch.no_grad():
        gru.bias.normal_(0, 0.3)
    mask = make_mask(rng, B, T)
    x = torch.from_numpy(rng.standard_normal((B, T, X)).astype(np.float32)).to(DEV).requires_grad_(True)
    out = gru(x, mask)
    W, U, bias = (p.detach().clone().requires_grad_(True) for p in (gru.kernel, gru.recurrent_kernel, gru.bias))
    xr = x.detach().clone().requires_grad_(True)
    ref = ref_gru(xr, W, U, bias, mask)
    _close(out, ref, "gru out")
    gout = torch.from_numpy(rng.standard_normal((B, T, H)).astype(np.float32)).to(DEV)
    gout = gout * mask.unsqueeze(-1)
    out.backward(gout)
    ref.backward(gout)
    for got, r, n in ((x.grad, xr.grad, "dx"), (gru.kernel.grad, W.grad, "dW"),
                      (gru.recurrent_kernel.grad, U.grad, "dU"), (gru.bias.grad, bias.grad, "db")):
        _close(got, r, n)


@pytest.mark.parametrize("H,B,T", [(36, 80, 19), (24, 80, 19), (36, 512, 100)])
def test_augru_fwd_bwd(H, B, T, rng):
    X = H
    ev = InterestEvolve(H, X, device=DEV)
    c = ev.augru
    with torch.no_grad():
        for d in (c.update_gate, c.reset_gate, c.hidden_layer):
            d.bias.normal_(0, 0.2)
    mask = make_mask(rng, B, T)
    x = torch.from_numpy(rng.standard_normal((B, T, X)).astype(np.float32)).to(DEV).requires_grad_(True)
    a = torch.from_numpy(rng.random((B, T, 1)).astype(np.float32)).to(DEV).requires_grad_(True)
    out = ev((x, a), mask=mask)
    params = [p.detach().clone().requires_grad_(True) for p in
              (c.update_gate.kernel, c.update_gate.bias, c.reset_gate.kernel, c.reset_gate.bias,
               c.hidden_layer.kernel, c.hidden_layer.bias)]
    xr = x.detach().clone().requires_grad_(True)
    ar = a.detach().clone().requires_grad_(True)
    ref = ref_augru(xr, ar, *params, mask)
    _close(out, ref, "augru out")
    g = torch.from_numpy(rng.standard_normal((B, H)).astype(np.float32)).to(DEV)
    out.backward(g)
    ref.backward(g)
    _close(x.grad, xr.grad, "dx")
    _close(a.grad * mask.unsqueeze(-1), ar.grad * mask.unsqueeze(-1), "datt")
    for got, r, n in zip((c.update_gate.kernel.grad, c.update_gate.bias.grad, c.reset_gate.kernel.grad,
                          c.reset_gate.bias.grad, c.hidden_layer.kernel.grad, c.hidden_layer.bias.grad),
                         [p.grad for p in params], ["dKu", "dbu", "dKr", "dbr", "dKh", "dbh"]):
        _close(got, r, n)


def test_augru_zero_attention_keeps_state(rng):
    """Known answer: with a = 0 the AUGRU never moves its (zero) initial state."""
    ev = InterestEvolve(36, 36, device=DEV)
    x = torch.from_numpy(rng.standard_normal((8, 10, 36)).astype(np.float32)).to(DEV)
    out = ev((x, torch.zeros(8, 10, 1, device=DEV)), mask=torch.ones(8, 10, dtype=torch.bool, device=DEV))
    assert (out == 0).all()


@pytest.mark.parametrize("T", [100, 7, 130])
def test_attention_fwd_bwd(T, rng):
    B, H, Xt = 64, 36, 36
    att = DIENAttention(H, Xt, device=DEV)
    mask = make_mask(rng, B, T)
    hs = torch.from_numpy(rng.standard_normal((B, T, H)).astype(np.float32)).to(DEV).requires_grad_(True)
    tg = torch.from_numpy(rng.standard_normal((B, 1, Xt)).astype(np.float32)).to(DEV).requires_grad_(True)
    a = att((tg, hs), mask=mask)
    K = att.kernel.detach().clone().requires_grad_(True)
    hr, tr = hs.detach().clone().requires_grad_(True), tg.detach().clone().requires_grad_(True)
    ref = ref_att(tr, hr, K, mask)
    _close(a, ref, "scores")
    g = torch.from_numpy(rng.standard_normal((B, T, 1)).astype(np.float32)).to(DEV)
    a.backward(g)
    ref.backward(g)
    _close(hs.grad, hr.grad, "dhs")
    _close(tg.grad, tr.grad, "dtarget")
    _close(att.kernel.grad, K.grad, "dK")


def test_dien_model_forward_and_train_step(rng):
    from recommender_amd.dien import DIEN
    from recommender_amd.dien.train import DIENStep, synthetic_batch

    g = torch.Generator(device=DEV)
    g.manual_seed(2)
    m = DIEN(36, 36, item_vocab_size=3001, item_embedding_size=18, cat_vocab_size=81,
             cat_embedding_size=18, mlp_units=[200, 80, 1], device=DEV, generator=g)
    feats, label = synthetic_batch(np.random.default_rng(1), 128, 50, 3001, 81)
    feats = {k: torch.from_numpy(v).to(DEV) for k, v in feats.items()}
    prob, aux = m(feats)
    # reference forward from the same parameters
    with torch.no_grad():
        mask = feats["pos_his_item"] != 0
        def emb(i, c):
            return torch.cat([m.item_embedding.weight[i.long()], m.cat_embedding.weight[c.long()]], -1)
        tgt = emb(feats["target_item"], feats["target_cat"])
        pos = emb(feats["pos_his_item"], feats["pos_his_cat"])
        gru = m.interest_extract_layer.gru
        hid = ref_gru(pos, gru.kernel, gru.recurrent_kernel, gru.bias, mask)
        sc = ref_att(tgt, hid, m.attention.kernel, mask)
        c = m.interest_evolve.augru
        rep = ref_augru(hid, sc, c.update_gate.kernel, c.update_gate.bias, c.reset_gate.kernel,
                        c.reset_gate.bias, c.hidden_layer.kernel, c.hidden_layer.bias, mask)
        x = torch.cat([tgt.squeeze(1), rep], -1)
        x = _mlp_ref(m, x, False)
    _close(prob, x, "dien prob")
    step = DIENStep(m)
    lab = torch.from_numpy(label).to(DEV)
    l0 = float(step(feats, lab)[0])
    for _ in range(5):
        l1 = float(step(feats, lab)[0])
    assert l1 < l0


def _dien_models(kind):
    from recommender_amd.dien import DIEN, DIN, BaseModel

    g = torch.Generator(device=DEV)
    g.manual_seed(2)
    kw = dict(item_vocab_size=3001, item_embedding_size=18, cat_vocab_size=81,
              cat_embedding_size=18, mlp_units=[200, 80, 1], device=DEV, generator=g)
    if kind == "DIEN":
        return DIEN(36, 36, **kw)
    return (DIN if kind == "DIN" else BaseModel)(**kw)


def _emb(m, i, c):
    return torch.cat([m.item_embedding.weight[i.long()], m.cat_embedding.weight[c.long()]], -1)


def _mlp_ref(m, x, training):
    bn = m.mlp.bn
    if training:
        mean, var = x.mean(0), x.var(0, unbiased=False)
    else:
        mean, var = bn.moving_mean, bn.moving_variance
    x = OD.batch_norm_inference(x, mean, var, bn.gamma, bn.beta, bn.epsilon)
    return OD.dense_stack(x, [(l.kernel, l.bias, "relu") for l in m.mlp.mlp[:-1]]
                          + [(m.mlp.mlp[-1].kernel, m.mlp.mlp[-1].bias, "sigmoid")])


@pytest.mark.parametrize("training", [False, True])
@pytest.mark.parametrize("kind", ["BASE", "DIN"])
def test_base_din_forward_vs_oracle(kind, training):
    """BASE (masked history mean, dien/layers.py:5-17) and DIN (unnormalised local activation,
    dien/layers.py:34-59) through their MLP (BatchNormalization in the mode `training` selects,
    dien/model.py:30,47) against oracle/dien.py, 2e-5 relative."""
    from recommender_amd.dien.train import synthetic_batch

    m = _dien_models(kind)
    feats, _ = synthetic_batch(np.random.default_rng(1), 256, 50, 3001, 81, negatives=False)
    feats = {k: torch.from_numpy(v).to(DEV) for k, v in feats.items()}
    with torch.no_grad():
        prob = m(feats, training=training)
        mask = feats["pos_his_item"] != 0
        tgt = _emb(m, feats["target_item"], feats["target_cat"])
        his = _emb(m, feats["pos_his_item"], feats["pos_his_cat"])
        if kind == "BASE":
            rep = OD.his_average(his, mask)
        else:
            lau = m.local_activation_unit
            rep = OD.local_activation(tgt, his, mask, [(lau.layer_1.kernel, lau.layer_1.bias, "sigmoid"),
                                                       (lau.layer_2.kernel, lau.layer_2.bias, "sigmoid"),
                                                       (lau.layer_3.kernel, lau.layer_3.bias, None)])
        ref = _mlp_ref(m, torch.cat([tgt.squeeze(1), rep], -1), training)
    _close(prob, ref, f"{kind} prob")


def test_base_empty_history_is_nan():
    """The reference's masked mean divides by Σmask: an all-padding history gives 0/0 = NaN
    (dien/layers.py:14-16), and BASE's probability for that example is NaN; the others stay
    finite."""
    from recommender_amd.dien.train import synthetic_batch

    m = _dien_models("BASE")
    feats, _ = synthetic_batch(np.random.default_rng(1), 16, 20, 3001, 81, negatives=False)
    feats["pos_his_item"][3] = 0
    feats["pos_his_cat"][3] = 0
    feats = {k: torch.from_numpy(v).to(DEV) for k, v in feats.items()}
    with torch.no_grad():
        prob = m(feats).cpu().numpy()
        mask = feats["pos_his_item"] != 0
        his = _emb(m, feats["pos_his_item"], feats["pos_his_cat"])
        ref = OD.his_average(his, mask).cpu().numpy()
    assert np.isnan(ref[3]).all() and np.isnan(prob[3]).all()
    assert np.isfinite(np.delete(prob, 3, 0)).all()


def test_dien_aux_loss_vs_oracle():
    """DIEN's auxiliary loss (dien/layers.py:89-108) per example against oracle/dien.py from
    the model's own GRU states: 1e-5 relative (floor 1e-3 of the largest)."""
    from recommender_amd.dien.train import synthetic_batch

    m = _dien_models("DIEN")
    feats, _ = synthetic_batch(np.random.default_rng(3), 512, 100, 3001, 81)
    feats = {k: torch.from_numpy(v).to(DEV) for k, v in feats.items()}
    with torch.no_grad():
        _, aux = m(feats)
        mask = feats["pos_his_item"] != 0
        pos = _emb(m, feats["pos_his_item"], feats["pos_his_cat"])
        neg = _emb(m, feats["neg_his_item"], feats["neg_his_cat"])
        gr = m.interest_extract_layer.gru
        hid = OD.gru(pos, gr.kernel, gr.recurrent_kernel, gr.bias, mask)
        an = m.interest_extract_layer.auxiliary_net.layers
        ref = OD.aux_loss(hid, pos, neg, mask, [(an[0].kernel, an[0].bias, "sigmoid"),
                                                (an[1].kernel, an[1].bias, "sigmoid"),
                                                (an[2].kernel, an[2].bias, None)])
    assert aux.shape == ref.shape == (512,)
    assert_close_rel(aux.cpu().numpy(), ref.cpu().numpy(), 1e-5, float(ref.abs().max()) * 1e-3, "aux")


@pytest.mark.parametrize("H,B,L,kind", [(36, 512, 100, "post"), (36, 64, 37, "random"),
                                        (36, 48, 17, "post"), (16, 96, 50, "random")])
def test_fused_aux_loss_fwd_bwd_vs_oracle(H, B, L, kind, rng):
    """The fused aux-net kernels (csrc/dien_aux.hip) forward and backward against
    oracle/dien.aux_loss under torch autograd: aux and every input / parameter gradient within
    2e-5 of (|value| + the tensor's largest value) — fp32 sums over different row orders. Masks:
    post-padded (dien/data_loader.py) or arbitrary; L = 17 puts the last row on a tile edge.
    One example has a length-1 history: its aux (0 / 0) and every parameter gradient are NaN,
    as the reference's."""
    from recommender_amd.dien.layers import InterestExtract

    g = torch.Generator(device=DEV).manual_seed(7)
    ie = InterestExtract(H, H, device=DEV, generator=g)
    an = ie.auxiliary_net.layers
    with torch.no_grad():
        for l in an:
            l.bias.copy_(torch.randn(l.bias.shape, generator=g, device=DEV) * 0.2)
    if kind == "post":
        mask = make_mask(rng, B, L)
    else:
        mask = torch.from_numpy(rng.random((B, L)) < 0.3).to(DEV)
        mask[:, 1] = True
    x = [torch.from_numpy(rng.standard_normal((B, L, H)).astype(np.float32) * 0.5).to(DEV)
         for _ in range(3)]
    daux = torch.from_numpy(rng.standard_normal(B).astype(np.float32)).to(DEV)
    assert ie._fused_aux_ready(x[0], x[1])
    got_in = [t.clone().requires_grad_(True) for t in x]
    aux = ie.compute_auxiliary_loss(tuple(got_in), mask=mask)
    aux.backward(daux)
    ref_in = [t.clone().requires_grad_(True) for t in x]
    params = [p.detach().clone().requires_grad_(True) for l in an for p in (l.kernel, l.bias)]
    layers = [(params[0], params[1], "sigmoid"), (params[2], params[3], "sigmoid"),
              (params[4], params[5], None)]
    ref = OD.aux_loss(ref_in[0], ref_in[1], ref_in[2], mask, layers)
    ref.backward(daux)
    _close(aux, ref, "aux")
    for got, r, n in zip([t.grad for t in got_in] + [p.grad for l in an for p in (l.kernel, l.bias)],
                         [t.grad for t in ref_in] + [p.grad for p in params],
                         ["dhidden", "dpos", "dneg", "dW1", "db1", "dW2", "db2", "dW3", "db3"]):
        _close(got, r, n)
    # a length-1 history: aux = 0 / 0 and NaN parameter gradients, as the reference
    mask1 = mask.clone()
    mask1[5, 1:] = False
    for p in ie.parameters():
        p.grad = None
    aux1 = ie.compute_auxiliary_loss(tuple(t.clone() for t in x), mask=mask1)
    assert torch.isnan(aux1[5]) and torch.isfinite(aux1[torch.arange(B, device=DEV) != 5]).all()
    aux1.backward(daux)
    assert torch.isnan(an[0].kernel.grad).all() and torch.isnan(an[2].bias.grad).all()


@pytest.mark.parametrize("B", [4096, 1000, 1])
@pytest.mark.parametrize("training", [True, False])
def test_batch_norm_kernels_vs_float64(B, training):
    """BatchNormalization on the fused kernels (csrc/batchnorm.hip) against a float64 evaluation
    of the Keras formulas: output, moving mean / variance after the update (training) or
    untouched (inference), and dx / dgamma / dbeta; ragged last chunk (B = 1000) and B = 1."""
    from recommender_amd.dien.layers import BatchNormalization

    g = torch.Generator(device=DEV).manual_seed(B + int(training))
    C = 72
    bn = BatchNormalization(C, device=DEV)
    bn.gamma.data = torch.rand(C, device=DEV, generator=g) + 0.5
    bn.beta.data = torch.randn(C, device=DEV, generator=g)
    bn.moving_mean.copy_(torch.randn(C, device=DEV, generator=g))
    bn.moving_variance.copy_(torch.rand(C, device=DEV, generator=g) + 0.5)
    mm0, mv0 = bn.moving_mean.clone().double(), bn.moving_variance.clone().double()
    x = (torch.randn(B, C, device=DEV, generator=g) * 3 + 1).requires_grad_()
    up = torch.randn(B, C, device=DEV, generator=g)
    y = bn(x, training=training)
    (y * up).sum().backward()
    x64 = x.detach().double().requires_grad_()
    ga64 = bn.gamma.detach().double().requires_grad_()
    be64 = bn.beta.detach().double().requires_grad_()
    if training:
        mean, var = x64.mean(0), x64.var(0, unbiased=False)
    else:
        mean, var = mm0, mv0
    y64 = (x64 - mean) * torch.rsqrt(var + 1e-3) * ga64 + be64
    (y64 * up.double()).sum().backward()
    _close(y, y64, "bn output")
    _close(x.grad, x64.grad, "bn dx")
    _close(bn.gamma.grad, ga64.grad, "bn dgamma")
    _close(bn.beta.grad, be64.grad, "bn dbeta")
    if training:
        d = 1.0 - 0.99
        _close(bn.moving_mean, mm0 - (mm0 - mean.detach()) * d, "moving mean")
        _close(bn.moving_variance, mv0 - (mv0 - var.detach()) * d, "moving variance")
    else:
        assert torch.equal(bn.moving_mean.double(), mm0)
        assert torch.equal(bn.moving_variance.double(), mv0)


def test_valid_rows_cache_follows_in_place_refill():
    """The valid-row list kept on a uint8 mask is rebuilt when the same buffer is refilled in
    place (a static step's inputs, an eval loop): never the previous batch's rows."""
    from recommender_amd.dien.layers import _valid_rows

    g = torch.Generator(device=DEV).manual_seed(5)
    m = (torch.rand(64, 20, device=DEV, generator=g) < 0.3).to(torch.uint8)
    idx, cnt = _valid_rows(m)
    ref = torch.nonzero(m.reshape(-1)).reshape(-1).to(torch.int32)
    assert int(cnt) == ref.numel() and torch.equal(idx[: ref.numel()], ref)
    m.copy_((torch.rand(64, 20, device=DEV, generator=g) < 0.6).to(torch.uint8))
    idx2, cnt2 = _valid_rows(m)
    ref2 = torch.nonzero(m.reshape(-1)).reshape(-1).to(torch.int32)
    assert int(cnt2) == ref2.numel() and torch.equal(idx2[: ref2.numel()], ref2)
