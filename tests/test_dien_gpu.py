"""GPU parity: DIEN recurrent kernels (GRU reset_after, AUGRU, attention) forward AND backward
vs a plain-torch fp32 reference with explicit time loops (autograd for the gradients), with
right-padded masks like dien/data_loader.py:44,48; then the whole DIEN model forward."""
import numpy as np
import pytest
import torch

from recommender_amd.dien.layers import GRU, DIENAttention, InterestEvolve
from tests.conftest import assert_close_rel

pytestmark = pytest.mark.gpu
DEV = "cuda"
RTOL = 2e-5


def ref_gru(x, W, U, bias, mask):
    B, T, X = x.shape
    H = U.shape[0]
    h = torch.zeros(B, H, device=x.device)
    outs = []
    for t in range(T):
        xw = x[:, t] @ W + bias[0]
        inner = h @ U + bias[1]
        z = torch.sigmoid(xw[:, :H] + inner[:, :H])
        r = torch.sigmoid(xw[:, H:2 * H] + inner[:, H:2 * H])
        hh = torch.tanh(xw[:, 2 * H:] + r * inner[:, 2 * H:])
        hn = z * h + (1 - z) * hh
        h = torch.where(mask[:, t:t + 1], hn, h)
        outs.append(h)
    return torch.stack(outs, 1)


def ref_augru(x, a, ku, bu, kr, br, kh, bh, mask):
    B, T, X = x.shape
    H = ku.shape[1]
    h = torch.zeros(B, H, device=x.device)
    for t in range(T):
        c = torch.cat([h, x[:, t]], -1)
        u = torch.sigmoid(c @ ku + bu)
        r = torch.sigmoid(c @ kr + br)
        hh = torch.tanh(torch.cat([x[:, t], r * h], -1) @ kh + bh)
        u = u * a[:, t]
        hn = u * hh + (1 - u) * h
        h = torch.where(mask[:, t:t + 1], hn, h)
    return h


def ref_att(target, hs, K, mask):
    s = (hs @ K) @ target.transpose(1, 2)
    s = s + (1.0 - mask.unsqueeze(-1).float()) * -1e9
    return torch.softmax(s, dim=1)


def make_mask(rng, B, T):
    lens = np.clip(2 + rng.geometric(0.1, B), 2, T)
    return torch.from_numpy(np.arange(T)[None, :] < lens[:, None]).to(DEV)


def _close(got, ref, name):
    r = ref.detach().cpu().numpy()
    assert_close_rel(got.detach().cpu().numpy(), r, RTOL, np.abs(r).max() + 1e-30, name)


@pytest.mark.parametrize("H,X", [(36, 36), (16, 8), (64, 20)])
def test_gru_fwd_bwd(H, X, rng):
    B, T = 96, 23
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


@pytest.mark.parametrize("H", [36, 24])
def test_augru_fwd_bwd(H, rng):
    B, T, X = 80, 19, H
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
        bn = m.mlp.bn
        x = (x - bn.moving_mean) * torch.rsqrt(bn.moving_variance + bn.epsilon) * bn.gamma + bn.beta
        for l in m.mlp.mlp:
            x = x @ l.kernel + l.bias
            x = l.activation(x) if l.activation is not None else x
    _close(prob, x, "dien prob")
    step = DIENStep(m)
    lab = torch.from_numpy(label).to(DEV)
    l0 = float(step(feats, lab)[0])
    for _ in range(5):
        l1 = float(step(feats, lab)[0])
    assert l1 < l0
