"""rs_dlrm_train_step_fwd_unit (the chunked train kernel of the production DLRM step: gather,
Z = X·Xᵀ, the composed top-MLP head, Keras BCE, G, the unit gradient rows U = (M + Mᵀ)·X and the
batch sums of the factored MLP backward) against a float64 torch restatement of the same
quantities (ctr/model.py:45-57 with the head composed, ctr/layers.py:23-43). Every product is
bounded per element by its magnitude: |got − ref| ≤ 1e-5 · Σ|terms| (the split-bf16 MFMA keeps
fp32 accuracy relative to that bound). Slot counts on both sides of 16 (the dense
row then sits in the first or second 16-row block of the Uᵀ product), D 128 / 64, int32 / int64
ids, out-of-range ids (zero row + flag), a batch that leaves waves empty."""
import numpy as np
import pytest
import torch

from recommender_amd import _lib as L

pytestmark = pytest.mark.gpu
DEV = "cuda"
NI = 13
EPS = 1e-7


def _inputs(B, S, D, V, id64, seed, oob=False):
    g = torch.Generator(device="cpu").manual_seed(seed)
    table = (torch.randn(V, D, generator=g) * 0.5).to(DEV)
    ids = torch.randint(0, V // S, (B, S), generator=g)
    if oob:
        ids[::7, 3 % S] = V  # beyond every slot's range
        ids[::11, 0] = -1
    ids = ids.to(torch.int64 if id64 else torch.int32).to(DEV).contiguous()
    offs = (torch.arange(S + 1, dtype=torch.int64) * (V // S)).to(DEV)
    dense = torch.randn(B, D, generator=g).to(DEV)
    xin = torch.rand(B, NI, generator=g).to(DEV)
    label = (torch.rand(B, generator=g) < 0.3).float().to(DEV)
    F = S + 1
    q = (torch.randn(F * (F - 1) // 2 + D, generator=g) * 0.05).to(DEV)
    c = torch.tensor([0.1]).to(DEV)
    return table, ids, offs, dense, xin, label, q, c


def _run(table, ids, offs, dense, xin, label, q, c, S, D):
    B = ids.shape[0]
    V = table.shape[0]
    y = torch.empty(B, device=DEV)
    rows = torch.full((B * S, D), float("nan"), device=DEV)
    sums = torch.empty(512 + 2 + NI * D + D, device=DEV)
    ws_n = L.lib().rs_dlrm_train_workspace_size(B)
    ws = torch.empty(ws_n, dtype=torch.uint8, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    G = torch.full((B,), float("nan"), device=DEV)
    L.call("rs_dlrm_train_step_fwd_unit", L.ptr(table), V, D, L.ptr(ids), L.id_dtype_code(ids), S,
           L.ptr(offs), L.ptr(dense), L.ptr(xin), NI, L.ptr(label), B, L.ptr(q), L.ptr(c), EPS,
           1.0 / B, L.ptr(y), L.ptr(rows), L.ptr(G), L.ptr(sums), L.ptr(ws), ws_n, L.ptr(err),
           L.stream_ptr(table.device))
    torch.cuda.synchronize()
    return y, rows, G, sums, int(err.item())


def _reference(table, ids, offs, dense, xin, label, q, c, S, D):
    """float64: y, G, the unit rows U[b, s] and the batch sums; plus the magnitude bound of each
    (the same sums over |terms|)."""
    f = torch.float64
    B = ids.shape[0]
    F = S + 1
    idl = ids.long()
    lo, hi = offs[:-1][None, :], offs[1:][None, :]
    ok = (idl >= 0) & (idl < hi - lo)
    rowi = torch.where(ok, lo + idl, torch.zeros_like(idl))
    X = torch.cat([table.to(f)[rowi] * ok[..., None], dense.to(f)[:, None, :]], 1)  # [B, F, D]
    iu = torch.triu_indices(F, F, 1, device=DEV)
    nz = iu.shape[1]
    qp, qd = q[:nz].to(f), q[nz:].to(f)
    Z = X @ X.transpose(1, 2)
    Zm = (X.abs() @ X.abs().transpose(1, 2))
    z = Z[:, iu[0], iu[1]]
    zm = Zm[:, iu[0], iu[1]]
    h = z @ qp + dense.to(f) @ qd + float(c)
    hm = zm @ qp.abs() + dense.to(f).abs() @ qd.abs() + abs(float(c))
    p = torch.sigmoid(h)
    lb = label.to(f)
    pc = p.clamp(EPS, 1 - EPS)
    loss = -(lb * torch.log(pc + EPS) + (1 - lb) * torch.log(1 - pc + EPS))
    inside = (p >= EPS) & (p <= 1 - EPS)
    dbce = -(lb / (pc + EPS)) + (1 - lb) / ((1 - pc) + EPS)
    G = torch.where(inside, dbce / B, torch.zeros_like(p)) * p * (1 - p)
    M = torch.zeros(F, F, dtype=f, device=DEV)
    M[iu[0], iu[1]] = qp
    Sm = M + M.T
    U = Sm[None] @ X                                      # [B, F, D]
    Um = Sm.abs()[None] @ X.abs()
    zrow = torch.cat([z, dense.to(f)], 1)
    zrm = torch.cat([zm, dense.to(f).abs()], 1)
    gbot = torch.where(dense > 0, G[:, None] * (U[:, S] + qd[None]), torch.zeros_like(U[:, S]))
    # error carried into G by h's (|dG/dh| = y(1-y)/B <= 1/(4B)) on top of G's own magnitude
    gm = G.abs() + hm / (4 * B)
    gbm = torch.where(dense > 0, gm[:, None] * (Um[:, S] + qd.abs()[None]),
                      torch.zeros_like(U[:, S]))
    sums = {"A_top": (zrow * G[:, None]).sum(0), "s_top": G.sum(), "loss": loss.sum(),
            "A_bot": xin.to(f).T @ gbot, "s_bot": gbot.sum(0)}
    mags = {"A_top": (zrm * gm[:, None]).sum(0), "s_top": gm.sum(),
            "loss": (dbce.abs() * 0.25 * hm).sum() + 0.1 * loss.abs().sum(),
            "A_bot": xin.to(f).abs().T @ gbm, "s_bot": gbm.sum(0)}
    return p, hm, G, U[:, :S], Um[:, :S], sums, mags, nz, bool((~ok).any())


def _close(got, ref, mag, msg, rel=1e-5):
    got = got.double()
    tol = rel * mag + 1e-30
    err = (got - ref).abs()
    bad = ~(err <= tol)
    assert not bool(bad.any()), (f"{msg}: {int(bad.sum())} / {bad.numel()} off, max err/tol "
                                 f"{float((err / tol).max()):.3g}")


@pytest.mark.parametrize("B,S,D,id64,oob", [
    (4096, 26, 128, False, False),
    (1000, 26, 128, True, True),
    (777, 8, 128, False, True),
    (2048, 15, 128, True, False),
    (3000, 26, 64, False, False),
    (513, 12, 64, True, True),
])
def test_chunked_train_kernel_vs_float64(B, S, D, id64, oob):
    V = 20_000 * S
    args = _inputs(B, S, D, V, id64, seed=B + S, oob=oob)
    y, U, G, sums, err = _run(*args, S, D)
    p, hm, G64, U64, Um, s64, m64, nz, has_oob = _reference(*args, S, D)
    assert (err != 0) == has_oob == oob
    assert torch.isfinite(G).all() and torch.isfinite(U).all()
    # y = σ(h): |dy| <= |dh| / 4 (+ the sigmoid's own rounding, a few ulps of y)
    _close(y, p, 0.25 * hm + 0.03 * p, "y")
    _close(U.view(B, S, D), U64, Um, "unit rows")
    # G = y(1-y)·dL/dy = (y - label) / B inside the clip: h's error moves it by <= |dh| / (4B)
    dG = (G.double() - G64).abs()
    assert bool((dG <= 2e-6 * G64.abs() + 1e-5 * hm / (4 * B)).all()), float(dG.max())
    a = 512
    _close(sums[:nz + D], s64["A_top"], m64["A_top"], "A_top")
    assert bool((sums[nz + D:a] == 0).all())
    _close(sums[a], s64["s_top"], m64["s_top"], "s_top")
    _close(sums[a + 1], s64["loss"], m64["loss"], "loss")
    _close(sums[a + 2:a + 2 + NI * D].view(NI, D), s64["A_bot"], m64["A_bot"], "A_bot")
    _close(sums[a + 2 + NI * D:], s64["s_bot"], m64["s_bot"], "s_bot")
