"""rs_dlrm_train_step_fwd_unit (the chunked train kernel: unit gradient rows U + per-example G)
against rs_dlrm_train_step_fwd_scaled (dlrm_train_pipe: G·U rows) on the same inputs: y and the
batch sums bit-identical (same Z products, same per-lane accumulation order), G[b]·U[p] (fmul_rn,
what rs_embedding_apply_scaled forms) equal to the G·U rows. Slot counts on both sides of 16
(the dense row then sits in the first or second 16-row block of the Uᵀ product), D 128 / 64,
int32 / int64 ids, out-of-range ids (zero row + flag), a batch that leaves waves empty."""
import numpy as np
import pytest
import torch

from recommender_amd import _lib as L

pytestmark = pytest.mark.gpu
DEV = "cuda"
NI = 13


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


def _run(unit, table, ids, offs, dense, xin, label, q, c, S, D):
    B = ids.shape[0]
    V = table.shape[0]
    y = torch.empty(B, device=DEV)
    rows = torch.full((B * S, D), float("nan"), device=DEV)
    sums = torch.empty(512 + 2 + NI * D + D, device=DEV)
    ws_n = L.lib().rs_dlrm_train_workspace_size(B)
    ws = torch.empty(ws_n, dtype=torch.uint8, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    common = (L.ptr(table), V, D, L.ptr(ids), L.id_dtype_code(ids), S, L.ptr(offs), L.ptr(dense), L.ptr(xin), NI,
              L.ptr(label), B, L.ptr(q), L.ptr(c), 1e-7, 1.0 / B, L.ptr(y))
    G = None
    if unit:
        G = torch.full((B,), float("nan"), device=DEV)
        L.call("rs_dlrm_train_step_fwd_unit", *common, L.ptr(rows), L.ptr(G), L.ptr(sums),
               L.ptr(ws), ws_n, L.ptr(err), L.stream_ptr(table.device))
    else:
        L.call("rs_dlrm_train_step_fwd_scaled", *common, L.ptr(rows), L.ptr(sums), L.ptr(ws), ws_n,
               L.ptr(err), L.stream_ptr(table.device))
    torch.cuda.synchronize()
    return y, rows, G, sums, int(err.item())


@pytest.mark.parametrize("B,S,D,id64,oob", [
    (4096, 26, 128, False, False),
    (1000, 26, 128, True, True),
    (777, 8, 128, False, True),
    (2048, 15, 128, True, False),
    (3000, 26, 64, False, False),
    (513, 12, 64, True, True),
])
def test_unit_rows_match_scaled_rows(B, S, D, id64, oob):
    V = 20_000 * S
    args = _inputs(B, S, D, V, id64, seed=B + S, oob=oob)
    y0, r0, _, s0, e0 = _run(False, *args, S, D)
    y1, u1, G, s1, e1 = _run(True, *args, S, D)
    assert e0 == e1 and (e0 != 0) == oob
    assert torch.equal(y0, y1)
    assert torch.equal(s0, s1)
    assert torch.isfinite(G).all() and torch.isfinite(u1).all()
    scaled = G.repeat_interleave(S)[:, None] * u1  # fp32 multiply, round to nearest (fmul_rn)
    diff = (scaled - r0).abs()
    tol = 2e-6 * r0.abs().amax(dim=1, keepdim=True) + 1e-30
    n_exact = int((scaled == r0).all(dim=1).sum())
    print(f"rows bit-identical: {n_exact} / {B * S}, max |diff| / row max "
          f"{float((diff / tol).max()) * 2e-6:.3e}")
    assert bool((diff <= tol).all())
