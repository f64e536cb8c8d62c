"""rs_gemm_x3 (csrc/gemm.hip: fp32 GEMM on the bf16 matrix cores, each operand split into three
bf16 parts, six part products) against a float64 torch evaluation of the same product. Bound per
element: |got - ref| <= 4e-6 · Σ_k |a_mk||b_kn| (+ the same for the bias), i.e. ≈64 fp32 ulps of the
term magnitude — an fp32 fma chain of these lengths errs by far less than its worst case K·u; the
library fp32 GEMM (hipBLASLt) is held to the same bound on the same inputs as a control. All four
operand layouts (the Dense layer's forward ta 0 tb 0, dgrad ta 0 tb 1, wgrad ta 1 tb 0, and ta 1
tb 1), edge tiles (M, N, K not multiples of the 128 / 32 tiles), batches with strides, the
split-K fold, bias and relu / sigmoid epilogues."""
import pytest
import torch

from recommender_amd import _lib as L

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _op(t, trans):
    return t.transpose(-1, -2) if trans else t


def _run(A, B, M, N, K, ta, tb, batch, bias, act, splits):
    C = torch.full((batch, M, N), float("nan"), device=DEV)
    ws_n = L.lib().rs_gemm_x3_workspace_size(M, N, batch, splits)
    ws = torch.empty(max(ws_n, 1), dtype=torch.uint8, device=DEV)
    lda = A.shape[-1]
    ldb = B.shape[-1]
    L.call("rs_gemm_x3", ta, tb, M, N, K, L.ptr(A), lda, A[0].numel(), L.ptr(B), ldb,
           B[0].numel(), L.ptr(C), N, M * N, batch, L.ptr(bias),
           0 if bias is None else bias.shape[-1], act, splits, L.ptr(ws), ws.numel(),
           L.stream_ptr(torch.device(DEV)))
    torch.cuda.synchronize()
    return C


def _act(x, act):
    return torch.relu(x) if act == 1 else (torch.sigmoid(x) if act == 2 else x)


@pytest.mark.parametrize("M,N,K,ta,tb,batch,splits,act", [
    (4096, 360, 324, 0, 0, 1, 1, 1),      # ESMM tower layer 1 forward (relu)
    (4096, 324, 360, 0, 1, 1, 1, 0),      # its dgrad
    (324, 360, 8192, 1, 0, 1, 16, 0),     # its wgrad, split-K
    (1000, 200, 1604, 0, 0, 3, 1, 2),     # batched, edge tiles, sigmoid
    (132, 76, 36, 1, 1, 2, 1, 0),
    (260, 80, 4100, 1, 0, 2, 7, 1),       # batched split-K with a ragged last split
    (8, 4, 4, 0, 0, 1, 1, 0),
])
def test_gemm_x3_vs_float64(M, N, K, ta, tb, batch, splits, act):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    a_shape = (batch, K, M) if ta else (batch, M, K)
    b_shape = (batch, N, K) if tb else (batch, K, N)
    A = torch.randn(*a_shape, device=DEV, generator=g)
    B = torch.randn(*b_shape, device=DEV, generator=g) * 0.1
    bias = torch.randn(batch, N, device=DEV, generator=g)
    C = _run(A, B, M, N, K, ta, tb, batch, bias, act, splits)
    a64, b64 = _op(A, ta).double(), _op(B, tb).double()
    z64 = a64 @ b64 + bias.double()[:, None, :]
    mag = a64.abs() @ b64.abs() + bias.double().abs()[:, None, :]
    ref = _act(z64, act)
    # the activations' slopes are <= 1: the pre-activation bound carries over
    tol = 4e-6 * mag + 1e-30
    err = (C.double() - ref).abs()
    assert torch.isfinite(C).all()
    assert bool((err <= tol).all()), f"max err/tol {float((err / tol).max()):.3g}"
    # control: the library fp32 GEMM on the same inputs meets the same bound
    z32 = torch.baddbmm(bias[:, None, :], _op(A, ta), _op(B, tb))
    assert bool(((_act(z32, act).double() - ref).abs() <= tol).all())


def test_gemm_x3_rejects_unaligned_shapes():
    A = torch.zeros(1, 6, 6, device=DEV)
    with pytest.raises(L.RecsysError):
        _run(A, A, 6, 6, 6, 0, 0, 1, None, 0, 1)
