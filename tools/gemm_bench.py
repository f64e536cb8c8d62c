"""A/B of rs_gemm_x3 (split-bf16 MFMA, fp32-accurate) against the library fp32 GEMMs the Dense
layers use today (torch addmm / mm / baddbmm -> hipBLASLt, and recommender_amd.nn.wgrad's split-K
bmm), on the cfg4 layer shapes (B = 65 536): ESMM towers 324 -> 360 -> 200 -> 80 and MMOE's
experts 324 -> 8 x 200 -> 8 x 80. Prints one JSON line per (shape, product): both times in us and
the TFLOP/s of each. Run on the GPU box: python tools/gemm_bench.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from recommender_amd import _lib as L  # noqa: E402
from recommender_amd.nn import bwgrad, wgrad  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def auto_splits(M, N, K, batch=1):
    """split-K ranges so the grid has >= ~1024 blocks, each range >= 512 deep"""
    tiles = -(-M // 128) * -(-N // 128) * batch
    return max(1, min(K // 512, -(-1024 // tiles)))


def x3(ta, tb, M, N, K, A, B, C, batch=1, bias=None, act=0, splits=1, ws=None):
    lda, ldb = A.shape[-1], B.shape[-1]
    sA = A[0].numel() if batch > 1 else 0
    sB = B[0].numel() if batch > 1 else 0
    L.call("rs_gemm_x3", ta, tb, M, N, K, L.ptr(A), lda, sA, L.ptr(B), ldb, sB, L.ptr(C), N,
           M * N, batch, L.ptr(bias), N if bias is not None else 0, act, splits, L.ptr(ws),
           0 if ws is None else ws.numel(), L.stream_ptr(torch.device("cuda")))


def main():
    dev = torch.device("cuda")
    L.load()
    Bt = 65536
    out = []
    for fi, fo in ((324, 360), (360, 200), (200, 80), (324, 1600)):
        x = torch.randn(Bt, fi, device=dev)
        w = torch.randn(fi, fo, device=dev) * 0.05
        b = torch.randn(fo, device=dev)
        dz = torch.randn(Bt, fo, device=dev)
        y = torch.empty(Bt, fo, device=dev)
        dx = torch.empty(Bt, fi, device=dev)
        dw = torch.empty(fi, fo, device=dev)
        splits = auto_splits(fi, fo, Bt)
        ws = torch.empty(L.lib().rs_gemm_x3_workspace_size(fi, fo, 1, splits), dtype=torch.uint8,
                         device=dev)
        fl = 2.0 * Bt * fi * fo
        rows = [
            ("forward+bias+relu", lambda: torch.relu_(torch.addmm(b, x, w)),
             lambda: x3(0, 0, Bt, fo, fi, x, w, y, bias=b, act=1)),
            ("dgrad", lambda: dz @ w.t(), lambda: x3(0, 1, Bt, fi, fo, dz, w, dx)),
            ("wgrad", lambda: wgrad(x, dz), lambda: x3(1, 0, fi, fo, Bt, x, dz, dw, splits=splits,
                                                       ws=ws)),
        ]
        for name, lib, ours in rows:
            tl, to = timeit(lib), timeit(ours)
            out.append({"shape": f"{Bt}x{fi}->{fo}", "product": name, "stages": os.environ.get("RS_GEMM_STAGES", "1"), "library_us": round(tl, 1),
                        "x3_us": round(to, 1), "library_TF": round(fl / tl / 1e6, 1),
                        "x3_TF": round(fl / to / 1e6, 1), "speedup": round(tl / to, 2)})
            print(json.dumps(out[-1]), flush=True)
    # MMOE's batched expert layer: [8, B, 200] x [8, 200, 80]
    E = 8
    h = torch.randn(E, Bt, 200, device=dev)
    k = torch.randn(E, 200, 80, device=dev) * 0.05
    bb = torch.randn(E, 1, 80, device=dev)
    g = torch.randn(E, Bt, 80, device=dev)
    yb = torch.empty(E, Bt, 80, device=dev)
    dwb = torch.empty(E, 200, 80, device=dev)
    splits = auto_splits(200, 80, Bt, E)
    ws = torch.empty(L.lib().rs_gemm_x3_workspace_size(200, 80, E, splits), dtype=torch.uint8,
                     device=dev)
    fl = 2.0 * E * Bt * 200 * 80
    for name, lib, ours in (
            ("batched forward+bias+relu", lambda: torch.relu_(torch.baddbmm(bb, h, k)),
             lambda: x3(0, 0, Bt, 80, 200, h, k, yb, batch=E, bias=bb.view(E, 80), act=1)),
            ("batched wgrad", lambda: bwgrad(h, g),
             lambda: x3(1, 0, 200, 80, Bt, h, g, dwb, batch=E, splits=splits, ws=ws))):
        tl, to = timeit(lib), timeit(ours)
        print(json.dumps({"shape": f"{E}x{Bt}x200->80", "product": name, "library_us": round(tl, 1),
                          "x3_us": round(to, 1), "library_TF": round(fl / tl / 1e6, 1),
                          "x3_TF": round(fl / to / 1e6, 1), "speedup": round(tl / to, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
