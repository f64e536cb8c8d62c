"""Is rs_gemm_x3's error biased? Mean signed error of C against float64, in units of the mean
term magnitude, for the Dense forward shape, next to the library fp32 GEMM's (gpurun)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_amd import nn as N  # noqa: E402

torch.manual_seed(0)
dev = "cuda"
for (M, K, Nn, pos) in ((65536, 324, 360, False), (65536, 324, 360, True), (8192, 4096, 256, True)):
    x = torch.randn(M, K, device=dev)
    w = torch.randn(K, Nn, device=dev) * 0.05
    if pos:  # one-signed operands: a rounding bias adds up instead of cancelling
        x, w = x.abs(), w.abs()
    ref = x.double() @ w.double()
    mag = x.double().abs() @ w.double().abs()
    N._GEMM_X3 = True
    c3 = N.gemm_x3(x, w)
    cl = x @ w
    torch.cuda.synchronize()
    for name, c in (("x3", c3), ("library", cl)):
        e = (c.double() - ref)
        print(f"M{M} K{K} N{Nn} pos={pos} {name:8s} mean signed err / mean mag {float(e.mean() / mag.mean()):+.3e}"
              f"  mean |err| / mean mag {float(e.abs().mean() / mag.mean()):.3e}  max |err|/mag {float((e.abs() / mag).max()):.3e}")
