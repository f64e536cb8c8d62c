"""Probe GEMM formulations for the MMOE expert layers (B 65536, 8 experts, 324→200→80)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_amd.nn import bwgrad, wgrad  # noqa: E402

dev = "cuda"


def bench(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


B, E, I, H0, H1 = 65536, 8, 324, 200, 80
x = torch.randn(B, I, device=dev)
k0 = torch.randn(I, E * H0, device=dev)
g0 = torch.randn(B, E * H0, device=dev)
r = {"L1 fwd": bench(lambda: x @ k0), "L1 dgrad": bench(lambda: g0 @ k0.t()),
     "L1 wgrad": bench(lambda: wgrad(x, g0))}
h = torch.randn(E, B, H0, device=dev)
hb = h.transpose(0, 1).contiguous()  # [B, E, H0]
k1 = torch.randn(E, H0, H1, device=dev)
g1 = torch.randn(E, B, H1, device=dev)
r["L2 bmm fwd"] = bench(lambda: torch.bmm(h, k1))
r["L2 loop fwd"] = bench(lambda: [h[e] @ k1[e] for e in range(E)])
r["L2 bmm dgrad"] = bench(lambda: torch.bmm(g1, k1.transpose(1, 2)))
r["L2 loop dgrad"] = bench(lambda: [g1[e] @ k1[e].t() for e in range(E)])
r["L2 bwgrad"] = bench(lambda: bwgrad(h, g1))
r["L2 loop wgrad"] = bench(lambda: [wgrad(h[e], g1[e]) for e in range(E)])
r["L2 fwd from [B,E,H]"] = bench(lambda: torch.bmm(hb.transpose(0, 1), k1))
gw = torch.randn(B, 1, E, device=dev)
ex = torch.randn(B, E, H1, device=dev)
r["gate bmm"] = bench(lambda: torch.bmm(gw, ex))
r["gate mul-sum"] = bench(lambda: (gw.transpose(1, 2) * ex).sum(1))
for k, v in r.items():
    print(f"{k:24s} {v:8.1f} us")
