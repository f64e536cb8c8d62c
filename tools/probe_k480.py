"""Top-MLP first layer GEMMs at K = 512 (current compact padding) vs 480 / 496 / 479."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_amd.nn import wgrad  # noqa: E402


def bench(fn, n=20):
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


B, N = 65536, 512
for K in (512, 480, 496, 479):
    x = torch.randn(B, K, device="cuda")
    w = torch.randn(K, N, device="cuda")
    g = torch.randn(B, N, device="cuda")
    f = bench(lambda: x @ w)
    d = bench(lambda: g @ w.t())
    wg = bench(lambda: wgrad(x, g))
    print(f"K={K}: fwd {f:.1f} dgrad {d:.1f} wgrad {wg:.1f} total {f + d + wg:.1f} us")
