"""Probe rs_masked_topk timing across shapes (rows, items, k, exclusion)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.bench_kernels import timed  # noqa: E402
from recommender_amd.pinsage.evaluation import masked_topk  # noqa: E402
from recommender_amd.pinsage.graph import HeteroGraph  # noqa: E402

for R, I, K, ex in [(6040, 3706, 10, True), (6040, 3706, 10, False), (6040, 3706, 1, False),
                    (6040, 256, 1, False), (24160, 3706, 10, False), (6040, 14824, 10, False),
                    (8192, 26744, 10, False)]:
    s = torch.randn(R, I, device="cuda")
    g = None
    if ex:
        u = torch.randint(0, R, (R * 165,))
        i = torch.randint(0, I, (R * 165,))
        g = HeteroGraph(u.numpy(), i.numpy(), R, I)
    us = timed(lambda: masked_topk(s, K, 0, g), 20)
    print(f"R={R} I={I} K={K} excl={ex}: {us:.1f} us  {R * I * 4 / us / 1e3:.0f} GB/s", flush=True)
