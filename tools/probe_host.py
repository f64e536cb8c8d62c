"""Host enqueue time vs GPU time per DLRM step (is the step host-bound?)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_amd import _lib as L  # noqa: E402
from recommender_amd.ctr.train import TrainStep, build_model  # noqa: E402
from recommender_amd.synthetic import criteo_batch, criteo_cardinalities  # noqa: E402

L.load()
dev = torch.device("cuda")
cards = criteo_cardinalities(40_000_000, 26)
g = torch.Generator(device=dev).manual_seed(4)
model = build_model("DLRM", 128, 40_000_000, 26, 13, dev, slot_cardinalities=cards,
                    bottom=[512, 256, 128], top=[512, 256, 1], generator=g)
step = TrainStep(model, "sgd", lr=0.01, fused=True)
rng = np.random.default_rng(4)
pool = []
for _ in range(4):
    c, d, lb = criteo_batch(rng, 65536, cards)
    pool.append((torch.from_numpy(c).to(dev), torch.from_numpy(d).to(dev), torch.from_numpy(lb).to(dev)))
for i in range(5):
    step(pool[i % 4])
torch.cuda.synchronize()
for n in (1, 20):
    t0 = time.perf_counter()
    for i in range(n):
        step(pool[i % 4])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{n} steps: host enqueue {(t1 - t0) / n * 1e3:.3f} ms/step, wall {(t2 - t0) / n * 1e3:.3f} ms/step")
# host time split: forward vs backward vs optimizer
import torch.nn.functional as F  # noqa: E402
ts = []
for i in range(10):
    torch.cuda.synchronize()
    a = time.perf_counter()
    step(pool[i % 4])
    b = time.perf_counter()
    torch.cuda.synchronize()
    c = time.perf_counter()
    ts.append((b - a, c - a))
print("isolated step: host %.3f ms, wall %.3f ms" % tuple(np.median(np.array(ts), 0) * 1e3))
