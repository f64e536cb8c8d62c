"""Host issue cost of the north-star DLRM step (run under gpurun): the time the host needs to
queue N steps while the GPU is held busy by a long sleep kernel queued first (so no launch ever
waits for the device), against the GPU-bound step time. python tools/host_time.py [--prefetch 1]
[--sharded 1 --batch 8192]: the row-sharded slab's fused step at world 1 (its exchange kernels,
its collectives as copies) — the host cost a strong-scaling rank would pay, minus the
collectives and the world > 1 extras (rows ahead, owner halves)"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_amd import _lib as L  # noqa: E402
from recommender_amd.ctr.train import TrainStep, build_model  # noqa: E402
from recommender_amd.synthetic import criteo_batch, criteo_cardinalities  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--prefetch", type=int, default=0)
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--profile", type=int, default=0)
ap.add_argument("--sharded", type=int, default=0)
ap.add_argument("--batch", type=int, default=65536)
a = ap.parse_args()
L.load()
dev = torch.device("cuda", 0)
S, D, V, B = 26, 128, 40_000_000, a.batch
cards = criteo_cardinalities(V, S)
g = torch.Generator(device=dev)
g.manual_seed(4)
if a.sharded:
    from recommender_amd.ctr.model import DLRM
    from recommender_amd.sharded import Comm, ShardedSlabEmbedding

    comm = Comm()
    emb = ShardedSlabEmbedding(cards, D, comm, device=dev, generator=g)
    m = DLRM([512, 256, D], [512, 256, 1], D, V, S, 13, device=dev, generator=g,
             embedding_layer=emb)
    st = TrainStep(m, "sgd", lr=0.01, fused=True, comm=comm, defer_sparse_join=True)
else:
    m = build_model("DLRM", D, V, S, 13, dev, slot_cardinalities=cards, bottom=[512, 256, D],
                    top=[512, 256, 1], generator=g)
    st = TrainStep(m, "sgd", lr=0.01, fused=True, defer_sparse_join=True)
rng = np.random.default_rng(4)
pool = [tuple(torch.from_numpy(x).to(dev) for x in criteo_batch(rng, B, cards)) for _ in range(4)]
P = len(pool)


def run(i):
    if a.prefetch:
        st.prefetch(pool[(i + 1) % P])
    st(pool[i % P])


for i in range(10):
    run(i)
torch.cuda.synchronize()
# GPU-bound time
t0 = time.perf_counter()
for i in range(a.steps):
    run(i)
torch.cuda.synchronize()
gpu = (time.perf_counter() - t0) / a.steps
# host issue time with the device held busy
torch.cuda._sleep(int(2.5e9))  # ~1 s of GPU spin ahead of the steps
t0 = time.perf_counter()
if a.profile:
    import cProfile
    import pstats

    pr = cProfile.Profile()
    pr.enable()
for i in range(a.steps):
    run(i)
host = (time.perf_counter() - t0) / a.steps
if a.profile:
    pr.disable()
torch.cuda.synchronize()
print(f"sharded {a.sharded} batch {B} prefetch {a.prefetch}: step {gpu * 1e3:.3f} ms, "
      f"host issue {host * 1e3:.3f} ms/step")
if a.profile:
    pstats.Stats(pr).sort_stats("cumulative").print_stats(35)
