"""Probe: the slot-segmented sort on the north-star shape with Zipf ids (Criteo-spread, hot
ids) vs uniform ids; run under rocprofv3 --kernel-trace for the per-kernel split
(tools/prof_db_stats.py reads its results database)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from recommender_amd import _lib as L
from recommender_amd.synthetic import criteo_batch, criteo_cardinalities
L.load()
dev = torch.device("cuda")
S, B = 26, 65536
cards = criteo_cardinalities(40_000_000, S)
so = torch.tensor(np.concatenate([[0], np.cumsum(cards)]), dtype=torch.int64, device=dev)
V = int(so[-1])
rng = np.random.default_rng(4)
zipf, _, _ = criteo_batch(rng, B, cards)
unif = np.stack([rng.integers(0, c, B) for c in cards], 1).astype(np.int64)
n = B * S
ws = torch.empty(L.lib().rs_sort_ids_workspace_size(n), dtype=torch.uint8, device=dev)
r = torch.empty(n, dtype=torch.int32, device=dev); p = torch.empty_like(r)
st = L.stream_ptr(dev)
for name, cat in (("zipf", zipf), ("uniform", unif), ("zipf", zipf), ("uniform", unif)):
    ids = torch.from_numpy(cat).to(dev)
    fn = lambda: L.call("rs_sort_ids_slots", L.ptr(ids), 1, n, None, L.ptr(so), S, V, max(cards),
                        L.ptr(r), L.ptr(p), None, None, L.ptr(ws), ws.numel(), st)
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(30): fn()
    e1.record(); torch.cuda.synchronize()
    print(name, round(e0.elapsed_time(e1) / 30 * 1e3, 1), "us", flush=True)
