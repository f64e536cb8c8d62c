"""A/B: slot-segmented sort (rs_sort_ids_slots) vs LSD (rs_sort_ids at n_rows > 2^24) on the
north-star ids; prints us per call and checks identical output."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from recommender_amd import _lib as L
from recommender_amd.synthetic import criteo_batch, criteo_cardinalities
L.load()
dev = torch.device("cuda")
S, B = 26, int(sys.argv[1]) if len(sys.argv) > 1 else 65536
cards = criteo_cardinalities(40_000_000, S)
so = torch.tensor(np.concatenate([[0], np.cumsum(cards)]), dtype=torch.int64, device=dev)
V = int(so[-1])
rng = np.random.default_rng(4)
cat, _, _ = criteo_batch(rng, B, cards)
ids = torch.from_numpy(cat).to(dev)
n = B * S
ws = torch.empty(L.lib().rs_sort_ids_workspace_size(n), dtype=torch.uint8, device=dev)
r1 = torch.empty(n, dtype=torch.int32, device=dev); p1 = torch.empty_like(r1)
r2 = torch.empty_like(r1); p2 = torch.empty_like(r1)
st = L.stream_ptr(dev)
def seg():
    L.call("rs_sort_ids_slots", L.ptr(ids), 1, n, None, L.ptr(so), S, V, max(cards), L.ptr(r1), L.ptr(p1), None, None, L.ptr(ws), ws.numel(), st)
def lsd():
    L.call("rs_sort_ids", L.ptr(ids), 1, n, L.ptr(so), S, V, L.ptr(r2), L.ptr(p2), None, None, L.ptr(ws), ws.numel(), st)
for name, fn in (("seg", seg), ("lsd", lsd), ("seg", seg), ("lsd", lsd)):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50): fn()
    e1.record(); torch.cuda.synchronize()
    print(name, round(e0.elapsed_time(e1) / 50 * 1e3, 1), "us")
print("identical", torch.equal(r1, r2) and torch.equal(p1, p2))
