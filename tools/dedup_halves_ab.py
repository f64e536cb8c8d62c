"""A/B: the mapped dedup over the whole key space (one call) vs two owner-half calls (world-2 key
split), isolated on one stream, north-star ids at B = 32768 (the world-2 strong per-rank batch)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from recommender_amd import _lib as L
from recommender_amd.synthetic import criteo_batch, criteo_cardinalities
L.load()
dev = torch.device("cuda")
S, B, D = 26, int(sys.argv[1]) if len(sys.argv) > 1 else 32768, 128
cards = criteo_cardinalities(40_000_000, S)
so = torch.tensor(np.concatenate([[0], np.cumsum(cards)]), dtype=torch.int64, device=dev)
V = int(so[-1])
cat, _, _ = criteo_batch(np.random.default_rng(4), B, cards)
ids = torch.from_numpy(cat).to(dev)
n = B * S
ws = torch.empty(L.lib().rs_sort_ids_workspace_size(n), dtype=torch.uint8, device=dev)
rows = torch.empty(n, dtype=torch.int32, device=dev); pos = torch.empty_like(rows)
nu = torch.zeros(1, dtype=torch.int32, device=dev)
st = L.stream_ptr(dev)
L.call("rs_sort_ids", L.ptr(ids), L.id_dtype_code(ids), n, L.ptr(so), S, V, L.ptr(rows), L.ptr(pos), L.ptr(nu), None, L.ptr(ws), ws.numel(), st)
torch.cuda.synchronize()
U = int(nu.item())
seg_map = torch.arange(n, dtype=torch.int32, device=dev)
uniq_rows = torch.empty(n, dtype=torch.int32, device=dev)
grad = torch.randn(n, D, device=dev)
scale = torch.rand(B, device=dev)
out1 = torch.zeros(U + 1, D, device=dev); out2 = torch.zeros(U + 1, D, device=dev)
dws = torch.empty(L.lib().rs_dedup_workspace_size(n, D), dtype=torch.uint8, device=dev)
K = V // 2
def call(out, lo, hi, ready):
    L.call("rs_embedding_dedup_grad_mapped_range", L.ptr(rows), L.ptr(pos), n, L.ptr(grad), L.ptr(scale), S, D, V, lo, hi, ready, None, L.ptr(seg_map), L.ptr(uniq_rows), L.ptr(out), L.ptr(dws), dws.numel(), st)
def one():
    call(out1, 0, V, 0)
def two():
    call(out2, 0, K, 0); call(out2, K, V, 1)
def halfA():
    call(out2, 0, K, 0)
for name, fn in (("full", one), ("halves", two), ("halfA", halfA), ("full", one), ("halves", two), ("halfA", halfA)):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): fn()
    e1.record(); torch.cuda.synchronize()
    print(name, round(e0.elapsed_time(e1) / 20 * 1e3, 1), "us", "U", U)
two(); one(); torch.cuda.synchronize()
print("identical", torch.equal(out1[:U], out2[:U]))
