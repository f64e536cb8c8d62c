"""A/B price of the north-star id sort: rs_sort_ids (the engine's 3-pass LSD radix, ids -> sorted
(row, position)) against rocPRIM's device radix_sort_pairs (onesweep) on the same keys, built as
tools/librocprim_sort_ref.so (reference only, never loaded by the product). Run on the GPU box:
python tools/sort_ab.py [--batch 65536]. Prints one JSON line per variant."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from recommender_amd import _lib as L  # noqa: E402
from recommender_amd.synthetic import criteo_batch, criteo_cardinalities  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--rows", type=int, default=40_000_000)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    L.load()
    cards = criteo_cardinalities(a.rows, 26)
    so = np.concatenate([[0], np.cumsum(cards)]).astype(np.int64)
    cat, _, _ = criteo_batch(np.random.default_rng(4), a.batch, cards)
    n = cat.size
    keys_h = (cat + so[:-1][None, :]).reshape(-1).astype(np.uint32)
    ids = torch.from_numpy(cat).to(dev)
    so_t = torch.from_numpy(so).to(dev)
    st = L.stream_ptr(dev)
    rows = torch.empty(n, dtype=torch.int32, device=dev)
    pos = torch.empty(n, dtype=torch.int32, device=dev)
    nu = torch.zeros(1, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = torch.empty(L.lib().rs_sort_ids_workspace_size(n), dtype=torch.uint8, device=dev)

    def ours():
        L.call("rs_sort_ids", L.ptr(ids), L.id_dtype_code(ids), n, L.ptr(so_t), 26, a.rows,
               L.ptr(rows), L.ptr(pos), L.ptr(nu), L.ptr(err), L.ptr(ws), ws.numel(), st)

    ref = C.CDLL(os.path.join(ROOT, "tools", "librocprim_sort_ref.so"))
    ref.ref_sort_ws.restype = C.c_size_t
    ref.ref_sort_ws.argtypes = [C.c_int64, C.c_int]
    ref.ref_sort_pairs.restype = C.c_int
    ref.ref_sort_pairs.argtypes = [C.c_void_p] * 4 + [C.c_int64, C.c_int, C.c_void_p, C.c_size_t,
                                                     C.c_void_p]
    bits = int(a.rows).bit_length()
    kin = torch.from_numpy(keys_h.view(np.int32)).to(dev)
    vin = torch.arange(n, dtype=torch.int32, device=dev)
    kout = torch.empty_like(kin)
    vout = torch.empty_like(vin)
    rws = torch.empty(ref.ref_sort_ws(n, bits), dtype=torch.uint8, device=dev)

    def rocprim():
        rc = ref.ref_sort_pairs(kin.data_ptr(), kout.data_ptr(), vin.data_ptr(), vout.data_ptr(), n,
                                bits, rws.data_ptr(), rws.numel(), st)
        assert rc == 0, rc

    out = {}
    for name, fn in (("rs_sort_ids", ours), ("rocprim_radix_sort_pairs", rocprim)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) / a.iters * 1e3
    same = bool(torch.equal(rows, kout) and torch.equal(pos, vout))
    for k, v in out.items():
        print(json.dumps({"sort": k, "n": n, "key_bits": bits, "avg_us": round(v, 2),
                          "identical_to_other": same}))


if __name__ == "__main__":
    main()
