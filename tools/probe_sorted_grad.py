"""Probe (round 6): what would the north-star apply cost if the gradient rows it reads were laid
out in SORTED order (row k of the buffer = sorted entry k), instead of gathered by position?
Runs rs_embedding_apply_scaled (SGD, lr 0: same bytes) on the bench's slab, ids and sort with
  real      sorted positions (production: each gradient row gathered by its position)
  contig    positions = 0..n-1 (each tile's 32 rows read contiguously; row_scale index wrong,
            timing only)
and the train kernel with its rows written in position order, plus a plain HBM copy of the same
bytes for reference. HIP events over 20 launches each, interleaved three times.
PROBE_VARIANT=<path to an A/B build's .so>: the production apply against that build's, interleaved.
    python tools/probe_sorted_grad.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_amd import _lib as L  # noqa: E402
from recommender_amd.ctr.train import build_model  # noqa: E402
from recommender_amd.synthetic import criteo_batch, criteo_cardinalities  # noqa: E402


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    dev = torch.device("cuda", 0)
    L.load()
    S, D, B, V = 26, 128, 65536, 40_000_000
    cards = criteo_cardinalities(V, S)
    g = torch.Generator(device=dev).manual_seed(4)
    model = build_model("DLRM", D, V, S, 13, dev, slot_cardinalities=cards, bottom=[512, 256, D],
                        top=[512, 256, 1], generator=g)
    emb = model.embedding_layer
    w, so, err = emb.weight, emb.slot_offsets, emb.err_flag
    cat, _, _ = criteo_batch(np.random.default_rng(4), B, cards)
    ids = torch.from_numpy(cat).to(dev).contiguous()
    n = B * S
    st = L.stream_ptr(dev)
    rows = torch.empty(n, dtype=torch.int32, device=dev)
    pos = torch.empty(n, dtype=torch.int32, device=dev)
    sws = torch.empty(L.lib().rs_sort_ids_workspace_size(n), dtype=torch.uint8, device=dev)
    L.call("rs_sort_ids_slots", L.ptr(ids), L.id_dtype_code(ids), n, None, L.ptr(so), S, V,
           emb.max_slot_rows, L.ptr(rows), L.ptr(pos), None, L.ptr(err), L.ptr(sws), sws.numel(), st)
    torch.cuda.synchronize()
    ar = torch.arange(n, dtype=torch.int32, device=dev)
    dxu = torch.randn(n, D, device=dev) * 1e-3
    gb = torch.rand(B, device=dev)
    aws = torch.empty(L.lib().rs_apply_workspace_size(n, D), dtype=torch.uint8, device=dev)
    prm = L.AdamParams(0.0, 0.0, 0.0, 0.0, 0.0, 0.0)

    def apply(p, scale=True):
        return lambda: L.call("rs_embedding_apply_scaled", L.RS_OPT_SGD, L.ptr(w), None, None, V, D,
                              L.ptr(rows), L.ptr(p), n, L.ptr(dxu), L.ptr(gb) if scale else None,
                              S, prm, None, L.ptr(aws), aws.numel(), st)

    dst = torch.empty_like(dxu)
    res = {}
    sort = lambda: L.call("rs_sort_ids_slots", L.ptr(ids), L.id_dtype_code(ids), n, None,  # noqa: E731
                          L.ptr(so), S, V, emb.max_slot_rows, L.ptr(rows), L.ptr(pos), None,
                          L.ptr(err), L.ptr(sws), sws.numel(), st)
    res["sort"] = [round(timed(sort), 1), round(timed(sort), 1)]
    variant = os.environ.get("PROBE_VARIANT")  # an A/B build of the library (same C-ABI)
    vapply = None
    if variant:
        import ctypes as C
        vl = C.CDLL(variant)
        f = vl.rs_embedding_apply_scaled
        f.restype, f.argtypes = L.lib().rs_embedding_apply_scaled.restype, L.lib().rs_embedding_apply_scaled.argtypes

        def vapply():
            rc = f(L.RS_OPT_SGD, L.ptr(w), None, None, V, D, L.ptr(rows), L.ptr(pos), n, L.ptr(dxu),
                   L.ptr(gb), S, prm, None, L.ptr(aws), aws.numel(), st)
            assert rc == 0
    for rep in range(3):
        cases = [("apply_real", apply(pos))]
        if vapply is not None:
            cases.append(("apply_variant", vapply))
        if not variant:
            cases += [("apply_contig", apply(ar)), ("apply_contig_noscale", apply(ar, False)),
                      ("copy_grad_bytes", lambda: dst.copy_(dxu))]
        for name, fn in cases:
            res.setdefault(name, []).append(round(timed(fn), 1))
    uniq = int(torch.unique(rows).numel())
    print(json.dumps({"probe": "sorted_grad", "unique_rows": uniq, "us": res}), flush=True)


if __name__ == "__main__":
    main()
