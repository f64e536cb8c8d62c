"""Per-kernel roofline table for the secondary paths (DIEN attention + GRU/AUGRU,
PinSage sampling + mean-pool, EGES, ESMM-shaped embedding) at their BASELINE config shapes.

Every kernel is called through the C ABI on device-resident inputs, timed with HIP events
over `--iters` launches on the stream it runs on, and reported with its ALGORITHMIC bytes per
launch (each input byte read once, each output byte written once; the formulas are next to
each case and in DESIGN.md §4), achieved GB/s and the fraction of the 8 TB/s HBM peak.
The recurrent DIEN kernels carry L dependent steps per example, so they are latency-bound by
construction ("DIEN is really latency-bound"); their fraction says how far.

Usage: python benchmarks/bench_kernels.py [--iters 20] > profiles/rNN_kernel_roofline.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_amd import _lib as L  # noqa: E402

PEAK = 8000.0  # GB/s, MI355X HBM3E spec
DEV = "cuda"


def timed(fn, iters):
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def report(name, cfg, us, nbytes, out):
    gbs = nbytes / (us * 1e-6) / 1e9
    line = {"kernel": name, "config": cfg, "avg_us": round(us, 2), "algorithmic_bytes": int(nbytes),
            "achieved_GBs": round(gbs, 1), "frac_of_hbm_peak": round(gbs / PEAK, 4)}
    out.append(line)
    print(json.dumps(line), flush=True)


def dien(iters, out):
    B, T, H = 4096, 100, 36
    g = torch.Generator(device=DEV).manual_seed(0)
    xw = torch.randn(B, T, 3 * H, device=DEV, generator=g)
    U = torch.randn(H, 3 * H, device=DEV, generator=g) * 0.1
    rb = torch.zeros(3 * H, device=DEV)
    lens = torch.randint(2, T + 1, (B,), device=DEV, generator=g)
    mask = (torch.arange(T, device=DEV)[None] < lens[:, None]).to(torch.uint8).contiguous()
    outp = torch.empty(B, T, H, device=DEV)
    saved = torch.empty(B, T, 4 * H, device=DEV)
    st = L.stream_ptr(DEV)
    cfg = {"B": B, "L": T, "H": H}
    us = timed(lambda: L.call("rs_gru_fwd", L.ptr(xw), L.ptr(U), L.ptr(rb), L.ptr(mask), B, T, H,
                              L.ptr(outp), L.ptr(saved), st), iters)
    report("rs_gru_fwd", cfg, us, B * T * (12 * H + 1 + 4 * H + 16 * H), out)
    dout = torch.randn(B, T, H, device=DEV, generator=g)
    dxw = torch.empty(B, T, 3 * H, device=DEV)
    din = torch.empty(B, T, 3 * H, device=DEV)
    us = timed(lambda: L.call("rs_gru_bwd", L.ptr(dout), L.ptr(outp), L.ptr(saved), L.ptr(U),
                              L.ptr(mask), B, T, H, L.ptr(dxw), L.ptr(din), 0, st), iters)
    report("rs_gru_bwd", cfg, us, B * T * (4 * H + 4 * H + 16 * H + 1 + 12 * H + 12 * H), out)
    att = torch.rand(B, T, device=DEV, generator=g)
    kuh = torch.randn(H, H, device=DEV, generator=g) * 0.1
    final = torch.empty(B, H, device=DEV)
    states = torch.empty(B, T, H, device=DEV)
    us = timed(lambda: L.call("rs_augru_fwd", L.ptr(xw), L.ptr(att), L.ptr(kuh), L.ptr(kuh),
                              L.ptr(kuh), L.ptr(mask), B, T, H, L.ptr(final), L.ptr(states),
                              L.ptr(saved), 0, st), iters)
    report("rs_augru_fwd", cfg, us, B * T * (12 * H + 4 + 1 + 4 * H + 16 * H) + 4 * B * H, out)
    dfinal = torch.randn(B, H, device=DEV, generator=g)
    datt = torch.empty(B, T, device=DEV)
    us = timed(lambda: L.call("rs_augru_bwd", L.ptr(dfinal), L.ptr(att), L.ptr(states),
                              L.ptr(saved), L.ptr(kuh), L.ptr(kuh), L.ptr(kuh), L.ptr(mask), B, T,
                              H, L.ptr(dxw), L.ptr(datt), 0, st), iters)
    report("rs_augru_bwd", cfg, us, B * T * (4 + 4 * H + 16 * H + 1 + 12 * H + 4) + 4 * B * H, out)
    hs = torch.randn(B, T, H, device=DEV, generator=g)
    q = torch.randn(B, H, device=DEV, generator=g)
    a = torch.empty(B, T, device=DEV)
    us = timed(lambda: L.call("rs_dien_attention_fwd", L.ptr(hs), L.ptr(q), L.ptr(mask), B, T, H,
                              L.ptr(a), st), iters)
    report("rs_dien_attention_fwd", cfg, us, B * T * (4 * H + 1 + 4) + 4 * B * H, out)
    da = torch.randn(B, T, device=DEV, generator=g)
    dhs = torch.empty_like(hs)
    dq = torch.empty_like(q)
    us = timed(lambda: L.call("rs_dien_attention_bwd", L.ptr(hs), L.ptr(q), L.ptr(a), L.ptr(da), B,
                              T, H, L.ptr(dhs), L.ptr(dq), st), iters)
    report("rs_dien_attention_bwd", cfg, us, B * T * (4 * H + 4 + 4 + 4 * H) + 8 * B * H, out)


def pinsage(iters, out):
    from recommender_amd.pinsage import PinSageSampler
    from recommender_amd.pinsage.layers import weighted_mean_agg  # noqa: F401
    from recommender_amd.pinsage.sampler import item_pairs
    from recommender_amd.pinsage.train import ML20M, build_graph

    g = build_graph(ML20M, 4)
    smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
    h, p, n = item_pairs(g, 4096, 4, 0)
    seeds, _, ns = smp.unique_first(torch.cat([h, p, n]), g.n_items)
    seeds = seeds[: int(ns.item())].contiguous()
    S = seeds.numel()
    cfg = {"graph": "ml20m_shaped", "edges": g.n_edges, "seeds": S, "walks": 4, "traversals": 2,
           "k": 3}
    # 4 walks x 4 hops, each hop: indptr pair (16 B) + one neighbour id (4 B); out 3 x (4 + 4) B
    us = timed(lambda: smp.neighbors(seeds, 0, None, 0), iters)
    report("rs_pinsage_neighbors", cfg, us, S * (4 + 4 * 4 * 20 + 3 * 8), out)
    nbr, cnt = smp.neighbors(seeds, 0, None, 0)
    ids = torch.cat([seeds, nbr.reshape(-1)])
    us = timed(lambda: smp.unique_first(ids, g.n_items), iters)
    report("rs_unique_first", {"n": ids.numel(), "n_nodes": g.n_items}, us,
           ids.numel() * (4 + 4 + 4 + 4) + g.n_items * 4, out)
    blk = smp.to_block(seeds, nbr, cnt)
    E = int(blk.n_edges.item())
    Hh = 32
    u = torch.randn(blk.n_src, Hh, device=DEV)
    nv = torch.empty(blk.n_dst, Hh, device=DEV)
    wsum = torch.empty(blk.n_dst, device=DEV)
    st = L.stream_ptr(DEV)
    acfg = {"n_dst": blk.n_dst, "n_src": blk.n_src, "edges": E, "H": Hh}
    us = timed(lambda: L.call("rs_weighted_mean_agg_fwd", L.ptr(u), blk.n_src, Hh, L.ptr(blk.indptr),
                              L.ptr(blk.edge_src), L.ptr(blk.edge_w), blk.n_dst, L.ptr(nv),
                              L.ptr(wsum), st), iters)
    report("rs_weighted_mean_agg_fwd", acfg, us, E * (4 + 4 + 4 * Hh) + blk.n_dst * (8 + 4 * Hh), out)
    gu = torch.empty_like(u)
    us = timed(lambda: L.call("rs_weighted_mean_agg_bwd", L.ptr(nv), Hh, L.ptr(blk.t_indptr),
                              L.ptr(blk.t_edge), L.ptr(blk.edge_dst), L.ptr(blk.edge_w), L.ptr(wsum),
                              blk.n_src, L.ptr(gu), st), iters)
    report("rs_weighted_mean_agg_bwd", acfg, us,
           E * (4 + 4 + 4 + 4 + 4 * Hh) + blk.n_src * (4 + 4 * Hh), out)


def eges(iters, out):
    from recommender_amd.embedding import Embedding

    B, M, D, V = 1024, 6, 160, 63001
    t = Embedding(V, D, device=DEV)
    ids = torch.randint(0, V, (B, M), device=DEV, dtype=torch.int32)
    h = torch.randn(B, D, device=DEV)
    logits = torch.empty(B, M, device=DEV)
    st = L.stream_ptr(DEV)
    cfg = {"B": B, "M": M, "D": D}
    us = timed(lambda: L.call("rs_match_logits_fwd", L.ptr(t.weight), V, D, L.ptr(ids), 0, M, L.ptr(h),
                              B, L.ptr(logits), L.ptr(t.err_flag), st), iters)
    report("rs_match_logits_fwd", cfg, us, B * M * (4 + 4 * D) + B * 4 * D + B * M * 4, out)
    rows = torch.empty(B * M, D, device=DEV)
    gh = torch.empty(B, D, device=DEV)
    us = timed(lambda: L.call("rs_match_logits_bwd", L.ptr(t.weight), V, D, L.ptr(ids), 0, M, L.ptr(h),
                              L.ptr(logits), B, L.ptr(rows), L.ptr(gh), st), iters)
    report("rs_match_logits_bwd", cfg, us,
           B * M * (4 + 4 * D + 4) + B * 4 * D + B * M * 4 * D + B * 4 * D, out)


def eges_sampler(iters, out):
    """EGES pair pipeline on a 63001-item weighted graph, 65536 walks of
    length 10 per refill. Bytes: traces written + per hop indptr pair / log2(deg) prefix probes
    / one index (random reads, latency-bound); skipgrams: traces read, flag + offset per slot,
    pairs written; negatives: ids written (the CDF table is L2-resident; the kernel is ALU-bound)."""
    from recommender_amd.eges.sampler import EGESPairSampler, skipgram_slots
    from tests.eges_graph import make_graph

    V, W, Lw = 63001, 65536, 10
    indptr, indices, w = make_graph(np.random.default_rng(4), V, 1_000_000, 50)
    s = EGESPairSampler(indptr, indices, w, V, device=DEV, walks_per_refill=W)
    deg = max(1.0, indices.size / V)
    probes = int(np.ceil(np.log2(deg + 1)))
    cfg = {"items": V, "edges": int(indices.size), "walks": W, "length": Lw}
    us = timed(lambda: s.walks(W, 1), iters)
    report("rs_eges_walks", cfg, us, W * (Lw + 1) * 4 + W * Lw * (16 + 4 + 8 * probes), out)
    tr = s.walks(W, 1)
    slots = skipgram_slots(Lw + 1, 5)
    us = timed(lambda: s.skipgrams(tr), iters)
    tgt, _ = s.skipgrams(tr)
    P = tgt.numel()
    report("rs_skipgram_pairs(+1 sync)", dict(cfg, pairs=P), us,
           W * (Lw + 1) * 4 * 2 + W * slots * 16 + P * 8, out)
    us = timed(lambda: s.negatives(P, 1), iters)
    report("rs_log_uniform_sample(ALU-bound: Philox + CDF walk)", {"pairs": P, "num_ns": 5,
                                                                 "range": V}, us, P * 5 * 4, out)
    def refill():
        s._target, s._context = s._target[:0], s._context[:0]
        s.refill()

    us = timed(refill, max(3, iters // 4))
    line = {"kernel": "eges_refill(walks+skipgrams+negatives)", "config": dict(cfg, pairs=P),
            "avg_us": round(us, 2), "pairs_per_s": round(P / (us * 1e-6))}
    out.append(line)
    print(json.dumps(line), flush=True)


def pinsage_eval(iters, out):
    """PinSage evaluation at ML-1M / ML-20M shapes: rs_masked_topk bytes =
    the score rows read once + the exclusion CSR + the top-k written; plus the whole
    get_item_reprs → recommend → hit_rate pass on ML-1M, wall clock."""
    import time

    from recommender_amd.pinsage import PinSageModel, PinSageSampler
    from recommender_amd.pinsage.evaluation import (get_item_reprs, hit_rate_eval, masked_topk,
                                                    recommend)
    from recommender_amd.pinsage.train import ML1M, build_dataset
    from recommender_amd.synthetic import ML20M

    for name, shape in (("ml1m", ML1M), ("ml20m", ML20M)):
        g, val, _ = build_dataset(shape, 4, DEV)
        R = min(g.n_users, 8192)
        scores = torch.randn(R, g.n_items, device=DEV)
        nb = R * g.n_items * 4 + int(g.u2i_indptr[R]) * 4 + R * 8 + R * 10 * 4
        us = timed(lambda: masked_topk(scores, 10, 0, g), iters)
        report("rs_masked_topk", {"graph": name, "rows": R, "items": g.n_items, "k": 10}, us, nb,
               out)
        if name != "ml1m":
            continue
        torch.manual_seed(0)
        model = PinSageModel(g, g.itype, 2, 8, 32, 16)
        smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reprs = get_item_reprs(model, smp, g, g.itype, 32)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            recs = recommend(g, 10, reprs, None, g.utype, "timestamp", 32)
            hr = hit_rate_eval(recs, val.tocsr())
            torch.cuda.synchronize()
            t2 = time.perf_counter()
        line = {"kernel": "pinsage_eval(get_item_reprs bs32 + recommend + hit_rate)",
                "config": {"graph": name, "users": g.n_users, "items": g.n_items, "k": 10},
                "item_reprs_ms": round((t1 - t0) * 1e3, 2),
                "recommend_hit_rate_ms": round((t2 - t1) * 1e3, 3), "hit_rate": hr}
        out.append(line)
        print(json.dumps(line), flush=True)


def embedding(iters, out):
    from recommender_amd.esmm import FEAT_VOCAB
    from recommender_amd.synthetic import aliccp_batch, scaled_vocab

    vocab = scaled_vocab(FEAT_VOCAB, 40_000_000)
    card = torch.tensor(list(vocab.values()), dtype=torch.int64)
    so = torch.zeros(card.numel() + 1, dtype=torch.int64)
    so[1:] = torch.cumsum(card, 0)
    V, D, B, S = int(so[-1]), 18, 65536, card.numel()
    table = torch.empty(V, D, device=DEV).uniform_(-0.05, 0.05)
    feats, _ = aliccp_batch(np.random.default_rng(4), B, vocab)
    ids = torch.from_numpy(np.concatenate(list(feats.values()), 1)).to(DEV).contiguous()
    so = so.to(DEV)
    outp = torch.empty(B, S, D, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    st = L.stream_ptr(DEV)
    cfg = {"tables": S, "rows": V, "D": D, "B": B}
    us = timed(lambda: L.call("rs_embedding_fwd", L.ptr(table), V, D, L.ptr(ids), 0, ids.numel(),
                              L.ptr(so), S, L.ptr(outp), L.ptr(err), st), iters)
    report("rs_embedding_fwd", cfg, us, ids.numel() * (4 + 2 * 4 * D), out)


def criteo(iters, out):
    """Criteo TSV ingestion: line index + parse + vocab lookup over a ~45 MB synthetic text
    (algorithmic bytes: text read once, outputs written once)."""
    from recommender_amd.data import CriteoVocab, read_criteo_tsv
    from tests.criteo_text import make_tsv

    text = make_tsv(np.random.default_rng(4), 200_000, vocab=5000).encode()
    vocab = CriteoVocab.build(text)
    n = text.count(b"\n") + 1
    out_bytes = n * (26 * 8 + 13 * 4 + 4)
    us = timed(lambda: vocab.encode(text), max(3, iters // 4))
    cfg = {"lines": n, "text_MB": round(len(text) / 1e6, 1), "vocab": vocab.size,
           "includes": "pinned host->device copy of the text + 3 host syncs"}
    report("criteo_encode(host tsv->device ids)", cfg, us, len(text) + out_bytes, out)
    dtext = torch.frombuffer(bytearray(text), dtype=torch.uint8).to(DEV)
    us = timed(lambda: vocab.encode(dtext), iters)
    cfg = dict(cfg, includes="text already in HBM; line index + parse + lookup + 3 host syncs")
    report("criteo_encode(device tsv->ids)", cfg, us, len(text) + out_bytes, out)
    _, _, hashes, _ = read_criteo_tsv(dtext)
    us = timed(lambda: vocab.lookup(hashes), iters)
    report("rs_vocab_lookup", {"tokens": hashes.numel(), "capacity": vocab.capacity}, us,
           hashes.numel() * 16, out)


def textpipe(iters, out):
    """Ali-CCP join + vocab + encode and Amazon (DIEN) vocab + encode on
    synthetic text already in HBM, beside the oracle's CPU time for the same text. Algorithmic
    bytes: every text byte read once + the id / label outputs written once."""
    import time

    from oracle import textpipe as O
    from recommender_amd.data import AliCCPVocab, DienVocab, aliccp_join
    from recommender_amd.data.aliccp import parse_kv_csv
    from tests.textpipe_text import make_aliccp, make_amazon

    rng = np.random.default_rng(4)
    sk, cm = make_aliccp(rng, 100_000, 5_000, n_vals=3000)
    dsk = torch.frombuffer(bytearray(sk.encode()), dtype=torch.uint8).to(DEV)
    dcm = torch.frombuffer(bytearray(cm.encode()), dtype=torch.uint8).to(DEV)
    rows = aliccp_join(dsk, dcm)
    vocab = AliCCPVocab.build(rows)

    def full():
        r = aliccp_join(dsk, dcm)
        v = AliCCPVocab.build(r)
        return v.encode(r)

    us = timed(full, max(3, iters // 4))
    t0 = time.perf_counter()
    orows = O.aliccp_join(sk, cm)
    O.aliccp_encode(orows, O.aliccp_vocab(orows))
    cpu_s = time.perf_counter() - t0
    nbytes = dsk.numel() + dcm.numel() + rows.n * (18 * 4 + 8)
    cfg = {"skeleton_lines": sk.count("\n"), "common_lines": cm.count("\n"), "kept": rows.n,
           "text_MB": round((dsk.numel() + dcm.numel()) / 1e6, 1), "vocab": sum(vocab.sizes),
           "oracle_cpu_s": round(cpu_s, 3),
           "includes": "parse both files, map, join, count, collect, sort, assign, encode; 6 host syncs"}
    report("aliccp_pipeline(device csv->ids)", cfg, us, nbytes, out)
    us = timed(lambda: parse_kv_csv(dsk, 3, 5, True), iters)
    report("rs_kv_parse(skeleton, incl. line index)", {"lines": cfg["skeleton_lines"]}, us,
           dsk.numel() + rows.n * 18 * 9, out)

    text = make_amazon(rng, 100_000, n_items=60_000, n_cats=800, max_hist=100)
    dt = torch.frombuffer(bytearray(text.encode()), dtype=torch.uint8).to(DEV)
    v = DienVocab.build(dt)

    def dien_full():
        vv = DienVocab.build(dt)
        return vv.encode(dt, 100, sample_negative=True, seed=4)

    us = timed(dien_full, max(3, iters // 4))
    t0 = time.perf_counter()
    items, cats, i2c = O.dien_vocab(text)
    O.dien_encode(text, items, cats, 100)
    cpu_s = time.perf_counter() - t0
    n = text.count("\n")
    nbytes = dt.numel() + n * (4 * 100 * 4 + 12)
    cfg = {"lines": n, "maxlen": 100, "text_MB": round(dt.numel() / 1e6, 1),
           "items": v.items.size, "cats": v.cats.size, "oracle_cpu_s_without_negatives": round(cpu_s, 3),
           "includes": "parse (2 passes), 2 vocab builds, item->cat map, encode + negatives; 5 host syncs"}
    report("dien_pipeline(device text->ids)", cfg, us, nbytes, out)
    us = timed(lambda: v.encode(dt, 100, sample_negative=True, seed=4), iters)
    report("dien_encode(device text->ids, vocab built)", {"lines": n}, us, nbytes, out)


def dlrm_path(iters, out):
    """The north-star embedding path's four launches run alone and back to back on one stream
    (no co-running GEMMs), at the bench config: 26 slots over a 40M x 128 fp32 slab, batch
    65 536, Zipf ids. SGD with lr 0 so repeated applies move the same bytes without drifting.
    Bytes: SURVEY §8(d) per-kernel formulas (bench.py kernel_bytes); path = §8(d) whole-path."""
    from bench import kernel_bytes
    from recommender_amd.optim import SortedIds
    from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

    S, D, B, V = 26, 128, 65536, 40_000_000
    cards = criteo_cardinalities(V, S)
    so = torch.tensor(np.concatenate([[0], np.cumsum(cards)]), dtype=torch.int64, device=DEV)
    table = torch.empty(V, D, device=DEV)
    table.uniform_(-0.05, 0.05)
    cat, _, _ = criteo_batch(np.random.default_rng(4), B, cards)
    ids = torch.from_numpy(cat).to(DEV)
    dense = torch.randn(B, D, device=DEV)
    Z = 27 * 26 // 2 + D
    inter = torch.empty(B, 512, device=DEV)
    gout = torch.randn(B, 512, device=DEV) * 1e-3
    gemb = torch.empty(B * S, D, device=DEV)
    gden = torch.empty(B, D, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    st = L.stream_ptr(torch.device(DEV))
    s0 = SortedIds(ids, V, so, err, count_unique=True)
    U = int(s0.n_unique.item())
    ws = torch.empty(L.lib().rs_apply_workspace_size(B * S, D), dtype=torch.uint8, device=DEV)
    prm = L.AdamParams(0.0, 0.0, 0.0, 0.0, 0.0, 0.0)

    def fwd():
        L.call("rs_dlrm_interaction_fwd", L.ptr(table), V, D, L.ptr(ids), 1, S, L.ptr(so),
               L.ptr(dense), B, 1, L.ptr(inter), 512, L.ptr(err), st)

    srows = torch.empty(B * S, dtype=torch.int32, device=DEV)
    spos = torch.empty(B * S, dtype=torch.int32, device=DEV)
    sws = torch.empty(L.lib().rs_sort_ids_workspace_size(B * S), dtype=torch.uint8, device=DEV)

    def srt():  # raw C call on preallocated buffers (no per-call Python allocation)
        L.call("rs_sort_ids", L.ptr(ids), 1, B * S, L.ptr(so), S, V, L.ptr(srows), L.ptr(spos),
               None, L.ptr(err), L.ptr(sws), sws.numel(), st)

    def bwd():
        L.call("rs_dlrm_interaction_bwd", L.ptr(table), V, D, L.ptr(ids), 1, S, L.ptr(so),
               L.ptr(dense), B, 1, L.ptr(gout), 512, L.ptr(gemb), L.ptr(gden), st)

    def apply():
        L.call("rs_embedding_apply", L.RS_OPT_SGD, L.ptr(table), None, None, V, D, L.ptr(s0.rows),
               L.ptr(s0.pos), B * S, L.ptr(gemb), prm, None, L.ptr(ws), ws.numel(), st)

    # the production path (fused forward + unit backward, sort, scaled apply)
    q = torch.randn(480, device=DEV) * 0.05
    cc = torch.zeros(1, device=DEV)
    yv = torch.empty(B, 1, device=DEV)
    G = torch.randn(B, device=DEV) * 1e-3

    xin = torch.rand(B, 13, device=DEV)
    lab = (torch.rand(B, device=DEV) < 0.25).float()
    sums = torch.empty(512 + 2 + 14 * 128, device=DEV)
    tws = torch.empty(L.lib().rs_dlrm_train_workspace_size(B), dtype=torch.uint8, device=DEV)
    yb = torch.empty(B, device=DEV)

    gb = torch.empty(B, device=DEV)

    def train_unit():
        L.call("rs_dlrm_train_step_fwd_unit", L.ptr(table), V, D, L.ptr(ids), 1, S, L.ptr(so),
               L.ptr(dense), L.ptr(xin), 13, L.ptr(lab), B, L.ptr(q), L.ptr(cc), 1e-7, 1.0 / B,
               L.ptr(yb), L.ptr(gemb), L.ptr(gb), L.ptr(sums), L.ptr(tws), tws.numel(), L.ptr(err),
               st)

    def apply_unit():
        L.call("rs_embedding_apply_scaled", L.RS_OPT_SGD, L.ptr(table), None, None, V, D,
               L.ptr(s0.rows), L.ptr(s0.pos), B * S, L.ptr(gemb), L.ptr(gb), S, prm, None,
               L.ptr(ws), ws.numel(), st)

    def fwd_dx():
        L.call("rs_dlrm_interaction_fwd_head_dx", L.ptr(table), V, D, L.ptr(ids), 1, S, L.ptr(so),
               L.ptr(dense), B, L.ptr(inter), 480, L.ptr(q), L.ptr(cc), 2, L.ptr(yv), L.ptr(gemb),
               L.ptr(gden), L.ptr(err), st)

    def apply_scaled():
        L.call("rs_embedding_apply_scaled", L.RS_OPT_SGD, L.ptr(table), None, None, V, D,
               L.ptr(s0.rows), L.ptr(s0.pos), B * S, L.ptr(gemb), L.ptr(G), S, prm, None,
               L.ptr(ws), ws.numel(), st)

    def apply_final():
        L.call("rs_embedding_apply_scaled", L.RS_OPT_SGD, L.ptr(table), None, None, V, D,
               L.ptr(s0.rows), L.ptr(s0.pos), B * S, L.ptr(gemb), None, 1, prm, None,
               L.ptr(ws), ws.numel(), st)

    bwd()
    cfg = {"B": B, "S": S, "D": D, "rows": V, "unique": U}
    per_ex = S * (8 + 8 * D) + S * (8 + 4 * D) + (U / B) * 8 * D
    # the chunked train kernel (unit rows + G, scaled apply)
    tot = 0.0
    for name, fn in (("rs_dlrm_train_step_fwd_unit", train_unit), ("rs_sort_ids", srt),
                     ("rs_embedding_apply_scaled", apply_unit)):
        us = timed(fn, iters)
        tot += us
        report(name + " (alone)", cfg, us, kernel_bytes(name, B, S, D, 8, U), out)
    report("embedding_path (chunked train kernel, sort, scaled apply; alone)",
           dict(cfg, bytes_per_example=round(per_ex, 1)), tot, per_ex * B, out)
    # the previous production path (fused forward + unit backward, scaled apply)
    tot = 0.0
    for name, fn in (("rs_dlrm_interaction_fwd_head_dx", fwd_dx), ("rs_sort_ids", srt),
                     ("rs_embedding_apply_scaled", apply_scaled)):
        us = timed(fn, iters)
        tot += us
        report(name + " (alone)", cfg, us, kernel_bytes(name, B, S, D, 8, U), out)
    report("embedding_path (fwd + unit bwd, scaled apply: 3 launches back to back, alone)",
           dict(cfg, bytes_per_example=round(per_ex, 1)), tot, per_ex * B, out)
    # the previous path (separate re-gathering backward), for the record
    tot = 0.0
    for name, fn in (("rs_dlrm_interaction_fwd", fwd), ("rs_sort_ids", srt),
                     ("rs_dlrm_interaction_bwd", bwd), ("rs_embedding_apply", apply)):
        us = timed(fn, iters)
        tot += us
        report(name + " (alone)", cfg, us, kernel_bytes(name, B, S, D, 8, U), out)
    report("embedding_path (fwd + re-gathering bwd: 4 launches back to back, alone)",
           dict(cfg, bytes_per_example=round(per_ex, 1)), tot, per_ex * B, out)


def sort_only(iters, out):
    """rs_sort_ids alone at the north-star batch (26 x 65 536 int64 ids over the 40M-row slab),
    called straight through the C ABI on preallocated buffers (no Python allocation per call)."""
    from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

    S, B, V = 26, 65536, 40_000_000
    cards = criteo_cardinalities(V, S)
    so = torch.tensor(np.concatenate([[0], np.cumsum(cards)]), dtype=torch.int64, device=DEV)
    ids = torch.from_numpy(criteo_batch(np.random.default_rng(4), B, cards)[0]).to(DEV)
    n = ids.numel()
    rows = torch.empty(n, dtype=torch.int32, device=DEV)
    pos = torch.empty(n, dtype=torch.int32, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    ws = torch.empty(L.lib().rs_sort_ids_workspace_size(n), dtype=torch.uint8, device=DEV)
    st = L.stream_ptr(torch.device(DEV))
    fn = lambda: L.call("rs_sort_ids", L.ptr(ids), 1, n, L.ptr(so), S, V, L.ptr(rows), L.ptr(pos),
                        None, L.ptr(err), L.ptr(ws), ws.numel(), st)
    us = timed(fn, iters)
    report("rs_sort_ids (raw C call)", {"n_ids": n, "rows": V}, us, n * 8 + n * 8, out)


def chain(iters, out):
    """rs_chain_reduce at the DLRM MLP shapes (factored backward): the top MLP's GEMV over the
    compact interaction row (n0 480, nl 1, sigmoid) and the bottom MLP's 13 x 128 outer
    reduction (relu). Bytes: x, dy, y read once (+ G written for the top)."""
    B = 65536
    for n0, nl, act, gout in ((480, 1, 2, True), (13, 128, 1, False)):
        x = torch.randn(B, n0, device=DEV)
        dy = torch.randn(B, nl, device=DEV)
        y = torch.rand(B, nl, device=DEV)
        o = torch.empty(n0 * nl + nl, device=DEV)
        g = torch.empty(B, nl, device=DEV) if gout else None
        nb = L.lib().rs_chain_reduce_workspace_size(B, n0, nl)
        ws = torch.empty(nb // 4 + 1, device=DEV)
        st = L.stream_ptr(torch.device(DEV))
        fn = lambda: L.call("rs_chain_reduce", L.ptr(x), n0, n0, L.ptr(dy), L.ptr(y), nl, act, B,
                            L.ptr(o), L.ptr(g), L.ptr(ws), ws.numel() * 4, st)
        us = timed(fn, iters)
        by = B * (n0 * 4 + 2 * nl * 4 + (nl * 4 if gout else 0))
        report("rs_chain_reduce", {"B": B, "n0": n0, "nl": nl, "act": act}, us, by, out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="dien,pinsage,pinsage_eval,eges,eges_sampler,embedding,criteo,textpipe")
    args = ap.parse_args()
    L.load()
    out = []
    for name in args.only.split(","):
        globals()[name](args.iters, out)


if __name__ == "__main__":
    main()
