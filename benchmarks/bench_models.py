"""Secondary benchmarks for the BASELINE.json configs other than the north star:
  cfg3 dien  : DIEN train step, B 4096, L 100, Amazon-Electronics-shaped vocab (63 001 / 801)
  cfg4 esmm  : MMOE (or ESMM) train step on 18 tables scaled to --rows, B 65 536 per GPU
  cfg1 deepfm: DeepFM, 1M-row shared table, B 1024, D 16 (the reference's CPU config, on GPU)
Prints one JSON line per run with examples/sec and per-kernel HIP-event times.
Usage: python benchmarks/bench_models.py --model dien|mmoe|esmm|deepfm [--steps K --warmup W]"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from recommender_amd import _lib as L  # noqa: E402


def run(step_fn, batches, steps, warmup, watch):
    for i in range(warmup):
        step_fn(*batches[i % len(batches)])
    timer = L.KernelTimer(watch)
    L.set_timer(timer)
    torch.cuda.synchronize()
    timer.enabled = True
    t0 = time.perf_counter()
    for i in range(steps):
        step_fn(*batches[i % len(batches)])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    timer.enabled = False
    L.set_timer(None)
    k = {n: round(ms / c * 1e3, 1) for n, (ms, c) in timer.totals_ms().items() if c}
    return dt / steps, k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="dien", choices=["dien", "mmoe", "esmm", "deepfm", "pinsage", "eges"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--rows", type=int, default=40_000_000)
    ap.add_argument("--tuned-gemms", type=int, default=-1,
                    help="1: replay the committed TunableOp GEMM choices (recommender_amd/gemm_tuning.py); "
                         "-1 (default): on for the fixed-shape models (dien, esmm, mmoe), off for the "
                         "variable-shape ones (pinsage, eges: 4.6 -> 10.8 ms, 1.16 -> 1.44 ms with it)")
    args = ap.parse_args()
    L.load()
    if args.tuned_gemms == 1 or (args.tuned_gemms < 0 and args.model in ("dien", "esmm", "mmoe")):
        from recommender_amd.gemm_tuning import use_tuned_gemms

        use_tuned_gemms()
    dev = "cuda"
    rng = np.random.default_rng(4)
    if args.model == "dien":
        from recommender_amd.dien import DIEN
        from recommender_amd.dien.train import DIENStep, synthetic_batch

        B = args.batch or 4096
        m = DIEN(36, 36, item_vocab_size=63001, item_embedding_size=18, cat_vocab_size=801,
                 cat_embedding_size=18, mlp_units=[200, 80, 1], device=dev)
        step = DIENStep(m)
        batches = []
        for _ in range(4):
            f, lab = synthetic_batch(rng, B, 100, 63001, 801)
            batches.append(({k: torch.from_numpy(v).to(dev) for k, v in f.items()}, torch.from_numpy(lab).to(dev)))
        watch = ["rs_gru_fwd", "rs_gru_bwd", "rs_augru_fwd", "rs_augru_bwd", "rs_dien_attention_fwd",
                 "rs_dien_attention_bwd", "rs_embedding_fwd", "rs_embedding_apply", "rs_keras_adam_dense_sweep"]
        cfg = {"workload": "dien_amazon_b4096_l100", "batch": B, "hist_len": 100, "gru_units": 36}
    elif args.model in ("mmoe", "esmm"):
        from recommender_amd.esmm import FEAT_VOCAB
        from recommender_amd.esmm.train import MultiTaskStep, build
        from recommender_amd.synthetic import aliccp_batch, scaled_vocab

        B = args.batch or 65536
        vocab = scaled_vocab(FEAT_VOCAB, args.rows)
        m = build(args.model.upper(), vocab, 18, dev)
        step = MultiTaskStep(m, "lazy_adam")
        batches = []
        for _ in range(4):
            f, lab = aliccp_batch(rng, B, vocab)
            batches.append(({k: torch.from_numpy(v).to(dev) for k, v in f.items()}, torch.from_numpy(lab).to(dev)))
        watch = ["rs_embedding_fwd", "rs_sort_ids", "rs_embedding_apply"]
        cfg = {"workload": f"{args.model}_aliccp_18x{args.rows}x18", "batch": B, "optimizer": "lazy_adam"}
    elif args.model == "pinsage":
        from recommender_amd.pinsage import PinSageModel, PinSageSampler
        from recommender_amd.pinsage.sampler import item_pairs
        from recommender_amd.pinsage.train import ML20M, PinSageStep, build_graph

        B = args.batch or 4096
        g = build_graph(ML20M, 4)
        m = PinSageModel(g, g.itype, 2, 8, 32, 16)
        train = PinSageStep(m)
        smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
        ctr = {"step": 0}

        def step(_):
            h, p, n = item_pairs(g, B, 4, ctr["step"])
            ctr["step"] += 1
            return train(*smp.sample_from_item_pairs(h, p, n))

        batches = [(None,)]
        watch = ["rs_item_pairs", "rs_pinsage_neighbors", "rs_unique_first", "rs_pinsage_block",
                 "rs_weighted_mean_agg_fwd", "rs_weighted_mean_agg_bwd",
                 "rs_frobenius_normalize_fwd", "rs_frobenius_normalize_bwd", "rs_embedding_fwd",
                 "rs_embedding_apply", "rs_keras_adam_dense_sweep"]
        cfg = {"workload": "pinsage_ml20m_b4096", "batch": B, "walk": [2, 4, 0, 3],
               "graph_edges": g.n_edges}
    elif args.model == "eges":
        from recommender_amd.eges.train import EGESStep, build, synthetic_batch

        B = args.batch or 1024
        n_items, n_cat, n_brand = 63001, 801, 3000
        m = build("EGES", n_items, n_cat, n_brand, 160)
        train = EGESStep(m)
        batches = []
        for _ in range(4):
            *inp, lab = synthetic_batch(rng, B, n_items, n_cat, n_brand)
            batches.append((tuple(torch.from_numpy(a).to(dev) for a in inp),
                            torch.from_numpy(lab).to(dev)))
        step = train
        watch = ["rs_embedding_fwd", "rs_side_pool_fwd", "rs_side_pool_bwd", "rs_match_logits_fwd",
                 "rs_match_logits_bwd", "rs_sort_ids", "rs_embedding_apply",
                 "rs_keras_adam_dense_sweep"]
        cfg = {"workload": "eges_b1024_d160_ns5", "batch": B, "items": n_items}
    else:
        from recommender_amd.ctr.train import TrainStep, build_model
        from recommender_amd.synthetic import criteo_batch

        B = args.batch or 1024
        m = build_model("DeepFM", 16, 1_000_000, 26, 13, dev)
        step0 = TrainStep(m, "keras_adam", fused=False)
        batches = []
        for _ in range(4):
            cat, dn, lb = criteo_batch(rng, B, [1_000_000] * 26)
            batches.append(((torch.from_numpy(cat).to(dev), torch.from_numpy(dn).to(dev), torch.from_numpy(lb).to(dev)),))
        step = step0
        watch = ["rs_embedding_fwd", "rs_fm_fwd", "rs_fm_bwd", "rs_sort_ids", "rs_embedding_apply",
                 "rs_keras_adam_dense_sweep"]
        cfg = {"workload": "deepfm_criteo_1M_b1024_d16", "batch": B, "optimizer": "keras_adam"}
    sec, k = run(step, batches, args.steps, args.warmup, watch)
    print(json.dumps({"model": args.model, "examples_per_sec": round(B / sec, 1),
                      "ms_per_step": round(sec * 1e3, 3), "config": cfg, "kernels_us": k}))


if __name__ == "__main__":
    main()
