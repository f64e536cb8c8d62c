"""Secondary benchmarks for the BASELINE.json configs other than the north star:
  cfg3 dien  : DIEN train step, B 4096, L 100, Amazon-Electronics-shaped vocab (63 001 / 801)
  cfg4 esmm  : MMOE (or ESMM) train step on 18 tables scaled to --rows, B 65 536 per GPU
  cfg1 deepfm: DeepFM, 1M-row shared table, B 1024, D 16 (the reference's CPU config, on GPU),
              with the oracle's NumPy step timed on the host beside it (cpu_baseline)
  cfg2 dlrm_cfg2: DLRM, 26 per-slot tables x 10M rows x D 64 in one 66.6 GB slab, B 8192,
              bottom [512, 256, 64], top [512, 256, 1], Zipf(1.05) ids, --optimizer sgd|lazy_adam|keras_adam
Prints one JSON line per run with examples/sec and per-kernel HIP-event times.
Usage: python benchmarks/bench_models.py --model dien|mmoe|esmm|deepfm|dlrm_cfg2 [--steps K --warmup W]"""
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
    ap.add_argument("--model", default="dien",
                    choices=["dien", "mmoe", "esmm", "deepfm", "deepfm_file", "pinsage", "eges",
                             "dlrm_cfg2"])
    ap.add_argument("--file-rows", type=int, default=1_000_000,
                    help="deepfm_file: rows of the Criteo-shaped TFRecord file written and trained on")
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "lazy_adam", "keras_adam"],
                    help="dlrm_cfg2 only (the reference DLRM SGD path or Keras / lazy Adam)")
    ap.add_argument("--cfg4-optimizer", default="keras_adam_deferred",
                    choices=["keras_adam_deferred", "keras_adam", "lazy_adam"],
                    help="esmm / mmoe: the reference's Keras Adam (esmm/train.py:125) with each "
                         "row's dense decay replayed when next read (default; its materialize() "
                         "is timed and amortised into the value), the same with the per-step "
                         "dense sweep, or lazy Adam (touched rows only; also reported as the "
                         "secondary key of the default run)")
    ap.add_argument("--cpu-baseline", type=int, default=1,
                    help="1: time the oracle's host step (the reference's CPU path restated) "
                         "beside the GPU step and report it under cpu_baseline")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--rows", type=int, default=40_000_000)
    ap.add_argument("--pinsage-mode", default="graph_all",
                    choices=["dynamic", "static", "graph", "graph_all"],
                    help="pinsage: dynamic = host-synced shapes (PinSageStep.__call__); static = "
                         "capacity-shaped sync-free batches, eager (static_step); graph = the same "
                         "step captured once and replayed (PinSageStep.capture), sampling eager; "
                         "graph_all = sampling inside the graph too (capture_with_sampling)")
    ap.add_argument("--deepfm-mode", default="graph", choices=["eager", "graph"],
                    help="deepfm: graph = the Keras-Adam step captured once as a HIP graph and replayed "
                         "(TrainStep.capture_static); eager: TrainStep.__call__")
    ap.add_argument("--dien-mode", default="graph", choices=["eager", "graph"],
                    help="dien: eager = DIENStep.__call__; graph = static_step captured once and "
                         "replayed (DIENStep.capture)")
    ap.add_argument("--eges-mode", default="graph", choices=["eager", "graph"],
                    help="eges: eager = EGESStep.__call__ (SparseAdam keras); graph = static_step "
                         "captured once and replayed (EGESStep.capture)")
    ap.add_argument("--cfg2-graph", type=int, default=2,
                    help="dlrm_cfg2 (sgd): 0 = eager steps; 1 = each step a HIP-graph replay "
                         "(TrainStep.capture); 2 (default, as the other launch-bound configs) = "
                         "the 4-batch pool as one graph (TrainStep.capture_sequence, updates "
                         "overlapped across steps), timed per step")
    ap.add_argument("--tuned-gemms", type=int, default=-1,
                    help="1: replay the committed TunableOp GEMM choices (recommender_amd/gemm_tuning.py); "
                         "-1 (default): on for the fixed-shape models (dien, esmm, mmoe), off for the "
                         "variable-shape ones (pinsage, eges: 4.6 -> 10.8 ms, 1.16 -> 1.44 ms with it)")
    args = ap.parse_args()
    L.load()
    if args.model == "deepfm_file":
        return deepfm_from_file(args)
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
        if args.dien_mode == "graph":
            st_f = {k: torch.empty_like(v) for k, v in batches[0][0].items()}
            st_l = torch.empty_like(batches[0][1])
            dctr = {"n": 0, "replay": None}
            train_d = step

            def step(f, lab):
                # the feed's refill of the static buffers: one multi-tensor copy
                torch._foreach_copy_([st_f[k] for k in f] + [st_l], list(f.values()) + [lab])
                dctr["n"] += 1
                if dctr["n"] == 1:
                    return train_d.static_step(st_f, st_l)
                if dctr["replay"] is None:
                    dctr["replay"] = train_d.capture(st_f, st_l)
                return dctr["replay"]()
        watch = ["rs_gru_fwd", "rs_gru_bwd", "rs_augru_fwd", "rs_augru_bwd", "rs_dien_attention_fwd",
                 "rs_dien_attention_bwd", "rs_embedding_fwd", "rs_embedding_apply", "rs_keras_adam_dense_sweep"]
        cfg = {"workload": "dien_amazon_b4096_l100", "batch": B, "hist_len": 100, "gru_units": 36,
               "mode": args.dien_mode}
    elif args.model in ("mmoe", "esmm"):
        from recommender_amd.esmm import FEAT_VOCAB
        from recommender_amd.esmm.train import MultiTaskStep, build
        from recommender_amd.synthetic import aliccp_batch, scaled_vocab

        B = args.batch or 65536
        vocab = scaled_vocab(FEAT_VOCAB, args.rows)
        m = build(args.model.upper(), vocab, 18, dev)
        cfg4_train = step = MultiTaskStep(m, args.cfg4_optimizer)
        batches = []
        for _ in range(4):
            f, lab = aliccp_batch(rng, B, vocab)
            batches.append(({k: torch.from_numpy(v).to(dev) for k, v in f.items()}, torch.from_numpy(lab).to(dev)))
        watch = ["rs_embedding_fwd", "rs_sort_ids_slots", "rs_embedding_apply",
                 "rs_embedding_apply_scaled", "rs_keras_adam_catchup", "rs_keras_adam_dense_sweep"]
        cfg = {"workload": f"{args.model}_aliccp_18x{args.rows}x18", "batch": B,
               "optimizer": args.cfg4_optimizer}
    elif args.model == "pinsage":
        from recommender_amd.pinsage import PinSageModel, PinSageSampler
        from recommender_amd.pinsage.sampler import item_pairs
        from recommender_amd.pinsage.train import ML20M, PinSageStep, build_graph

        B = args.batch or 4096
        g = build_graph(ML20M, 4)
        m = PinSageModel(g, g.itype, 2, 8, 32, 16)
        train = PinSageStep(m)
        smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
        ctr = {"step": 0, "replay": None}

        def step(_):
            it = ctr["step"]
            ctr["step"] += 1
            if args.pinsage_mode == "dynamic":
                h, p, n = item_pairs(g, B, 4, it)
                return train(*smp.sample_from_item_pairs(h, p, n))
            if args.pinsage_mode == "graph_all" and it > 0:
                if ctr["replay"] is None:
                    ctr["replay"] = train.capture_with_sampling(smp, B, 4, it)
                return ctr["replay"]()
            batch = smp.sample_static(*smp.sample_pairs_static(B, 4, it))
            if args.pinsage_mode == "static" or it == 0:
                return train.static_step(*batch)
            if ctr["replay"] is None:
                ctr["replay"] = train.capture(batch)
            return ctr["replay"]()

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
        if args.eges_mode == "graph":
            # static input buffers refilled from the batch pool, then one graph replay per step
            st_in = tuple(torch.empty_like(a) for a in batches[0][0])
            st_lab = torch.empty_like(batches[0][1])
            gctr = {"n": 0, "replay": None}

            def step(inp, lab):
                torch._foreach_copy_(list(st_in) + [st_lab], list(inp) + [lab])
                gctr["n"] += 1
                if gctr["n"] == 1:
                    return train.static_step(st_in, st_lab)
                if gctr["replay"] is None:
                    gctr["replay"] = train.capture(st_in, st_lab)
                return gctr["replay"]()
        watch = ["rs_embedding_fwd", "rs_side_pool_fwd", "rs_side_pool_bwd", "rs_match_logits_fwd",
                 "rs_match_logits_bwd", "rs_sort_ids", "rs_embedding_apply",
                 "rs_keras_adam_dense_sweep"]
        cfg = {"workload": "eges_b1024_d160_ns5", "batch": B, "items": n_items,
               "mode": args.eges_mode}
    elif args.model == "dlrm_cfg2":
        from recommender_amd.ctr.train import TrainStep, build_model
        from recommender_amd.synthetic import criteo_batch

        B = args.batch or 8192
        S, D, per = 26, 64, 10_000_000
        cards = [per] * S
        m = build_model("DLRM", D, per * S, S, 13, torch.device(dev), slot_cardinalities=cards,
                        bottom=[512, 256, D], top=[512, 256, 1])
        step0 = TrainStep(m, args.optimizer, lr=0.01 if args.optimizer == "sgd" else 1e-3,
                          fused=True, defer_sparse_join=True)
        batches = []
        for _ in range(4):
            cat, dn, lb = criteo_batch(rng, B, cards)
            batches.append(((torch.from_numpy(cat).to(dev), torch.from_numpy(dn).to(dev),
                             torch.from_numpy(lb).to(dev)),))
        step = step0
        cfg2_batches = list(batches)
        if args.cfg2_graph and args.optimizer == "sgd":
            for b in batches:  # eager warm-up (compositions, caches) before capture
                step0(*b)
            if args.cfg2_graph == 1:
                reps = [step0.capture(*b) for b in batches]
                gc = {"n": 0}

                def step(_):
                    r = reps[gc["n"] % len(reps)]
                    gc["n"] += 1
                    return r()
            else:
                seq = step0.capture_sequence([b[0] for b in batches])
                B_pool = len(batches)
                batches = [(None,)]
                args.steps = max(1, args.steps // B_pool)
                args.warmup = max(1, args.warmup // B_pool)

                def step(_):
                    return seq()
        watch = ["rs_dlrm_train_step_fwd_unit", "rs_sort_ids", "rs_embedding_apply",
                 "rs_dlrm_dense_tail", "rs_keras_adam_dense_sweep"]
        cfg = {"workload": f"dlrm_criteo_26x{per}x{D}_b{B}", "batch": B, "rows": per * S,
               "slab_GB": round(per * S * D * 4 / 1e9, 1), "optimizer": args.optimizer,
               "graph": args.cfg2_graph if args.optimizer == "sgd" else 0}
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
        if args.deepfm_mode == "graph":
            # the launch-bound B = 1024 step as one HIP graph (TrainStep.capture_static), replayed
            # on static input buffers refilled per batch
            static = tuple(torch.empty_like(t) for t in batches[0][0])
            fctr = {"n": 0, "replay": None}

            def step(b):
                torch._foreach_copy_(list(static), list(b))
                fctr["n"] += 1
                if fctr["n"] == 1:
                    return step0.static_step(static)
                if fctr["replay"] is None:
                    fctr["replay"] = step0.capture_static(static)
                return fctr["replay"]()
        watch = ["rs_embedding_fwd", "rs_fm_fwd", "rs_fm_bwd", "rs_sort_ids", "rs_embedding_apply",
                 "rs_keras_adam_dense_sweep"]
        cfg = {"workload": "deepfm_criteo_1M_b1024_d16", "batch": B, "optimizer": "keras_adam",
               "mode": args.deepfm_mode}
    sec, k = run(step, batches, args.steps, args.warmup, watch)
    if args.model == "dlrm_cfg2" and args.cfg2_graph == 2 and args.optimizer == "sgd":
        sec /= B_pool  # one replay = the whole pool of steps
    extra = {}
    dense_fl = None
    if args.model in ("esmm", "mmoe"):
        # the dense layers' GEMM work (forward, input gradient and weight gradient of every Dense
        # layer, 2·in·out FLOP each per example), counted before the model is released below
        from recommender_amd.nn import Dense

        dense_fl = sum(6.0 * B * l.kernel.shape[0] * l.kernel.shape[1]
                       for l in m.modules() if isinstance(l, Dense) and l.kernel is not None)
    if args.model in ("esmm", "mmoe") and args.cfg4_optimizer == "keras_adam_deferred":
        # the replayed decay of every row not touched since the start: materialize() brings the
        # slab to the dense sweep's state; its time is amortised over every step run so far
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cfg4_train.materialize()
        torch.cuda.synchronize()
        mat = time.perf_counter() - t0
        extra["steps_only_ms_per_step"] = round(sec * 1e3, 3)
        extra["materialize_ms"] = round(mat * 1e3, 2)
        extra["materialize_amortised_over_steps"] = args.steps + args.warmup
        sec = sec + mat / (args.steps + args.warmup)
        # lazy Adam (touched rows only, not the reference's update rule) as the secondary key
        del cfg4_train, step
        m = None
        torch.cuda.empty_cache()
        from recommender_amd.esmm.train import MultiTaskStep, build

        m2 = build(args.model.upper(), vocab, 18, dev)
        lz = MultiTaskStep(m2, "lazy_adam")
        sec_l, _ = run(lz, batches, args.steps, args.warmup, [])
        extra["lazy_adam"] = {"examples_per_sec": round(B / sec_l, 1),
                              "ms_per_step": round(sec_l * 1e3, 3),
                              "note": "touched rows only: not the reference's Keras Adam"}
        del lz, m2
    out = {"model": args.model, "examples_per_sec": round(B / sec, 1),
           "ms_per_step": round(sec * 1e3, 3), "config": cfg, "kernels_us": k, **extra}
    if args.cpu_baseline:
        fns = {"deepfm": lambda: deepfm_cpu_baseline(B),
               "dlrm_cfg2": cfg2_cpu_baseline,
               "dien": dien_cpu_baseline,
               "esmm": lambda: esmm_cpu_baseline("esmm", args.rows),
               "mmoe": lambda: esmm_cpu_baseline("mmoe", args.rows),
               "pinsage": pinsage_cpu_baseline,
               "eges": eges_cpu_baseline}
        try:
            out["cpu_baseline"] = fns[args.model]()
        except Exception as e:  # reported, not fatal: the GPU line stands on its own
            out["cpu_baseline"] = {"error": repr(e)[:300]}
    if args.model == "dlrm_cfg2":
        # SURVEY 8(d)'s path bytes per step at the measured unique-row count (fwd S(id + 8D) +
        # bwd S(id + 4D) + (U/B)·8D per example) over the WHOLE step time (dense half included:
        # a lower bound on the path's own fraction, which graph replay does not time apart)
        S_, D_ = 26, 64
        offs = torch.arange(S_, device=dev, dtype=torch.int64) * per
        Us = [int(torch.unique(b[0][0].reshape(-1, S_).to(torch.int64) + offs).numel())
              for b in cfg2_batches]
        U = sum(Us) / len(Us)
        by = B * (S_ * (8 + 8 * D_) + S_ * (8 + 4 * D_)) + U * 8 * D_
        gbs = by / sec / 1e9
        out["roofline"] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s",
                           "frac": round(gbs / 8000.0, 4), "algorithmic_bytes_per_step": int(by),
                           "unique_rows_per_step": U, "note": "path bytes / whole step time"}
    if args.model == "deepfm":
        # cfg1's bytes per step: Keras Adam's dense sweep of the 1M x 16 table (table, m, v read
        # and written: 24·V·D B — the reference's update touches every row every step) plus the
        # lookup and its gradient rows (B·26·(8 B id + 4D read + 4D gradient)), over the whole
        # replayed step (MLPs and glue included in the time)
        V_, D_ = 1_000_000, 16
        by = 24 * V_ * D_ + B * 26 * (8 + 8 * D_)
        gbs = by / sec / 1e9
        out["roofline"] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s",
                           "frac": round(gbs / 8000.0, 4), "algorithmic_bytes_per_step": int(by),
                           "note": "dense Keras Adam sweep + lookup/gradient bytes / whole step time"}
    if args.model == "eges":
        # every table densified and updated by Keras Adam each step (GraphKerasAdam: parameter,
        # m, v read and written = 24 B per element, the densified gradient written and read =
        # 8 B): 32 B per parameter element, over the whole replayed step
        n_el = sum(t.weight.numel() for t in m.tables())  # the tables are the variables
        by = 32 * n_el
        gbs = by / sec / 1e9
        out["roofline"] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s",
                           "frac": round(gbs / 8000.0, 4), "algorithmic_bytes_per_step": int(by),
                           "parameters": int(n_el),
                           "note": "dense Keras Adam over every table / whole step time"}
    if args.model == "dien":
        out["roofline"] = dien_roofline(args, train_d if args.dien_mode == "graph" else step,
                                        batches, B, sec)
    if args.model == "pinsage":
        out["roofline"] = pinsage_roofline(train, smp, B, sec)
    if args.model in ("esmm", "mmoe"):
        # the dense layers' GEMM work against the fp32 MFMA peak (157.3 TF/s: no xf32 on gfx950)
        # — the floor the library fp32 GEMMs set for the step
        fl = dense_fl
        floor_ms = fl / 157.3e12 * 1e3
        out["roofline"] = {"bound": "mfma_fp32", "dense_gflop_per_step": round(fl / 1e9, 1),
                           "achieved_TFs": round(fl / sec / 1e12, 1), "peak_TFs": 157.3,
                           "frac": round(floor_ms / (sec * 1e3), 4),
                           "floor_ms_at_peak": round(floor_ms, 3),
                           "note": "the whole step's time over its dense GEMM FLOPs (embedding, "
                                   "apply and elementwise work included in the time)"}
    print(json.dumps(out))


def dien_roofline(args, ds, batches, B, sec):
    """cfg3's step against what bounds it. The four recurrences (GRU / AUGRU, forward and
    backward) walk L = 100 dependent steps each, so their figure is µs per dependent step
    (timed on two eager static_steps after the run: graph replays record no kernel events);
    the step's GEMM-shaped arithmetic (recurrences' input and recurrent products, the aux net on
    its live rows, the head MLP: forward + both backward products, 6·in·out FLOP per row) is
    set against the fp32 MFMA peak (157.3 TF/s, no xf32 on gfx950) over the whole step."""
    names = ["rs_gru_fwd", "rs_gru_bwd", "rs_augru_fwd", "rs_augru_bwd", "rs_dien_aux_fwd",
             "rs_dien_aux_bwd_acc", "rs_dien_attention_fwd", "rs_dien_attention_bwd"]
    timer = L.KernelTimer(names)
    L.set_timer(timer)
    timer.enabled = True
    for f, lab in batches[:2]:
        ds.static_step(f, lab)
    torch.cuda.synchronize()
    timer.enabled = False
    L.set_timer(None)
    kt = {n: round(ms / c * 1e3, 1) for n, (ms, c) in timer.totals_ms().items() if c}
    L_, H, E = 100, 36, 36
    rec_us = sum(kt.get(n, 0.0) for n in names[:4])
    # the aux net's live rows: history steps t whose next step t + 1 is not padding (mask_zero)
    live = float((batches[0][0]["pos_his_item"][:, 1:] != 0).sum())
    rows = B * L_  # the recurrences as Keras runs them: every step of every history, masked
    fl = 6.0 * rows * (E * 3 * H + H * 3 * H) * 2          # GRU + AUGRU: x·W and h·U
    fl += 6.0 * 2 * live * ((H + E) * 80 + 80 * 40 + 40)   # aux net, pos + neg, live rows
    head_in = 2 * E + 2 * H + E + 18                        # the head's concat width (approx.)
    fl += 6.0 * B * (head_in * 200 + 200 * 80 + 80)
    return {"bound": "latency (4 recurrences x L = 100 dependent steps)",
            "recurrences_us": round(rec_us, 1),
            "us_per_dependent_step": round(rec_us / (4 * L_), 3),
            "kernels_us_eager": kt,
            "gemm_gflop_per_step": round(fl / 1e9, 2), "achieved_TFs": round(fl / sec / 1e12, 2),
            "peak_TFs": 157.3, "frac": round(fl / sec / 157.3e12, 4),
            "note": "frac = GEMM-shaped FLOPs / whole step time vs the fp32 MFMA peak; the step "
                    "is bound by the recurrences' dependent chains, not by FLOPs or bytes"}


def pinsage_roofline(train, smp, B, sec):
    """cfg5's step in HBM bytes (algorithmic, the live sizes of one sampled batch): the metapath
    walks (per seed 4 walks x 2 item-user-item steps, each hop an indptr pair + a neighbour:
    20 B), the two SAGE layers' weighted mean aggregation forward and backward (per live edge a
    source row read, 4·H B, each way; per destination its row written / read), the item
    features (id / year lookups + genre multi-hot mean) of every source node forward and
    backward, and Keras Adam over every variable (GraphKerasAdam: 32 B per element). Over the
    whole replayed step; the step is bound by dependent random loads (the walks) and launches."""
    batch = smp.sample_static(*smp.sample_pairs_static(B, 4, 10_000))
    _, _, blocks = batch
    torch.cuda.synchronize()
    H = 32
    by = 0
    for blk in blocks:
        n_dst = int(blk.n_dst_live.item()) if blk.n_dst_live is not None else blk.n_dst
        n_src = int(blk.n_src_live.item()) if blk.n_src_live is not None else blk.n_src
        n_e = int(blk.n_edges.item())
        by += n_dst * 4 * 2 * 20                    # the walks that sampled this block's sources
        by += 2 * (n_e * (4 * H + 12) + n_dst * 4 * H)  # aggregation forward + backward
        by += 2 * n_src * (8 + 4 * 16)              # item features of the sources, fwd + bwd
    n_el = sum(p.numel() for p in train.opt_graph.params) if getattr(train, "opt_graph", None) \
        else sum(p.numel() for p in train.dense)
    by += 32 * n_el
    gbs = by / sec / 1e9
    return {"bound": "hbm (latency: dependent walk loads)", "achieved": round(gbs, 1),
            "peak": 8000.0, "unit": "GB/s", "frac": round(gbs / 8000.0, 4),
            "algorithmic_bytes_per_step": int(by), "adam_elements": int(n_el),
            "note": "live-size algorithmic bytes of one sampled batch / whole replayed step"}


def deepfm_from_file(args):
    """cfg1 as BASELINE names it: ctr/train.py's DeepFM trained from a 1M-row Criteo-shaped
    TFRecord file (ctr/train.py:59-66: read_tfrecord → shuffle(100·batch) → batch(1024); DeepFM
    [512, 256, 1], D 16, joint 1M vocab, Keras Adam). The file is written by the engine's
    writer (the reference's tf.train.Example layout, tfrecord_io.py:66-75), read back by the
    device reader (host framing index + one wave per record parse, rs_tfrecord_parse_criteo),
    shuffled on the device (a seeded permutation: TF's 100·batch shuffle-buffer order is
    parity-unpinned) and trained for one epoch. Times each stage; the oracle's NumPy step is
    timed beside it (cpu_baseline)."""
    from recommender_amd.ctr.train import TrainStep, build_model
    from recommender_amd.data.tfrecord import read_tfrecord, write_tfrecord
    from recommender_amd.synthetic import criteo_batch

    dev = torch.device("cuda")
    n, B, V = args.file_rows, args.batch or 1024, 1_000_000
    rng = np.random.default_rng(4)
    cat, dn, lb = criteo_batch(rng, n, [V] * 26)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"cfg1_criteo_{n}.tfrecord")
    t0 = time.perf_counter()
    write_tfrecord(path, dn, cat, lb.astype(np.int64))
    t_write = time.perf_counter() - t0
    size = os.path.getsize(path)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    feats, label = read_tfrecord(path, dev)
    torch.cuda.synchronize()
    t_read = time.perf_counter() - t0
    ok = (torch.equal(feats["cat_features"].cpu(), torch.from_numpy(cat))
          and torch.equal(feats["int_features"].cpu(), torch.from_numpy(dn))
          and torch.equal(label.cpu(), torch.from_numpy(lb.astype(np.int64))))
    m = build_model("DeepFM", 16, V, 26, 13, dev)
    train = TrainStep(m, "keras_adam", fused=False)
    g = torch.Generator(device=dev).manual_seed(4)
    n_steps = n // B
    first = (feats["cat_features"][:B], feats["int_features"][:B], label[:B].float())
    if args.deepfm_mode == "graph":
        # the step captured once as a HIP graph (TrainStep.capture_static) and replayed on static
        # buffers refilled from each batch of the file
        static = tuple(torch.empty_like(t) for t in first)
        for d, s_ in zip(static, first):
            d.copy_(s_)
        train.static_step(static)
        replay = train.capture_static(static)

        def step(b):
            torch._foreach_copy_(list(static), list(b))
            return replay()
    else:
        step = train
    # warm-up on the first batches (library handles, workspaces), not counted in the epoch
    for i in range(3):
        step((feats["cat_features"][i * B:(i + 1) * B], feats["int_features"][i * B:(i + 1) * B],
              label[i * B:(i + 1) * B].float()))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    perm = torch.randperm(n, device=dev, generator=g)
    cats, dens, labs = (feats["cat_features"][perm], feats["int_features"][perm],
                        label[perm].float())
    loss = None
    for i in range(n_steps):
        sl = slice(i * B, (i + 1) * B)
        loss = step((cats[sl], dens[sl], labs[sl]))
    torch.cuda.synchronize()
    t_epoch = time.perf_counter() - t0
    out = {"model": "deepfm_file", "config": {"workload": f"deepfm_criteo_tfrecord_{n}_b{B}_d16",
                                                "rows": n, "batch": B, "optimizer": "keras_adam",
                                                "file_bytes": size, "mode": args.deepfm_mode},
           "examples_per_sec": round(n_steps * B / t_epoch, 1),
           "ms_per_step": round(t_epoch / n_steps * 1e3, 3),
           "examples_per_sec_incl_read": round(n_steps * B / (t_epoch + t_read), 1),
           "read_parse_s": round(t_read, 3), "read_GBs": round(size / t_read / 1e9, 2),
           "write_s": round(t_write, 2), "file_roundtrip_bit_exact": bool(ok),
           "epoch_steps": n_steps, "final_loss": float(loss),
           "cpu_baseline": deepfm_cpu_baseline(B)}
    os.remove(path)
    print(json.dumps(out))


def _host_threads():
    cores = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(cores, omp) if omp > 0 else cores


def _time_host(fn, n_warm, n_meas):
    """Median seconds of fn() over n_meas calls after n_warm, with the host's thread share (the
    box's OMP_NUM_THREADS for one GPU) given to torch and the BLAS pools; returns (s, threads)."""
    from threadpoolctl import threadpool_info, threadpool_limits

    threads = _host_threads()
    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    times = []
    try:
        with threadpool_limits(threads):
            used = max([i.get("num_threads", 1) for i in threadpool_info()] + [threads])
            for i in range(n_warm + n_meas):
                t0 = time.perf_counter()
                fn(i)
                if i >= n_warm:
                    times.append(time.perf_counter() - t0)
    finally:
        torch.set_num_threads(old)
    return float(np.median(times)), int(used)


def _baseline(B, sec, used, sample):
    return {"value": round(B / sec, 1), "unit": "examples/sec", "cores": used, "kind": "port",
            "sample": f"{sample}; median {sec * 1e3:.1f} ms/step"}


def cfg2_cpu_baseline(B=1024, rows_per_slot=100_000, n_warm=2, n_meas=5):
    """cfg2 on the host: oracle/ctr.py dlrm_sgd_step (NumPy fp32: gather, interaction, the
    [512, 256, 64] / [512, 256, 1] MLPs, BCE, backward, tiled dedup + SGD) at D 64, batch B,
    26 slots of rows_per_slot rows (a row's work does not depend on the table size)."""
    from oracle.ctr import DLRMState, dlrm_sgd_step
    from recommender_amd.synthetic import criteo_batch

    S, D = 26, 64
    rng = np.random.default_rng(4)
    cards = [rows_per_slot] * S
    so = np.concatenate([[0], np.cumsum(cards)]).astype(np.int64)
    table = rng.uniform(-0.05, 0.05, (int(so[-1]), D)).astype(np.float32)

    def mlp(fin, units):
        out = []
        for u in units:
            lim = np.sqrt(6.0 / (fin + u))
            out.append((rng.uniform(-lim, lim, (fin, u)).astype(np.float32), np.zeros(u, np.float32)))
            fin = u
        return out

    F = S + 1
    st = DLRMState(table, so, mlp(13, [512, 256, D]), mlp(F * F + D, [512, 256, 1]))
    pool = [criteo_batch(rng, B, cards) for _ in range(3)]

    def one(i):
        cat, dn, lb = pool[i % 3]
        dlrm_sgd_step(st, cat, dn, lb, 0.01)

    sec, used = _time_host(one, n_warm, n_meas)
    return _baseline(B, sec, used, f"oracle/ctr.py dlrm_sgd_step, D 64, batch {B}, 26 x "
                                   f"{rows_per_slot} rows, {n_warm} warm-up + {n_meas}")


def dien_cpu_baseline(B=64, n_warm=1, n_meas=3):
    """cfg3 on the host: oracle/dien.py dien_step (torch fp32 autograd on the CPU: GRU, aux
    loss, attention, AUGRU, head MLP — the reference's dien/train.py:14-22 forward + tape) plus
    the Keras Adam update of every dense parameter and of both tables (dense, as Keras does),
    on a CPU-built DIEN of the cfg3 shape, L 100."""
    from oracle.dien import dien_step
    from oracle.models import keras_adam_torch
    from oracle.embedding import keras_adam_coefficients
    from recommender_amd.dien import DIEN
    from recommender_amd.dien.train import synthetic_batch

    m = DIEN(36, 36, item_vocab_size=63001, item_embedding_size=18, cat_vocab_size=801,
             cat_embedding_size=18, mlp_units=[200, 80, 1], device="cpu")
    rng = np.random.default_rng(4)
    pool = []
    for _ in range(2):
        f, lab = synthetic_batch(rng, B, 100, 63001, 801)
        pool.append(({k: torch.from_numpy(v) for k, v in f.items()}, torch.from_numpy(lab)))
    state = {}

    def one(i):
        feats, lab = pool[i % 2]
        r = dien_step(m, feats, lab, dtype=torch.float32)
        c = {k: float(v) for k, v in keras_adam_coefficients(i + 1).items()}
        named = dict(m.named_parameters())
        with torch.no_grad():
            for n, g in r["grads"].items():
                p = named[n]
                mm, vv = state.get(n, (torch.zeros_like(p), torch.zeros_like(p)))
                w2, mm, vv = keras_adam_torch(p, mm, vv, g, c)
                p.copy_(w2)
                state[n] = (mm, vv)
            for t in (m.item_embedding, m.cat_embedding):  # Keras Adam on the whole table
                w = t.weight
                mm, vv = state.get(id(t), (torch.zeros_like(w), torch.zeros_like(w)))
                w2, mm, vv = keras_adam_torch(w, mm, vv, torch.zeros_like(w), c)
                w.copy_(w2)
                state[id(t)] = (mm, vv)

    sec, used = _time_host(one, n_warm, n_meas)
    return _baseline(B, sec, used, f"oracle/dien.py dien_step (torch fp32 autograd, CPU) + Keras "
                                   f"Adam of the dense parameters and both tables, batch {B}, "
                                   f"L 100, {n_warm} warm-up + {n_meas}")


def esmm_cpu_baseline(kind, rows, B=2048, n_warm=1, n_meas=3):
    """cfg4 on the host: oracle/models.py esmm_family_step (torch fp32 autograd on the CPU) of a
    CPU-built ESMM / MMOE over the same 18-table slab (`rows` rows, D 18), then the reference
    optimizer (esmm/train.py:125, Keras Adam): the dense parameters, and the slab's tiled dedup
    (oracle segment_sum_tiled) + Keras Adam over every row (m, v decayed densely)."""
    from oracle import embedding as OE
    from oracle.models import esmm_family_step, keras_adam_torch
    from recommender_amd.esmm import FEAT_VOCAB
    from recommender_amd.esmm.train import build
    from recommender_amd.synthetic import aliccp_batch, scaled_vocab

    vocab = scaled_vocab(FEAT_VOCAB, rows)
    m = build(kind.upper(), vocab, 18, "cpu")
    slab = m.embedding_layer.slab
    rng = np.random.default_rng(4)
    pool = []
    for _ in range(2):
        f, lab = aliccp_batch(rng, B, vocab)
        pool.append(({k: torch.from_numpy(v) for k, v in f.items()}, torch.from_numpy(lab)))
    so = slab.slot_offsets.numpy()
    table = slab.weight.numpy()
    mt, vt = np.zeros_like(table), np.zeros_like(table)
    dense = [p for n, p in m.named_parameters() if not n.endswith("grad_handle")]
    dstate = [(torch.zeros_like(p), torch.zeros_like(p)) for p in dense]

    def one(i):
        nonlocal table, mt, vt
        feats, lab = pool[i % 2]
        loss, y, dg, rows_g = esmm_family_step(m, slab.weight, slab.slot_offsets, feats, lab)
        co = OE.keras_adam_coefficients(i + 1)
        c = {k: float(v) for k, v in co.items()}
        with torch.no_grad():
            for j, (p, g) in enumerate(zip(dense, dg)):
                w2, mm, vv = keras_adam_torch(p, dstate[j][0], dstate[j][1], g, c)
                p.copy_(w2)
                dstate[j] = (mm, vv)
        ids = np.stack([feats[k].reshape(-1).numpy() for k in feats], 1)
        sr, sp, _ = OE.sort_ids(ids, table.shape[0], so)
        ur, ug = OE.segment_sum_tiled(sr, sp, rows_g.numpy(), table.shape[0])
        t2, mt, vt = OE.apply_keras_adam(table, mt, vt, ur.astype(np.int64), ug, co)
        table[...] = t2

    sec, used = _time_host(one, n_warm, n_meas)
    return _baseline(B, sec, used, f"oracle/models.py esmm_family_step (torch fp32 autograd, "
                                   f"CPU) + Keras Adam (dense parameters; slab: tiled dedup + "
                                   f"dense m / v sweep over all {table.shape[0]} rows), "
                                   f"{kind.upper()}, batch {B}, {n_warm} warm-up + {n_meas}")


def pinsage_cpu_baseline(B=256, n_warm=1, n_meas=3):
    """cfg5 on the host: the sampling of oracle/pinsage.py (item pairs, metapath walks, visit
    counts, top-k, to_block; NumPy) and oracle/pinsage.py torch_train_step (torch fp32 autograd,
    CPU) on a CPU-built PinSageModel over the same ML-20M-shaped graph, batch B pairs."""
    from oracle import pinsage as OP
    from recommender_amd.pinsage import PinSageModel
    from recommender_amd.pinsage.train import ML20M, build_graph

    g = build_graph(ML20M, 4, device="cpu")
    m = PinSageModel(g, g.itype, 2, 8, 32, 16, device="cpu")
    og = OP.BipartiteGraph(g.i2u_indptr.numpy(), g.i2u.numpy(), g.u2i_indptr.numpy(),
                           g.u2i.numpy())
    year = m.feature_projector.year.numpy()
    genre = m.feature_projector.genre.numpy()

    def one(i):
        heads, pos, neg = OP.item_pairs(og, i * B, B, 4, i)
        seeds, pe, ne, blocks = OP.sample_from_item_pairs(og, heads, pos, neg, 2, 4, 2, 0.0, 3, 4, i)
        OP.torch_train_step(m, blocks, pe, ne, year, genre)

    sec, used = _time_host(one, n_warm, n_meas)
    return {"value": round(B / sec, 1), "unit": "pairs/sec", "cores": used, "kind": "port",
            "sample": f"oracle/pinsage.py sampling (NumPy) + torch_train_step (torch fp32 autograd, "
                      f"CPU), batch {B} pairs, {n_warm} warm-up + {n_meas}; median "
                      f"{sec * 1e3:.1f} ms/step"}


def eges_cpu_baseline(B=1024, n_warm=2, n_meas=5):
    """EGES on the host: oracle/models.py eges_step (torch fp32 autograd, CPU) of a CPU-built
    EGES (63 001 items, D 160, 5 negatives) plus Keras Adam of its tables (dense, as Keras)."""
    from oracle.models import eges_step, keras_adam_torch
    from oracle.embedding import keras_adam_coefficients
    from recommender_amd.eges.train import build, synthetic_batch

    m = build("EGES", 63001, 801, 3000, 160, device="cpu")
    rng = np.random.default_rng(4)
    pool = []
    for _ in range(2):
        *inp, lab = synthetic_batch(rng, B, 63001, 801, 3000)
        pool.append((tuple(torch.from_numpy(a) for a in inp), torch.from_numpy(lab)))
    state = {}

    def one(i):
        inp, lab = pool[i % 2]
        loss, logits, out = eges_step(m, inp, lab)
        c = {k: float(v) for k, v in keras_adam_coefficients(i + 1).items()}
        with torch.no_grad():
            for name, (ids, rows) in out.items():
                w = getattr(m, name).weight
                g = torch.zeros_like(w).index_add_(0, ids, rows)
                mm, vv = state.get(name, (torch.zeros_like(w), torch.zeros_like(w)))
                w2, mm, vv = keras_adam_torch(w, mm, vv, g, c)
                w.copy_(w2)
                state[name] = (mm, vv)

    sec, used = _time_host(one, n_warm, n_meas)
    return _baseline(B, sec, used, f"oracle/models.py eges_step (torch fp32 autograd, CPU) + "
                                   f"Keras Adam of every table, batch {B}, {n_warm} warm-up + "
                                   f"{n_meas}")


def deepfm_cpu_baseline(B, n_warm=5, n_meas=20):
    """cfg1 is the reference's CPU-only config: the oracle's NumPy DeepFM Keras-Adam step
    (oracle/ctr.py deepfm_keras_adam_step, the same 1M x 16 table, MLP [512, 256, 1]) timed on
    the host cores — warm-up 5, median of 20."""
    from threadpoolctl import threadpool_info, threadpool_limits

    from oracle.ctr import deepfm_keras_adam_step
    from recommender_amd.synthetic import criteo_batch

    rng = np.random.default_rng(4)
    V, D, S = 1_000_000, 16, 26
    cores = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(cores, omp) if omp > 0 else cores
    st = {"table": rng.uniform(-0.05, 0.05, (V, D)).astype(np.float32),
          "m": np.zeros((V, D), np.float32), "v": np.zeros((V, D), np.float32)}
    fin, layers = S * D + 13, []
    for u in (512, 256, 1):
        lim = np.sqrt(6.0 / (fin + u))
        layers.append((rng.uniform(-lim, lim, (fin, u)).astype(np.float32), np.zeros(u, np.float32)))
        fin = u
    st["layers"] = layers
    st["dense_m"] = [(np.zeros_like(k), np.zeros_like(b)) for k, b in layers]
    st["dense_v"] = [(np.zeros_like(k), np.zeros_like(b)) for k, b in layers]
    pool = [criteo_batch(rng, B, [V] * S) for _ in range(4)]
    times = []
    with threadpool_limits(threads):
        used = max([i.get("num_threads", 1) for i in threadpool_info()] + [1])
        for i in range(n_warm + n_meas):
            cat, dn, lb = pool[i % 4]
            t0 = time.perf_counter()
            _, st2, _ = deepfm_keras_adam_step(st["table"], st["m"], st["v"], st["layers"],
                                               st["dense_m"], st["dense_v"], cat % V, dn, lb, i + 1)
            if i >= n_warm:
                times.append(time.perf_counter() - t0)
            st.update(st2)
    med = float(np.median(times))
    return {"value": round(B / med, 1), "unit": "examples/sec", "cores": int(used), "kind": "port",
            "sample": f"oracle/ctr.py deepfm_keras_adam_step, batch {B}, {n_warm} warm-up + median "
                      f"of {n_meas} ({med * 1e3:.1f} ms/step)"}


if __name__ == "__main__":
    main()
