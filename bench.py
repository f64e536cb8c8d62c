"""North-star benchmark: Criteo-shaped DLRM train step (fwd + bwd + optimizer) on MI355X.

metric: examples/sec fwd+bwd, Criteo-DLRM 26×40M×128 batch 65536 (BASELINE.json): the global
batch 65 536 split over the ranks (strong scaling, the metric line); --scaling weak keeps 65 536
per GPU, and N > 1 also reports the weak-scaling rate as a secondary key. One step = DLRM forward (bottom MLP, fused gather +
MFMA DotInteraction, top MLP), mean BCE, backward (fused re-gather interaction bwd, MLPs),
dense SGD and the fused sparse SGD apply on the embedding slab (the reference's DLRM SGD path,
ctr/train.py:77-79). Inputs are pre-generated on device (no host I/O in the timed region).

Usage: python bench.py [--gpus N --steps K --warmup W]. N > 1: under torch.distributed.run
(WORLD_SIZE must equal N), or, when WORLD_SIZE is unset, bench.py launches torch.distributed.run
with N ranks itself as a child process before touching the GPU and exits with its status.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from datetime import timedelta

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from recommender_amd import _lib as L  # noqa: E402
from recommender_amd.ctr.layers import MLP  # noqa: E402
from recommender_amd.ctr.train import TrainStep, build_model  # noqa: E402
from recommender_amd.synthetic import criteo_batch, criteo_cardinalities  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
WATCH = ["rs_dlrm_train_step_fwd_unit", "rs_dlrm_train_step_fwd_unit_nofold",
         "rs_dlrm_interaction_fwd", "rs_dlrm_interaction_fwd_head",
         "rs_dlrm_interaction_fwd_head_dx",
         "rs_dlrm_interaction_bwd", "rs_dlrm_interaction_bwd_rank1", "rs_sort_ids_slots",
         "rs_embedding_apply", "rs_embedding_apply_scaled", "rs_sort_ids_sharded",
         "rs_embedding_dedup_grad", "rs_embedding_dedup_grad_mapped", "rs_gather_rows_padded",
         "rs_embedding_dedup_grad_mapped_range", "rs_exchange_classify", "rs_exchange_mark",
         "rs_exchange_scatter_late"]
# the embedding path of SURVEY §8(d) (lookup fwd + bwd + dedup + apply) as the production step
# launches it: the fused gather + interaction + unit-backward kernel (main stream), the radix
# sort and the segmented-sum apply (fused optimizer's side stream, co-running with dense GEMMs:
# their event spans include that co-run time)
PATH_KERNELS = ("rs_dlrm_train_step_fwd_unit",
                "rs_dlrm_interaction_fwd", "rs_dlrm_interaction_fwd_head",
                "rs_dlrm_interaction_fwd_head_dx", "rs_dlrm_interaction_bwd",
                "rs_dlrm_interaction_bwd_rank1", "rs_sort_ids_slots", "rs_sort_ids_sharded",
                "rs_embedding_apply", "rs_embedding_apply_scaled")
SIDE_STREAM = {"rs_sort_ids_slots", "rs_embedding_apply", "rs_embedding_apply_scaled",
               "rs_sort_ids_sharded", "rs_embedding_dedup_grad", "rs_embedding_dedup_grad_mapped",
               "rs_gather_rows_padded", "rs_embedding_dedup_grad_mapped_range",
               "rs_exchange_classify", "rs_exchange_mark", "rs_exchange_scatter_late"}
# device symbols behind each C-ABI entry (for the PMC passes)
# (entry, device-symbol regex of its kernels, the one kernel every call launches once)
PMC_SYMBOLS = [
    ("rs_dlrm_train_step_fwd_unit", r"dlrm_train_chunk", "dlrm_train_chunk"),
    ("rs_dlrm_interaction_fwd_head_dx", r"dlrm_fwd_dx_pipe", "dlrm_fwd_dx_pipe"),
    ("rs_dlrm_interaction_fwd_head", r"inter_fwd_mfma<128, rs::GatherSrc, true, true, false>",
     "inter_fwd_mfma"),
    ("rs_dlrm_interaction_bwd_rank1", r"dlrm_bwd_pipe", "dlrm_bwd_pipe"),
    # the slot-segmented sort's pass-0 histogram runs once per sort (the LSD form's pass-0
    # histogram, keys built from the ids, when a slab takes that form)
    ("rs_sort_ids_slots", r"slot_sort_|small_sort|radix_|scan_|count_unique",
     r"slot_sort_hist0_kernel|small_sort_kernel|radix_hist_kernel<\d+, true"),
    ("rs_embedding_apply", r"seg_tile|seg_group|seg_chunk|seg_fixup", "seg_tile|seg_group"),
]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # SURVEY 8(d) timing method: warm-up 10, measure 100 steps (0.1 s of GPU time)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=65536,
                    help="global batch (strong scaling) or per-GPU batch (--scaling weak)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong: the global batch is split over the ranks (the metric's fixed "
                         "global batch); weak: every rank runs --batch")
    ap.add_argument("--keras-line", type=int, default=1,
                    help="N = 1, SGD: also time the reference's active optimizer (Keras Adam with "
                         "the deferred exact decay) on the same model and report it under keras_adam")
    ap.add_argument("--weak-secondary", type=int, default=1,
                    help="N > 1, strong scaling: also time --batch per GPU (weak scaling) and "
                         "report it under weak_scaling")
    ap.add_argument("--rows", type=int, default=40_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--slots", type=int, default=26)
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "lazy_adam", "keras_adam"])
    ap.add_argument("--pool", type=int, default=4, help="distinct synthetic batches cycled")
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--cpu-baseline-steps", type=int, default=50)
    ap.add_argument("--cpu-baseline-batch", type=int, default=4096)
    ap.add_argument("--defer-decay", type=int, default=0,
                    help="keras_adam: replay the dense decay per row when it is next read instead "
                         "of sweeping all rows each step (exact after materialize)")
    ap.add_argument("--prefetch", type=int, default=-1,
                    help="1: the next batch's ids handled one step ahead (TrainStep.prefetch): one "
                         "GPU, its sort after this step's train kernel; row-sharded (--gpus > 1), "
                         "the exchange's sort / unique / split sizes, so the step's one host sync "
                         "waits on work queued a step earlier. -1 (default): on for --gpus > 1, off "
                         "for one GPU (measured: 0.745 vs 0.707 ms/step there, host-bound)")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: HIP-graph replays of single steps; 2: one graph per pool of steps "
                         "(updates overlapped across steps inside the graph)")
    ap.add_argument("--fused", type=int, default=1, help="fused side-stream sparse optimizer")
    ap.add_argument("--prio", type=int, default=0,
                    help="1: run the step on a high-priority HIP stream (side-stream work fills in)")
    ap.add_argument("--defer-join", type=int, default=1,
                    help="1: the sparse update joins at the next step's first table read "
                         "(overlaps the next bottom MLP) instead of at the end of the step")
    ap.add_argument("--mlp-bwd", default="factored", choices=["factored", "layerwise"],
                    help="ctr MLP backward: factored linear chain (default) or layer by layer")
    ap.add_argument("--mlp-fwd", default="composed", choices=["composed", "layerwise"],
                    help="ctr MLP forward on the chain path: the chain's single affine map "
                         "(default) or layer by layer")
    ap.add_argument("--compare-layerwise", type=int, default=1,
                    help="1: after the timed steps, also time the layer-by-layer MLP forward "
                         "(factored backward) and the fully layer-by-layer MLP")
    ap.add_argument("--tuned-gemms", type=int, default=1,
                    help="1: replay the committed TunableOp GEMM choices (recommender_amd/gemm_tuning.py)")
    ap.add_argument("--pmc-child", type=int, default=0,
                    help=argparse.SUPPRESS)  # internal: the PMC child run (timed steps only)
    ap.add_argument("--pmc", type=int, default=1,
                    help="1: measure the roofline kernel's HBM traffic with two rocprofv3 --pmc "
                         "child runs (FETCH_SIZE, WRITE_SIZE) before this process touches the GPU")
    return ap.parse_args()


PMC_KERNEL_REGEX = ("dlrm_train_chunk|inter_fwd_mfma|dlrm_fwd_dx_pipe|dlrm_bwd_pipe|slot_sort_|"
                    "small_sort|radix_|scan_|count_unique|seg_tile|seg_group|seg_chunk|seg_fixup")
FETCH_CORRECTION = 2.0  # MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE reports 1/2 of 16 B/lane reads


def measure_traffic(args):
    """HBM bytes per step of each embedding-path kernel family from PMC counters, collected as
    the microarchitecture guide prescribes: separate `rocprofv3 --pmc` passes for FETCH_SIZE and
    WRITE_SIZE (they do not fit one pass), kernel-filtered, on a short child run of this same
    benchmark (same config, 1 warm-up + 2 steps). Units are KiB; FETCH_SIZE is doubled (the
    path's gathers are 16 B/lane). Must run before this process initialises the GPU.
    Returns ({C-ABI entry: bytes per call}, detail)."""
    import csv
    import re
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, {"error": "rocprofv3 not found"}
    child = [sys.executable, os.path.abspath(__file__), "--steps", "2", "--warmup", "1",
             "--cpu-baseline-steps", "0", "--pmc", "0", "--batch", str(args.batch), "--rows",
             str(args.rows), "--dim", str(args.dim), "--slots", str(args.slots), "--optimizer",
             args.optimizer, "--pool", str(args.pool), "--seed", str(args.seed), "--fused",
             str(args.fused), "--defer-join", str(args.defer_join), "--mlp-bwd", args.mlp_bwd,
             "--mlp-fwd", args.mlp_fwd, "--compare-layerwise", "0", "--tuned-gemms",
             str(args.tuned_gemms), "--keras-line", "0", "--pmc-child", "1"]
    child_steps = 1 + 2  # warm-up + timed steps of the child: one launch of each main kernel each
    vals = {}
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        with tempfile.TemporaryDirectory() as d:
            cmd = [prof, "--pmc", counter, "--kernel-include-regex", PMC_KERNEL_REGEX, "-d", d,
                   "-o", "run", "--output-format", "csv", "--"] + child
            try:
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env)
            except subprocess.TimeoutExpired:
                return None, {"error": f"{counter} pass timed out"}
            if r.returncode != 0:
                return None, {"error": f"{counter} pass rc={r.returncode}: {r.stderr[-300:]}"}
            per, calls = {}, {}
            for root, _, files in os.walk(d):
                for f in files:
                    if f.endswith("counter_collection.csv"):
                        for row in csv.DictReader(open(os.path.join(root, f))):
                            if row["Counter_Name"] != counter:
                                continue
                            name = row.get("Kernel_Name", "")
                            for entry, pat, main in PMC_SYMBOLS:
                                if re.search(pat, name):
                                    per[entry] = per.get(entry, 0.0) + float(row["Counter_Value"])
                                    if re.search(main, name):
                                        calls[entry] = calls.get(entry, 0) + 1
                                    break
            if not per:
                return None, {"error": f"no {counter} rows"}
            # every family seen must have launched its main kernel once per child step: a
            # family total divided by a wrong count is not a per-call figure
            bad = {k: calls.get(k, 0) for k in per if calls.get(k, 0) != child_steps}
            if bad:
                return None, {"error": f"{counter}: main-kernel launches per family {bad}, "
                                       f"expected {child_steps} (the child's steps)"}
            # KiB → bytes per call of the C-ABI entry
            vals[counter] = {k: v * 1024.0 / calls[k] for k, v in per.items()}
    out, detail = {}, {}
    for k in set(vals["FETCH_SIZE"]) | set(vals["WRITE_SIZE"]):
        rd = vals["FETCH_SIZE"].get(k, 0.0) * FETCH_CORRECTION
        wr = vals["WRITE_SIZE"].get(k, 0.0)
        out[k] = rd + wr
        detail[k] = {"read_bytes": round(rd), "write_bytes": round(wr)}
    detail["method"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, "
                        f"--kernel-include-regex {PMC_KERNEL_REGEX}; per call (family total / "
                        f"launches of its main kernel), FETCH_SIZE x {FETCH_CORRECTION}")
    return out, detail


def init_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(local % max(ndev, 1))
        # RS_DIST_BACKEND=gloo: rehearse several ranks on one GPU (exchange staged through host)
        backend = os.environ.get("RS_DIST_BACKEND", "nccl")
        # a stuck collective ends the run with an error well inside the driver's limit (the
        # NCCL watchdog aborts the rank) instead of hanging for the 10-minute default
        to = timedelta(seconds=int(os.environ.get("RS_DIST_TIMEOUT_S", "180")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=to)
        else:
            dist.init_process_group(backend, timeout=to)
    return world, rank, local


def exchange_info(emb):
    """The row-sharded exchange's counters over the run: capacity, spill rounds, the
    rows-ahead modes and, on late steps, the share of the capacity block re-sent after the
    previous step's apply."""
    late = getattr(emb, "late_slots", [0, 0])
    return {"capacity": getattr(emb, "capacity", None), "spill_rounds": getattr(emb, "spill_rounds", 0),
            "rows_ahead_modes": dict(getattr(emb, "rows_ahead_modes", {})),
            "late_fraction": round(late[0] / late[1], 4) if late[1] else None,
            "split_halves": bool(getattr(emb, "split_halves", False))}


def barrier(world):
    if world > 1:
        dist.barrier()


def make_pool(args, cards, rank, dev, batch=None):
    rng = np.random.default_rng([args.seed, rank])
    pool = []
    for _ in range(args.pool):
        cat, dn, lb = criteo_batch(rng, batch or args.batch, cards)
        pool.append((torch.from_numpy(cat).to(dev), torch.from_numpy(dn).to(dev),
                     torch.from_numpy(lb).to(dev)))
    return pool


def measured_unique(pool, model):
    from recommender_amd.optim import SortedIds

    t = model.embedding_layer
    us = [int(SortedIds(b[0], t.input_dim, t.slot_offsets).n_unique.item()) for b in pool]
    return float(np.mean(us))


def kernel_bytes(name, B, S, D, id_bytes, U, world=1, cap=0):
    """Algorithmic HBM bytes of one launch. The interaction row is the
    compact one: F(F-1)/2 pair values + D bottom values (the zero padding is not counted).
    world > 1 (row-sharded slab; B = the per-rank batch, U = its unique rows,
    cap = the exchange capacity): the owner's sort and apply run over the E = world·cap received
    slots, of which ≈U hold rows (each rank sends every owner ≈U/world rows); the owner's
    distinct rows are taken as ≈U too (an upper bound: ranks that share a row send it twice)."""
    F = S + 1
    N = B * S
    Z = F * (F - 1) // 2 + D
    if world > 1:
        E = world * cap
        if name == "rs_sort_ids_sharded":
            return N * id_bytes + N * 8
        if name == "rs_embedding_dedup_grad_mapped":  # rank-local sum per unique row into its slot
            return N * 8 + N * 4 * D + U * 4 * D
        if name == "rs_sort_ids_slots":  # the owner's masked sort of the received slots
            return E * (4 + 1) + E * 8
        if name == "rs_embedding_apply":  # E sorted entries, ≈U rows read, their rows updated
            return E * 8 + U * 4 * D + U * 2 * 4 * D
        if name == "rs_gather_rows_padded":  # the owner serves the requested rows (the early
            # block; a late round's call moves only its C_late slots, so the average overstates)
            return E * 4 + E * 2 * 4 * D
        if name == "rs_embedding_dedup_grad_mapped_range":  # one owner half of the dedup
            return (N * 8 + N * 4 * D + U * 4 * D) // 2
        if name == "rs_exchange_classify":  # slots, stamps read, the late lists written
            return E * 4 + E * 4 + E * 8
        if name == "rs_exchange_mark":  # one requested-slot block (or a spill block)
            return E * 4 + E * 4
    if name == "rs_dlrm_interaction_fwd":
        return B * (S * id_bytes + S * 4 * D + 4 * D + 4 * Z)
    if name == "rs_dlrm_interaction_fwd_head":  # + the fused top-MLP output y[b]
        return B * (S * id_bytes + S * 4 * D + 4 * D + 4 * Z + 4)
    if name == "rs_dlrm_interaction_bwd":
        return B * (S * id_bytes + S * 4 * D + 4 * D + 4 * Z + S * 4 * D + 4 * D)
    if name == "rs_dlrm_interaction_bwd_rank1":  # grad row = G[b] * p: 4 B per example, not 4Z
        return B * (S * id_bytes + S * 4 * D + 4 * D + 4 + S * 4 * D + 4 * D)
    if name in ("rs_dlrm_train_step_fwd_unit", "rs_dlrm_train_step_fwd_unit_nofold"):
        # ids, rows, bottom row, 13 inputs + label in;
        # y, G[b] and the S unit gradient rows out (the batch sums are weight-sized)
        return B * (S * id_bytes + S * 4 * D + 4 * D + 13 * 4 + 4 + 4 + 4 + S * 4 * D)
    if name == "rs_dlrm_interaction_fwd_head_dx":  # + the unit gradient rows (S + 1 per example)
        return B * (S * id_bytes + S * 4 * D + 4 * D + 4 * Z + 4 + S * 4 * D + 4 * D)
    if name == "rs_embedding_apply":
        return N * 8 + N * 4 * D + U * 2 * 4 * D
    if name == "rs_embedding_apply_scaled":  # + G[b] when the step hands unit rows (4 B/example)
        return N * 8 + N * 4 * D + U * 2 * 4 * D
    if name in ("rs_sort_ids_slots", "rs_sort_ids"):
        return N * id_bytes + N * 8
    return 0


def isolated_path(model, ids, iters=10):
    """The production embedding path's three launches run alone and back to back on the main
    stream, after the timed region, on the model's own slab, ids and workspaces: the fused
    train-step kernel (gather + interaction + head + BCE + gradient rows + batch sums, with its
    block fold), the radix sort, the segmented-sum SGD apply with lr 0 (the table does not move;
    the same bytes are read and written). Each is
    timed with HIP events over `iters` launches on the stream it is launched on. In the step the
    sort and the apply run on the side stream beside other kernels, so their in-step event spans
    include co-run time; these isolated averages are what the roofline divides by."""
    torch.cuda.synchronize()  # the last step's deferred side-stream update has landed
    emb = model.embedding_layer
    w, so, err = emb.weight, emb.slot_offsets, emb.err_flag
    V, D = w.shape
    ids = ids.contiguous()
    B, S = ids.shape
    dev = w.device
    st = L.stream_ptr(dev)
    nzc = (S + 1) * S // 2 + D
    g = torch.Generator(device=dev).manual_seed(7)
    dense = torch.rand(B, D, device=dev, generator=g)
    q = torch.randn(nzc, device=dev, generator=g) * 0.05
    cc = torch.zeros(1, device=dev)
    y = torch.empty(B, device=dev)
    dxu = torch.empty(B * S, D, device=dev)
    xin = torch.rand(B, 13, device=dev, generator=g)
    lab = (torch.rand(B, device=dev, generator=g) < 0.25).float()
    sums = torch.empty(512 + 2 + 14 * 128, device=dev)
    tws = torch.empty(L.lib().rs_dlrm_train_workspace_size(B), dtype=torch.uint8, device=dev)
    n = B * S
    rows = torch.empty(n, dtype=torch.int32, device=dev)
    pos = torch.empty(n, dtype=torch.int32, device=dev)
    sws = torch.empty(L.lib().rs_sort_ids_workspace_size(n), dtype=torch.uint8, device=dev)
    aws = torch.empty(L.lib().rs_apply_workspace_size(n, D), dtype=torch.uint8, device=dev)
    prm = L.AdamParams(0.0, 0.0, 0.0, 0.0, 0.0, 0.0)
    gb = torch.empty(B, device=dev)
    train = ("rs_dlrm_train_step_fwd_unit", lambda: L.call(
        "rs_dlrm_train_step_fwd_unit", L.ptr(w), V, D, L.ptr(ids), L.id_dtype_code(ids), S,
        L.ptr(so), L.ptr(dense), L.ptr(xin), 13, L.ptr(lab), B, L.ptr(q), L.ptr(cc), 1e-7,
        1.0 / B, L.ptr(y), L.ptr(dxu), L.ptr(gb), L.ptr(sums), L.ptr(tws), tws.numel(),
        L.ptr(err), st))
    calls = {
        train[0]: train[1],
        "rs_sort_ids_slots": lambda: L.call(
            "rs_sort_ids_slots", L.ptr(ids), L.id_dtype_code(ids), n, None, L.ptr(so), S, V,
            emb.max_slot_rows, L.ptr(rows), L.ptr(pos), None, L.ptr(err), L.ptr(sws), sws.numel(),
            st),
        "rs_embedding_apply_scaled": lambda: L.call(
            "rs_embedding_apply_scaled", L.RS_OPT_SGD, L.ptr(w), None, None, V, D, L.ptr(rows),
            L.ptr(pos), n, L.ptr(dxu), L.ptr(gb), S, prm, None,
            L.ptr(aws), aws.numel(), st),
    }
    out = {}
    for name, fn in calls.items():
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) / iters * 1e3
    return out


def cpu_baseline(args, cards):
    """The oracle's NumPy DLRM SGD step (oracle/ctr.py) on the host cores, bounded sample
    (warm-up 5 steps, then the median of 50, on len(sched_getaffinity) cores)."""
    from threadpoolctl import threadpool_info, threadpool_limits

    from oracle.ctr import DLRMState, dlrm_sgd_step

    cores = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(cores, omp) if omp > 0 else cores  # the box caps its CPU share via OMP_NUM_THREADS
    D, S = args.dim, args.slots
    rng = np.random.default_rng(args.seed)
    V = sum(cards)
    table = np.empty((V, D), np.float32)
    table[:] = np.float32(0.01)
    so = np.concatenate([[0], np.cumsum(cards)]).astype(np.int64)

    def mk(units, fin):
        out = []
        for u in units:
            lim = np.sqrt(6.0 / (fin + u))
            out.append((rng.uniform(-lim, lim, (fin, u)).astype(np.float32), np.zeros(u, np.float32)))
            fin = u
        return out

    F = S + 1
    st = DLRMState(table, so, mk([512, 256, D], 13), mk([512, 256, 1], F * F + D))
    B = args.cpu_baseline_batch
    n_warm, n_meas = 5, args.cpu_baseline_steps
    pool = [criteo_batch(rng, B, cards) for _ in range(4)]
    times = []
    with threadpool_limits(threads):
        used = max([i.get("num_threads", 1) for i in threadpool_info()] + [1])
        for i in range(n_warm + n_meas):
            t0 = time.perf_counter()
            dlrm_sgd_step(st, *pool[i % len(pool)], 0.01)
            if i >= n_warm:
                times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return {"value": B / med, "unit": "examples/sec", "cores": int(used),
            "kind": "port", "host_cpus_visible": cores,
            "cores_note": "threads = min(sched_getaffinity, OMP_NUM_THREADS): the GPU pool sets "
                          "OMP_NUM_THREADS to the host-core share of one GPU (16 on a 1-GPU box, "
                          "whose nproc shows the whole machine's cores)",
            "p10_p90_s": [round(float(np.percentile(times, 10)), 4), round(float(np.percentile(times, 90)), 4)],
            "sample": f"oracle/ctr.py dlrm_sgd_step (NumPy fp32, {used} BLAS threads), batch {B} on "
                      f"the same 26x{V}x{D} slab / Zipf ids: {n_warm} warm-up steps, then the median "
                      f"of {n_meas} ({med:.3f} s/step, {sum(times):.1f} s timed)"}


def launch_ranks(args) -> int:
    """--gpus N > 1 without an external launcher: run torch.distributed.run with N ranks as a
    child process (this process has not touched the GPU) and return its exit status."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        raise SystemExit(launch_ranks(args))
    if env_world is not None and int(env_world) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={env_world}: launch N ranks for "
                         "--gpus N (or leave WORLD_SIZE unset and bench.py launches them)")
    MLP.factored_backward = args.mlp_bwd == "factored"
    MLP.composed_forward = args.mlp_fwd == "composed"
    traffic, traffic_detail = None, None
    if args.pmc and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        traffic, traffic_detail = measure_traffic(args)  # before any GPU initialisation
    world, rank, local = init_dist(args)
    requested_batch = args.batch
    if args.scaling == "strong":
        if args.batch % world:
            raise SystemExit("strong scaling: --batch must be divisible by the number of ranks")
        args.batch //= world  # from here on args.batch is the per-GPU batch
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    L.load()
    if L.lib().rs_device_count() < 1:
        raise SystemExit("no GPU visible to librecsys_hip")
    if args.tuned_gemms:
        from recommender_amd.gemm_tuning import use_tuned_gemms

        use_tuned_gemms()
    D, S = args.dim, args.slots
    cards = criteo_cardinalities(args.rows, S)
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed)
    comm = None
    if world > 1:
        # row-sharded slab over the ranks (RCCL all-to-all), data-parallel dense MLPs
        from recommender_amd.ctr.model import DLRM
        from recommender_amd.sharded import Comm, ShardedSlabEmbedding

        comm = Comm()
        g.manual_seed(args.seed + 1000 * rank)
        emb = ShardedSlabEmbedding(cards, D, comm, device=dev, generator=g)
        g.manual_seed(args.seed)
        model = DLRM([512, 256, D], [512, 256, 1], D, args.rows, S, 13, device=dev,
                     generator=g, embedding_layer=emb)
    else:
        model = build_model("DLRM", D, args.rows, S, 13, dev, slot_cardinalities=cards,
                            bottom=[512, 256, D], top=[512, 256, 1], generator=g)
    step = TrainStep(model, args.optimizer, lr=0.01 if args.optimizer == "sgd" else 1e-3,
                     fused=bool(args.fused), comm=comm, defer_sparse_join=bool(args.defer_join),
                     defer_decay=bool(args.defer_decay))
    pool = make_pool(args, cards, rank, dev)
    # the PMC child counts one launch of each path kernel per step: no extra sorts here
    U = 0.0 if args.pmc_child else measured_unique(pool, model)

    if args.prio:
        hp = torch.cuda.Stream(device=dev, priority=-1)
        hp.wait_stream(torch.cuda.current_stream(dev))
        torch.cuda.set_stream(hp)
    P = len(pool)
    if args.prefetch < 0:
        args.prefetch = 1 if world > 1 else 0
    if args.prefetch and not args.graph:
        # the loader's next batch is on the device a step early: its sort is queued one step
        # ahead (TrainStep.prefetch), beside the current step's kernels
        def runner(i):
            step.prefetch(pool[(i + 1) % P])
            return step(pool[i])

        runners = [lambda i=i: runner(i) for i in range(P)]
    else:
        runners = [lambda b=b: step(b) for b in pool]
    for i in range(args.warmup):
        runners[i % P]()
    per_call = 1
    if args.graph == 1:
        runners = [step.capture(b) for b in pool]
    elif args.graph == 2:
        # the pool's steps as one graph (per-step updates overlapped inside it); a remainder of
        # steps that does not fill a whole graph runs through single-step graphs
        runners = [step.capture_sequence(pool)]
        singles = [step.capture(b) for b in pool]
        per_call = len(pool)
    # the timed steps run with no per-kernel instrumentation; the in-step kernel spans
    # (`kernels`) come from a second, instrumented pass over the same steps afterwards
    timer = L.KernelTimer(WATCH)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    if per_call > 1:
        for _ in range(args.steps // per_call):
            loss = runners[0]()
        for i in range(args.steps % per_call):
            loss = singles[i]()
    else:
        for i in range(args.steps):
            loss = runners[i % len(runners)]()
    ev1.record()
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    wall = t1 - t0
    if world > 1:
        tt = torch.tensor([wall], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall = float(tt.item())
    materialize_ms = None
    if getattr(step.opt_sparse, "defer_decay", False):
        # outside the timed region: bring every row up to date (what a checkpoint or an
        # evaluation pass needs), timed on its own
        torch.cuda.synchronize()
        tm0 = time.perf_counter()
        step.opt_sparse.materialize()
        torch.cuda.synchronize()
        materialize_ms = round((time.perf_counter() - tm0) * 1e3, 3)
    if materialize_ms is not None:
        # the deferred decay the timed steps left behind belongs to them: amortise it
        wall += materialize_ms * 1e-3
    ms_step = wall / args.steps * 1e3
    value = args.batch * world * args.steps / wall
    if args.pmc_child:  # the counters cover the warm-up + timed steps only
        if world > 1:
            dist.destroy_process_group()
        return

    # the same steps with the layer-by-layer MLP forward, and with the MLPs entirely layer by
    # layer (the reference's evaluation order), for the record: same model, same batches, timed
    # the same way
    def time_variant(factored, composed):
        MLP.factored_backward, MLP.composed_forward = factored, composed
        for i in range(2):
            step(pool[i % len(pool)])
        torch.cuda.synchronize()
        barrier(world)
        ta = time.perf_counter()
        for i in range(args.steps):
            step(pool[i % len(pool)])
        torch.cuda.synchronize()
        barrier(world)
        lw = time.perf_counter() - ta
        if world > 1:
            tt = torch.tensor([lw], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            lw = float(tt.item())
        return round(lw / args.steps * 1e3, 3)

    # per-step distribution (after the timed region, same steps): intervals between consecutive
    # step starts on the main stream (the deferred update overlaps the next step, so this is the
    # steady-state step time), reported as p10 / median / p90 (SURVEY 8(d) timing method)
    step_dist = None
    if per_call == 1 and args.steps >= 4:
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        for i in range(args.steps):
            evs[i].record()
            loss = runners[i % len(runners)]()
        evs[-1].record()
        torch.cuda.synchronize()
        raw = [round(evs[i].elapsed_time(evs[i + 1]), 3) for i in range(args.steps)]
        d = sorted(raw)
        q = lambda f: round(d[min(len(d) - 1, int(f * (len(d) - 1) + 0.5))], 3)  # noqa: E731
        step_dist = {"p10": q(0.1), "median": q(0.5), "p90": q(0.9), "steps": args.steps,
                     "ms": raw}

    # instrumented pass: HIP-event span of every watched kernel inside the steps
    L.set_timer(timer)
    timer.enabled = True
    if per_call > 1:
        for _ in range(args.steps // per_call):
            loss = runners[0]()
    else:
        for i in range(args.steps):
            loss = runners[i % len(runners)]()
    torch.cuda.synchronize()
    timer.enabled = False
    L.set_timer(None)

    layerwise_ms = layerwise_fwd_ms = None
    if args.compare_layerwise and args.mlp_bwd == "factored" and not args.graph:
        if args.mlp_fwd == "composed":
            layerwise_fwd_ms = time_variant(True, False)
        layerwise_ms = time_variant(False, False)
        MLP.factored_backward, MLP.composed_forward = True, args.mlp_fwd == "composed"

    tot = timer.totals_ms()
    kern = {}
    for name, (ms, cnt) in tot.items():
        if cnt:
            avg = ms / cnt
            by = kernel_bytes(name, args.batch, S, D, 8, U, world,
                              getattr(model.embedding_layer, "capacity", 0) or 0)
            kern[name] = {"avg_us": round(avg * 1e3, 2), "calls": cnt,
                          "algorithmic_bytes": int(by),
                          "achieved_GBs": round(by / (avg * 1e-3) / 1e9, 1),
                          "stream": "side (co-running)" if (name in SIDE_STREAM and (args.fused or world > 1)) else "main"}
    # headline roofline: the whole embedding path of SURVEY §8(d) — fwd S(id+8D) + bwd S(id+4D)
    # + (U/B)·8D bytes per example at the measured U — over the summed isolated launch times of
    # the production path's three kernels (world 1, fused composed-head path)
    per_ex = S * (8 + 8 * D) + S * (8 + 4 * D) + (U / args.batch) * 8 * D
    path_bytes = per_ex * args.batch
    roof = None
    if world == 1 and D == 128 and args.fused and args.mlp_fwd == "composed":
        iso = isolated_path(model, pool[0][0])
        path_us = sum(iso.values())
        a = path_bytes / (path_us * 1e-6) / 1e9
        pmc_key = {"rs_embedding_apply_scaled": "rs_embedding_apply"}
        per_kernel = {}
        for n_, us in iso.items():  # noqa: B007
            by = kernel_bytes(n_, args.batch, S, D, 8, U)
            t = (traffic or {}).get(pmc_key.get(n_, n_))
            per_kernel[n_] = {"avg_us": round(us, 2), "algorithmic_bytes": int(by),
                              "achieved_GBs": round(by / (us * 1e-6) / 1e9, 1),
                              "frac": round(by / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                              "traffic": round(t) if t is not None else None,
                              "in_step_span_us": kern.get(n_, kern.get(n_ + "_scaled", kern.get(
                                  n_ + "_nofold", {}))).get("avg_us")}
        tsum = sum(v["traffic"] for v in per_kernel.values()) if traffic and all(
            v["traffic"] is not None for v in per_kernel.values()) else None
        dom = max(iso, key=iso.get)
        # measured STREAM-copy bandwidth of this GPU: a 4 GiB device-to-device copy
        # with 16-byte accesses (rs_stream_copy; torch's copy_ measured ≈4.7 TB/s on the same
        # boxes, below the float4 copy's ≈6.3 TB/s the guide lists)
        src = torch.zeros(1 << 30, dtype=torch.float32, device=dev)
        dst = torch.empty_like(src)
        nb = src.numel() * 4
        st_ = L.stream_ptr(dev)
        L.call("rs_stream_copy", L.ptr(src), L.ptr(dst), nb, st_)
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record()
        for _ in range(10):
            L.call("rs_stream_copy", L.ptr(src), L.ptr(dst), nb, st_)
        c1.record()
        torch.cuda.synchronize()
        copy_gbs = 2 * nb * 10 / (c0.elapsed_time(c1) * 1e-3) / 1e9
        del src, dst
        roof = {"bound": "hbm", "kernel": "embedding_path (" + " + ".join(iso) + ")",
                "achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(a / HBM_PEAK_GBS, 4), "traffic": tsum,
                "algorithmic_bytes": int(path_bytes), "us_per_step": round(path_us, 1),
                "bytes_per_example": round(per_ex, 1), "unique_rows_per_step": U,
                "dominant_kernel": dom, "per_kernel": per_kernel,
                "measured_copy_GBs": round(copy_gbs, 1),
                "frac_of_measured_copy": round(a / copy_gbs, 4),
                "traffic_detail": traffic_detail,
                "note": "achieved = SURVEY 8(d) path bytes at measured U / the sum of the path "
                        "kernels' isolated launch times (HIP events, after the timed region, on "
                        "the model's slab and ids); in_step_span_us = the same kernel's HIP-event "
                        "span inside the timed steps (side-stream spans include co-run time); "
                        "traffic = PMC FETCH+WRITE per call; measured_copy_GBs = a 4 GiB "
                        "device copy with 16-byte accesses (rs_stream_copy; read + write bytes / "
                        "time), the STREAM-copy reference"}

    # the reference's active ctr optimizer (ctr/train.py:80,84: Keras Adam on every variable) on
    # the same model and batches, with the deferred exact decay (bit-identical to the per-step
    # dense sweep after materialize(); tests/test_northstar_gpu.py), for the record
    keras = None
    if world == 1 and args.keras_line and args.optimizer == "sgd" and not args.graph:
        torch.cuda.synchronize()
        kstep = TrainStep(model, "keras_adam", lr=1e-3, fused=True, defer_sparse_join=True,
                          defer_decay=True)
        for i in range(3):
            kstep(pool[i % len(pool)])
        torch.cuda.synchronize()
        tk0 = time.perf_counter()
        for i in range(args.steps):
            kstep(pool[i % len(pool)])
        torch.cuda.synchronize()
        tk = time.perf_counter() - tk0
        tm0 = time.perf_counter()
        kstep.opt_sparse.materialize()
        torch.cuda.synchronize()
        tmat = time.perf_counter() - tm0
        # value: the steps AND the deferred decay they left behind (materialize brings every row
        # to the dense sweep's state, bit for bit), amortised over the steps; the steps alone
        # beside it
        keras = {"value": round(args.batch * args.steps / (tk + tmat), 1), "unit": "examples/sec",
                 "ms_per_step": round((tk + tmat) / args.steps * 1e3, 3), "steps": args.steps,
                 "optimizer": "keras_adam (deferred exact decay, amortised)",
                 "materialize_ms_after_run": round(tmat * 1e3, 2),
                 "steps_only": {"value": round(args.batch * args.steps / tk, 1),
                                "ms_per_step": round(tk / args.steps * 1e3, 3),
                                "note": "excludes the deferred decay materialize() pays"},
                 "fused_step": bool(kstep.fused_step_ready(pool[0]))}
        # materialize replays only the (m, v) chunks that are not zero (a zero state decays to
        # itself, exactly): its cost grows with the rows the run has touched
        mt, vt, _ = kstep.opt_sparse._slots(model.embedding_layer)
        keras["rows_with_state"] = int(((mt.abs().amax(dim=1) + vt.abs().amax(dim=1)) != 0).sum())
        keras["rows"] = int(mt.shape[0])
        keras["materialize_note"] = ("the replay skips zero (m, v) state (the identity for any "
                                     "number of steps) without reading its weights; its cost "
                                     "grows with rows_with_state as a run touches more rows")
        del kstep, mt, vt
        torch.cuda.empty_cache()

    # N > 1 under strong scaling: the same step at --batch per GPU (weak scaling), for the record
    weak = None
    if world > 1 and args.scaling == "strong" and args.weak_secondary:
        wpool = make_pool(args, cards, rank, dev, batch=requested_batch)
        WP = len(wpool)
        emb = model.embedding_layer
        if hasattr(emb, "capacity"):
            emb.capacity = None  # the exchange capacity recalibrated on this batch size

        def wstep(i):
            if args.prefetch:
                step.prefetch(wpool[(i + 1) % WP])
            step(wpool[i % WP])

        for i in range(3):
            wstep(i)
        torch.cuda.synchronize()
        barrier(world)
        tw0 = time.perf_counter()
        for i in range(args.steps):
            wstep(i)
        torch.cuda.synchronize()
        barrier(world)
        tw = time.perf_counter() - tw0
        tt = torch.tensor([tw], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        tw = float(tt.item())
        weak = {"value": round(requested_batch * world * args.steps / tw, 1), "unit": "examples/sec",
                "per_gpu_batch": requested_batch, "global_batch": requested_batch * world,
                "ms_per_step": round(tw / args.steps * 1e3, 3), "steps": args.steps}
        del wpool

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline_steps > 0:
        cpu = cpu_baseline(args, cards)

    if rank == 0:
        out = {
            "metric": "examples/sec fwd+bwd, Criteo-DLRM 26×40M×128 batch 65536, 1/2/4/8 GPU",
            "value": round(value, 1), "unit": "examples/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "fp32",
            "step_ms_distribution": step_dist,
            "data": "synthetic (Criteo-Kaggle-skewed 26-slot slab, bounded Zipf(1.05) ids, seed 4)",
            "config": {"workload": f"dlrm_criteo_{S}x{args.rows}x{D}", "global_batch": args.batch * world,
                       "per_gpu_batch": args.batch, "rows": args.rows, "dim": D, "slots": S,
                       "bottom_mlp": [512, 256, D], "top_mlp": [512, 256, 1],
                       "optimizer": args.optimizer + (" (deferred exact decay)" if materialize_ms is not None else ""),
                       "parallelism": (f"row-sharded slab x{world} (RCCL all-to-all of the unique rows and of their "
                                       f"gradient rows) + dp{world} MLPs (all-reduce of the fused kernel's "
                                       f"batch sums)") if world > 1 else "single",
                       "prefetch": bool(args.prefetch),
                       **({"exchange": exchange_info(model.embedding_layer)} if world > 1 else {})},
            "mlp": {"backward": args.mlp_bwd, "forward": args.mlp_fwd,
                    "note": "ctr MLP hidden layers are linear (ctr/layers.py:8), so each MLP is one "
                            "affine map: the composed forward evaluates x·K1·K2·K3 + c as x·(K1K2K3) + c "
                            "and the factored backward takes every layer's gradient from the last "
                            "layer's. Every layer's parameters are kept and updated; same values in "
                            "exact arithmetic, fp32 rounding order differs (tests/test_mlp_chain_gpu.py "
                            "bounds both against a float64 oracle)",
                    "ms_per_step_layerwise_fwd": layerwise_fwd_ms,
                    "ms_per_step_layerwise_fwd_bwd": layerwise_ms},
            "roofline": roof, "kernels": kern,
            **({"weak_scaling": weak} if weak is not None else {}),
            **({"keras_adam": keras} if keras is not None else {}),
            "cpu_baseline": cpu, "loss": float(loss.item()),
            **({"keras_materialize_ms": materialize_ms} if materialize_ms is not None else {}),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
