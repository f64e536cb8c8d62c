"""PinSage training loop counterpart of pinsage/train/train.py.

Per step (train.py:79-90): item2item pairs → sample_from_item_pairs (compact + 2 blocks) →
PinSageModel → margin_loss(delta=1) → backward → Keras Adam on every variable (dense params:
KerasAdam; the three embedding tables: SparseAdam(mode='keras'), the IndexedSlices path of
train.py:45-46). Hyper-parameters default to train.py:63-70.

Multi-GPU: pairs are sharded by global pair index (rank r draws pairs
[r*B, (r+1)*B) of each step), the graph and tables are replicated, and one bucketed
all-reduce averages the dense grads together with the densified table grads. Graph
synthetic: MovieLens-shaped (recommender_amd.synthetic.movielens_graph) with synthetic rating
times; no dataset is reachable offline. Every `--eval_every` steps (test_steps = 1000,
train.py:69,84-88) the device evaluation of pinsage/evaluation.py runs: item reprs →
recommend(top_k 10) → hit-rate against the time-split validation matrix.
"""
from __future__ import annotations

import argparse
import time

import numpy as np
import torch

from ..optim import GraphKerasAdam, KerasAdam, SparseAdam, _Workspace, dedup_grad, densify_grad
from ..synthetic import ML20M, movielens_graph
from .evaluation import (build_val_test_matrix, get_item_reprs, hit_rate_eval, recommend,
                         train_test_split_by_time)
from .graph import HeteroGraph
from .model import PinSageModel, check_oob
from .sampler import PinSageSampler, item_pairs

ML1M = dict(n_users=6_040, n_items=3_706, n_edges=1_000_209)


def build_graph(shape: dict, seed: int = 4, device="cuda") -> HeteroGraph:
    rng = np.random.default_rng(seed)
    users, items, year, genre = movielens_graph(rng, **shape)
    return HeteroGraph(users, items, shape["n_users"], shape["n_items"], device=device,
                       item_data={"year": year, "genre": genre})


def build_dataset(shape: dict, seed: int = 4, device="cuda"):
    """(train_g, val_matrix, test_matrix): the synthetic graph with rating times, split per user
    by time (util.py:5-39; the reference's process_movielens.py does this offline)."""
    rng = np.random.default_rng(seed)
    users, items, year, genre = movielens_graph(rng, **shape)
    ts = rng.integers(0, 1_000_000_000, users.size)
    tr, va, te = train_test_split_by_time(users, ts)
    g = HeteroGraph(users[tr], items[tr], shape["n_users"], shape["n_items"], device=device,
                    item_data={"year": year, "genre": genre},
                    edge_data={"timestamp": ts[tr]})
    val, test = build_val_test_matrix(users, items, va, te, shape["n_users"], shape["n_items"])
    return g, val, test


class PinSageStep:
    def __init__(self, model: PinSageModel, lr: float = 1e-3, comm=None):
        self.model = model
        self.dense = model.dense_parameters()
        self.opt_dense = KerasAdam(self.dense, lr=lr)
        self.opt_sparse = SparseAdam(model.tables(), lr=lr, mode="keras")
        self.comm = comm
        self.world = comm.world if comm is not None else 1

    def __call__(self, pos_graph, neg_graph, blocks):
        self.opt_dense.zero_grad(set_to_none=True)
        loss = self.model.margin_loss(pos_graph, neg_graph, blocks, 1.0)
        loss.backward()
        if self.world > 1:
            self._allreduce_and_apply_tables()
            self.opt_dense.step()
        else:
            self.opt_dense.step()
            self.opt_sparse.step()
        check_oob(loss.device)  # the dynamic step syncs on its shapes anyway
        return loss.detach()

    # -- sync-free step on capacity-shaped batches (PinSageSampler.sample_static) ------------
    def static_step(self, pos_graph, neg_graph, blocks):
        """One training step with no host sync, so it can be captured into a HIP graph: masked
        margin loss over the live pairs, and Keras Adam (GraphKerasAdam: lr_t from device
        memory) on the dense parameters and on the three tables' densified IndexedSlices
        gradients — Keras' sparse Adam decays m / v and moves every row anyway
        (_resource_apply_sparse [3p TF 2.2]), so the dense form is the same update. Equal to
        __call__ on the unpadded batch up to fp32 rounding order (tests/test_pinsage_gpu.py).
        Its Adam state (GraphKerasAdam) is its own: do not interleave with __call__.

        world > 1 (pairs sharded over the ranks, graph and tables replicated):
        every gradient lands in GraphKerasAdam's one flat gradient buffer, which is all-reduced
        (one collective: RCCL under nccl, so the sharded step captures into a HIP graph too) and
        scaled 1/W before the Adam launch — MirroredStrategy's mean of the replicas' gradients
        (pinsage/train/train.py:40-48), as __call__ does eagerly. The layout is fixed, so every
        parameter must have a gradient on every rank (capacity-shaped batches look up every
        table)."""
        if (self.world > 1 and getattr(self.comm, "staged", False)
                and torch.cuda.is_current_stream_capturing()):
            raise ValueError("a gloo-staged all-reduce cannot be captured: capture the sharded "
                             "step under RCCL (nccl)")
        tables = self.model.tables()
        if getattr(self, "opt_graph", None) is None:
            self.opt_graph = GraphKerasAdam(self.dense + [t.weight for t in tables],
                                            lr=self.opt_dense.param_groups[0]["lr"])
            self._ws = _Workspace()
            self.opt_sparse.release_state()  # the graph path's Adam state is opt_graph's
        for p in self.dense:
            p.grad = None
        loss = self.model.margin_loss(pos_graph, neg_graph, blocks, 1.0)
        loss.backward()
        grads = [p.grad for p in self.dense]  # None: Keras skips the variable
        nd = len(self.dense)
        for i, t in enumerate(tables):  # densified straight into the flat gradient buffer
            got = t.take_grad(segments=True)
            grads.append(densify_grad(t, got[0], got[1], self._ws,
                                      out=self.opt_graph.grad_view(nd + i)) if got is not None
                         else None)
        if self.comm is not None and self.comm.collective:
            if any(g is None for g in grads):
                raise ValueError("sharded static_step: a parameter has no gradient on this rank; "
                                 "the all-reduce needs the same flat layout on every rank")
            opt = self.opt_graph
            opt.collect(grads)
            self.comm.all_reduce_(opt.grad_flat)
            opt.grad_flat.mul_(1.0 / self.world)
            grads = [opt.grad_view(i) for i in range(len(grads))]
        if not torch.cuda.is_current_stream_capturing():
            self.opt_graph.prepare()
            self.opt_graph.iterations += 1  # a capture records the step; replay() counts it
        self.opt_graph.apply(grads)
        return loss.detach()

    def capture(self, batch):
        """Record one static_step on `batch` (a PinSageSampler.sample_static batch: the
        sampler's persistent buffers) into a HIP graph. Returns replay(): one training step on
        whatever the sampler last wrote into those buffers, and the step's loss tensor. Run at
        least one eager static_step first (library handles, workspaces)."""
        opt = self.opt_graph
        opt.prepare()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            loss = self.static_step(*batch)
        self._graph = g

        def replay():
            opt.prepare()
            g.replay()
            opt.iterations += 1
            return loss
        return replay

    def capture_with_sampling(self, sampler, batch_size: int, seed: int, step: int,
                              pair_base: int = 0):
        """One HIP graph for the WHOLE step: pair sampling (sample_pairs_static), neighbour
        walks and blocks (sample_static), forward, backward and Keras Adam. The two RNG steps
        (the pair sampler's `step` and the sampler's walk step) live in device memory and the
        graph advances them, so replay k samples exactly what eager step `step` + k would.
        Returns replay() -> loss tensor. Run at least one eager static_step first."""
        dev = sampler.g.device
        pair_step = torch.tensor([step], dtype=torch.int32, device=dev)
        walk_step = torch.tensor([sampler.step], dtype=torch.int32, device=dev)
        opt = self.opt_graph
        opt.prepare()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        host_step = sampler.step
        with torch.cuda.graph(g):
            batch = sampler.sample_static(
                *sampler.sample_pairs_static(batch_size, seed, 0, pair_base, step_dev=pair_step),
                step_dev=walk_step)
            loss = self.static_step(*batch)
            pair_step.add_(1)
            walk_step.add_(1)
        sampler.step = host_step  # the capture ran no step
        self._graph = g

        def replay():
            opt.prepare()
            g.replay()
            opt.iterations += 1
            sampler.step += 1
            return loss
        return replay

    def _allreduce_and_apply_tables(self):
        """Densify each table's IndexedSlices grad (deterministic segmented sum), bucket it
        with the dense grads into one all-reduce, average over ranks, then apply the tables
        as fully-touched slices (identical to Keras' dense m/v decay for untouched rows)."""
        # every rank must hand the all-reduce the same bucket layout: a parameter without a
        # gradient on this rank contributes zeros, and a has-gradient flag rides along in the
        # bucket so a parameter no rank produced a gradient for stays None (Keras skips it)
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self.dense]
        dev = self.dense[0].device if self.dense else self.model.tables()[0].weight.device
        has = torch.tensor([0.0 if p.grad is None else 1.0 for p in self.dense], device=dev)
        tables = self.model.tables()
        dense_tab = []
        for t in tables:
            got = t.take_grad()
            g = torch.zeros(t.input_dim, t.output_dim, device=t.weight.device)
            if got is not None:
                rows, ug = dedup_grad(t, got[0], got[1])
                g.index_copy_(0, rows, ug)
            dense_tab.append(g)
        bucket = grads + dense_tab + [has]
        flat = torch._utils._flatten_dense_tensors(bucket)
        self.comm.all_reduce_(flat)
        flat.mul_(1.0 / self.world)
        out = torch._utils._unflatten_dense_tensors(flat, bucket)
        any_grad = (out[-1] > 0).tolist()
        for p, g, present in zip(self.dense, out[: len(self.dense)], any_grad):
            p.grad = g if present else None
        params = self.opt_sparse._params()
        for t, g in zip(tables, out[len(self.dense):]):
            ids = torch.arange(t.input_dim, device=g.device, dtype=torch.int32)
            self.opt_sparse.apply(t, ids, g, params)
        self.opt_sparse.iterations += 1


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", choices=["ml1m", "ml20m"], default="ml1m")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--train_batch_size", type=int, default=32)
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--eval_every", type=int, default=1000)
    ap.add_argument("--top_k", type=int, default=10)
    ap.add_argument("--hip_graph", type=int, default=1,
                    help="1: sync-free capacity-shaped batches, sampling + step replayed as one "
                         "HIP graph (PinSageStep.capture_with_sampling); 0: the DGL-shaped step")
    args = ap.parse_args(argv)
    num_layers = 2
    embedding_size = 8
    conv_hidden_size, conv_output_size = 32, 16
    random_walk_length, num_random_walks, termination_prob, num_neighbors = 2, 4, 0, 3
    torch.manual_seed(args.seed)
    g, val_matrix, _ = build_dataset(ML1M if args.graph == "ml1m" else ML20M, args.seed)
    model = PinSageModel(g, g.itype, num_layers, embedding_size, conv_hidden_size,
                         conv_output_size)
    step_fn = PinSageStep(model)
    sampler = PinSageSampler(g, g.itype, g.utype, num_layers, random_walk_length,
                             num_random_walks, termination_prob, num_neighbors, seed=args.seed)
    t0 = time.perf_counter()
    replay = None
    for step in range(args.steps):
        if args.hip_graph:
            if step == 0:
                loss = step_fn.static_step(*sampler.sample_static(
                    *sampler.sample_pairs_static(args.train_batch_size, args.seed, step)))
            else:  # sampling + step in one graph, RNG steps advanced on the device
                replay = replay or step_fn.capture_with_sampling(
                    sampler, args.train_batch_size, args.seed, step)
                loss = replay()
        else:
            heads, pos, neg = item_pairs(g, args.train_batch_size, args.seed, step)
            batch = sampler.sample_from_item_pairs(heads, pos, neg, g.itype)
            loss = step_fn(*batch)
        if step % 50 == 0:
            print(f"step {step} step_loss {float(loss):.4f}")
            check_oob(loss.device)  # the graph steps' out-of-range node ids, checked here
        if args.eval_every and step % args.eval_every == 0:
            reprs = get_item_reprs(model, sampler, g, g.itype, 32)
            recs = recommend(g, args.top_k, reprs, None, g.utype, "timestamp", 32)
            print(f"step {step} hit_rate {hit_rate_eval(recs, val_matrix.tocsr()):.4f}")
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{args.steps / dt:.1f} it/s, {args.steps * args.train_batch_size / dt:.0f} pairs/s")


if __name__ == "__main__":
    main()
