"""ctr/train.py counterpart (reference ctr/train.py:11-97): DLRM / DeepFM training on
synthetic Criteo-shaped data through the MI355X engine.

Same flags and defaults as the reference (--gpus, --gpu_memory_limit, --model_type,
--train_batch_size, --test_batch_size, --seed; 26 cat / 13 int features, vocab 1 000 000,
dim 16, 3 epochs, DLRM units [512,256,64,16] / [512,256,1], Adam) plus:
  --optimizer  keras_adam (reference default, ctr/train.py:80,84) | lazy_adam | sgd
               (the commented DLRM SGD + DLRMScheduler path, ctr/train.py:77-79)
  --steps_per_epoch, --rows/--slab (per-slot tables), --embedding_size.
Loss: BinaryCrossentropy(reduction=NONE) (ctr/train.py:85) still calls
keras.losses.binary_crossentropy, which averages over the LAST axis [3p TF 2.2]; the models
output [B] (ctr/model.py:27,57), so the loss the reference differentiates is the batch mean.
--loss_reduction keeps `sum` available.
"""
from __future__ import annotations

import argparse
import contextlib
import os
import time

import numpy as np
import torch

from .. import _lib as L
from ..functional import binary_crossentropy
from ..nn import invalidate_compose_cache, overlapped_param_grads, overlapped_weight_grads
from ..metrics import AUC
from ..optim import DLRMScheduler, KerasAdam, SparseAdam, SparseSGD
from ..synthetic import criteo_batch, criteo_cardinalities
from .model import DLRM, DeepFM


class TrainStep:
    """One optimizer step of a ctr model: forward, BCE, backward, dense + sparse apply."""

    def __init__(self, model, optimizer="sgd", lr=None, loss_reduction="mean", sched=None,
                 fused=True, overlap_wgrad=False, comm=None, defer_sparse_join=False,
                 overlap_param_grads=False, fused_step=True, defer_decay=False):
        """comm: a recommender_amd.sharded.Comm for data-parallel dense parameters (gradients
        all-reduced and averaged over ranks); with a ShardedSlabEmbedding the table is updated
        by its owners inside the backward.
        fused_step: the production DLRM step (D = 128 or 64, composed / factored MLP chains, fused
        sparse optimizer, one GPU) runs its forward, loss and backward reductions in one kernel
        (functional.dlrm_fused_train_forward) instead of autograd over the fused interaction;
        other configurations take the autograd path.
        defer_decay: with optimizer='keras_adam', replay the dense Keras decay of rows without a
        gradient when they are next read instead of sweeping all rows every step (exact; call
        step.opt_sparse.materialize() before reading the table)."""
        from ..sharded import ShardedSlabEmbedding

        self.model = model
        self.comm = comm
        dense = [p for n, p in model.named_parameters() if not n.endswith("grad_handle")]
        self.dense = dense
        emb = model.embedding_layer
        self.sharded = isinstance(emb, ShardedSlabEmbedding)
        tables = [emb.shard if self.sharded else emb]
        if self.sharded:
            fused = False
        self.loss_reduction = loss_reduction
        self.fused_step = bool(fused_step)
        # the fused step's plain-SGD MLP update + next compositions in rs_dlrm_dense_tail
        # (RS_DENSE_TAIL=0: chain_param_grads + torch.optim.SGD, bit-identical)
        self.dense_tail = os.environ.get("RS_DENSE_TAIL", "1") == "1"
        self.overlap_wgrad, self.overlap_pgrad = overlap_wgrad, overlap_param_grads
        # measured on MI355X: a weight-grad GEMM beside the interaction backward only
        # time-slices the CUs (no net gain), so the overlap is opt-in
        self.wgrad = overlapped_weight_grads(dense[0].device) if overlap_wgrad else None
        # opt-in: the MLP chains' parameter gradients on a second stream (measured: they slow the
        # co-running interaction backward by as much as they hide, 320 -> 364 us)
        self.pgrad = (overlapped_param_grads(dense[0].device) if overlap_param_grads
                      else contextlib.nullcontext())
        if optimizer == "sgd":
            lr = sched or (lr if lr is not None else 0.01)
            self.opt_dense = torch.optim.SGD(dense, lr=lr if not callable(lr) else lr(0))
            self.opt_sparse = SparseSGD(tables, lr=lr, fused=fused, defer_join=defer_sparse_join)
            self._sched = lr if callable(lr) else None
        elif optimizer in ("keras_adam", "lazy_adam"):
            lr = lr if lr is not None else 1e-3
            self.opt_dense = KerasAdam(dense, lr=lr)
            self.opt_sparse = SparseAdam(tables, lr=lr, mode="keras" if optimizer == "keras_adam" else "lazy",
                                         fused=fused, defer_join=defer_sparse_join,
                                         defer_decay=defer_decay and optimizer == "keras_adam")
            self._sched = None
        else:
            raise ValueError(f"unknown optimizer {optimizer}")
        if self.sharded:
            emb.set_optimizer(self.opt_sparse)

    def capture(self, batch, warmup: int = 3):
        """Capture one whole step (forward, loss, backward, dense + sparse apply) on `batch`'s
        tensors into a HIP graph; returns a replay callable. Scalars (learning rates) are
        frozen into the graph, so capture only with constant-lr SGD."""
        if self._sched is not None or not isinstance(self.opt_sparse, SparseSGD):
            raise RuntimeError("graph capture needs constant-lr SGD (scalars are frozen)")
        if self.sharded:
            raise RuntimeError("a row-sharded slab's step reads its spill / late-round sizes on "
                               "the host each step and cannot be captured")
        # the graph must join every stream it forks: the sparse update joins inside the step
        # (a replay is ordered after the previous one as a whole)
        defer = self.opt_sparse.defer_join
        self.opt_sparse.defer_join = False
        torch.cuda.synchronize()
        for t in self.opt_sparse.tables:
            t._pending_update = None
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self(batch)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        invalidate_compose_cache()  # the graph must record the compositions it reads
        with torch.cuda.graph(g):
            loss = self(batch)
        invalidate_compose_cache()
        self._graph_loss = loss
        self.opt_sparse.defer_join = defer

        def replay():
            g.replay()
            # the replay moved the parameters in place (no version bump): eager steps recompose
            invalidate_compose_cache()
            return loss

        return replay

    def capture_sequence(self, batches, warmup: int = 2):
        """Capture len(batches) consecutive steps into ONE HIP graph (constant-lr SGD): no host
        launch cost per kernel, and inside the graph each step's sparse update (side stream)
        overlaps the next step's bottom MLP exactly as the deferred join does eagerly; only the
        last step's update is joined at the end of the graph. Returns a replay callable that
        runs all the steps and returns the last loss."""
        if self._sched is not None or not isinstance(self.opt_sparse, SparseSGD):
            raise RuntimeError("graph capture needs constant-lr SGD (scalars are frozen)")
        if self.sharded:
            raise RuntimeError("a row-sharded slab's step reads its spill / late-round sizes on "
                               "the host each step and cannot be captured")
        defer = self.opt_sparse.defer_join
        self.opt_sparse.defer_join = self.opt_sparse.fused
        torch.cuda.synchronize()
        for t in self.opt_sparse.tables:
            t._pending_update = None
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                for b in batches:
                    self(b)
            for t in self.opt_sparse.tables:
                t.wait_update()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        invalidate_compose_cache()
        with torch.cuda.graph(g):
            for b in batches:
                loss = self(b)
            for t in self.opt_sparse.tables:  # join the last update inside the graph
                t.wait_update()
        invalidate_compose_cache()
        self.opt_sparse.defer_join = defer

        def replay():
            g.replay()
            invalidate_compose_cache()
            return loss

        return replay

    # -- graph-capturable Keras-Adam step (non-fused tables: DeepFM, cfg1) -------------------
    def static_step(self, batch):
        """One Keras-Adam step with no host-side per-step scalars, so it can sit in a HIP graph
        (as DIENStep.static_step): the table's IndexedSlices gradient densified (densify_grad:
        the sort + tiled segmented sum of the sparse apply, no sync) into the flat gradient buffer
        and Keras Adam over every variable with lr_t from device memory (GraphKerasAdam). Keras'
        sparse Adam decays m / v and moves every row each step anyway, so this dense step is the
        same update as __call__'s sparse apply + dense sweep (tests/test_deepfm_gpu.py: bit for
        bit). Its Adam state is its own: do not interleave with __call__."""
        from ..optim import GraphKerasAdam, _Workspace, densify_grad

        if (not isinstance(self.opt_sparse, SparseAdam) or self.opt_sparse.kind != L.RS_OPT_KERAS_ADAM
                or self.opt_sparse.fused or self.sharded):
            raise RuntimeError("static_step: Keras Adam on non-fused, unsharded tables only")
        tables = list(self.opt_sparse.tables)
        if getattr(self, "opt_graph", None) is None:
            tw = {id(t.weight) for t in tables}
            self._gdense = [p for p in self.dense if id(p) not in tw and p.numel() > 0]
            self.opt_graph = GraphKerasAdam(self._gdense + [t.weight for t in tables],
                                            lr=self.opt_dense.param_groups[0]["lr"])
            self._gws = _Workspace()
            self.opt_sparse.release_state()  # the graph path's Adam state is opt_graph's
        for p in self._gdense:
            p.grad = None
        cat, dense_x, label = batch
        pred = self.model({"cat_features": cat, "int_features": dense_x})
        self.last_pred = pred.detach()
        loss = binary_crossentropy(label, pred, reduction=self.loss_reduction)
        loss.backward()
        grads = [p.grad for p in self._gdense]  # None: Keras skips the variable
        nd = len(self._gdense)
        for i, t in enumerate(tables):  # densified straight into the flat gradient buffer
            got = t.take_grad(with_valid=True, segments=True)
            grads.append(densify_grad(t, got[0], got[1], self._gws, valid=got[2],
                                      out=self.opt_graph.grad_view(nd + i))
                         if got is not None else None)
        if not torch.cuda.is_current_stream_capturing():
            self.opt_graph.prepare()
            self.opt_graph.iterations += 1
        self.opt_graph.apply(grads)
        return loss.detach()

    def capture_static(self, batch):
        """Record one static_step on `batch` (static device tensors the caller refills before
        each replay) into a HIP graph; returns replay() -> loss. Run one eager static_step first
        (it builds the optimizer state the graph reads)."""
        opt = self.opt_graph
        opt.prepare()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        invalidate_compose_cache()  # the graph must record the compositions it reads
        with torch.cuda.graph(g):
            out = self.static_step(batch)
        invalidate_compose_cache()
        self._static_graph = g

        def replay():
            opt.prepare()
            g.replay()
            opt.iterations += 1
            invalidate_compose_cache()  # the replay moved the parameters in place
            return out
        return replay

    def prefetch(self, batch):
        """Sort a LATER batch's ids now (Embedding.prefetch, fused sparse optimizer; on a
        row-sharded slab the exchange's first half, ShardedSlabEmbedding.prefetch): call
        it before the step that precedes the batch's own step, e.g.
        `step.prefetch(batches[i + 1]); step(batches[i])` — the data pipeline's prefetch of the
        next batch. The batch's ids must already be on the device and must not change before
        their step runs."""
        emb = self.model.embedding_layer
        ids = batch[0].reshape(-1, self.model.num_cat_fea).contiguous()
        if self.sharded:
            # row-sharded slab: the exchange's sort, unique pass and split sizes a step ahead
            emb.prefetch(ids)
            return
        if not self.opt_sparse.fused or not hasattr(emb, "prefetch"):
            return
        emb.prefetch(ids)

    def fused_step_ready(self, batch) -> bool:
        """True when __call__ takes the one-kernel production DLRM step."""
        from ..embedding import Embedding
        from ..nn import narrow_chain_hip_ready, vec_chain_ready
        from .layers import MLP
        from .model import DLRM

        from ..sharded import ShardedSlabEmbedding

        m = self.model
        emb = m.embedding_layer
        # one GPU: the fused side-stream sparse optimizer; row-sharded: the owners' apply inside
        # the backward exchange, with plain SGD (the gradient rows carry the global 1/(B·W))
        if self.sharded:
            sparse_ok = (isinstance(emb, ShardedSlabEmbedding) and isinstance(self.opt_sparse, SparseSGD)
                         and not callable(self.opt_sparse.lr)
                         and (self.comm is None or self.comm.world == emb.world))
        else:
            sparse_ok = (self.opt_sparse.fused and (self.comm is None or self.comm.world == 1)
                         and isinstance(emb, Embedding) and emb.weight.data_ptr() % 16 == 0)
        if not (self.fused_step and isinstance(m, DLRM) and m.compact and sparse_ok
                and not self.overlap_wgrad and not self.overlap_pgrad
                and self.loss_reduction in ("mean", "sum") and torch.is_grad_enabled()):
            return False
        cat, dense_x, _ = batch
        B = cat.numel() // m.num_cat_fea
        bl, tl = list(m.bottom_mlp.mlp), list(m.top_mlp.mlp)
        return (emb.output_dim in (64, 128) and m.num_cat_fea <= 27
                and m.num_int_fea == 13 and cat.is_cuda
                and MLP.factored_backward and MLP.composed_forward and B >= MLP.factored_min_batch
                and all(l.act_code == 0 for l in bl[:-1] + tl[:-1])
                and bl[-1].act_code == 1 and tl[-1].act_code == 2
                and narrow_chain_hip_ready(bl, m.num_int_fea)
                and vec_chain_ready(tl, m.compact_rows.numel()))

    def __call__(self, batch):
        cat, dense_x, label = batch
        if self._sched is not None:
            for g in self.opt_dense.param_groups:
                g["lr"] = self._sched(self.opt_sparse.iterations)
        self.opt_dense.zero_grad(set_to_none=True)
        if self.fused_step_ready(batch):
            from ..functional import dense_tail_ready, dlrm_fused_train_forward

            tail = self.dense_tail and dense_tail_ready(self.model, self.opt_dense)
            lr = self.opt_dense.param_groups[0]["lr"] if tail else None
            comm = self.comm if self.sharded else None
            if comm is None and self.sharded:
                comm = self.model.embedding_layer.comm
            y, loss = dlrm_fused_train_forward(self.model, cat, dense_x, label, self.loss_reduction,
                                               sgd_lr=lr, comm=comm)
            self.last_pred = y
            if not tail:
                self.opt_dense.step()
            if self.sharded:
                self.opt_sparse.iterations += 1  # the owners applied inside the exchange
            else:
                self.opt_sparse.step()
            return loss
        p = self.model({"cat_features": cat, "int_features": dense_x})
        self.last_pred = p.detach()
        loss = binary_crossentropy(label, p, reduction=self.loss_reduction)
        with self.pgrad:
            if self.wgrad is not None:
                with self.wgrad:
                    loss.backward()
            else:
                loss.backward()
        if self.comm is not None and self.comm.world > 1:
            self._allreduce_dense()
        self.opt_dense.step()
        if self.sharded:
            self.model.embedding_layer.join()
            self.opt_sparse.iterations += 1
        else:
            self.opt_sparse.step()
        return loss

    def _allreduce_dense(self):
        """One bucketed RCCL all-reduce of every dense gradient (≈3 MB for the DLRM MLPs),
        averaged over ranks — the MirroredStrategy dense-gradient sync."""
        grads = [p.grad for p in self.dense if p.grad is not None]
        flat = torch._utils._flatten_dense_tensors(grads)
        self.comm.all_reduce_(flat)
        flat.mul_(1.0 / self.comm.world)
        torch._foreach_copy_(grads, list(torch._utils._unflatten_dense_tensors(flat, grads)))


def build_model(model_type, embedding_size, vocab_size, num_cat_fea, num_int_fea, device,
                slot_cardinalities=None, bottom=None, top=None, mlp_units=None, generator=None):
    if model_type == "DLRM":
        bottom = bottom or [512, 256, 64, embedding_size]
        top = top or [512, 256, 1]
        return DLRM(bottom, top, embedding_size, vocab_size, num_cat_fea, num_int_fea, device=device,
                    slot_cardinalities=slot_cardinalities, generator=generator)
    if model_type == "DeepFM":
        return DeepFM(embedding_size, vocab_size, num_int_fea, num_cat_fea, mlp_units or [512, 256, 1],
                      device=device, slot_cardinalities=slot_cardinalities, generator=generator)
    raise ValueError(model_type)


def train(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=str, default="0")
    ap.add_argument("--gpu_memory_limit", type=int, default=20480)  # parsed, unused (as reference)
    ap.add_argument("--model_type", type=str, default="DLRM")
    ap.add_argument("--train_batch_size", type=int, default=1024)
    ap.add_argument("--test_batch_size", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--optimizer", default="keras_adam", choices=["keras_adam", "lazy_adam", "sgd"])
    ap.add_argument("--loss_reduction", default="mean", choices=["sum", "mean"])
    ap.add_argument("--embedding_size", type=int, default=16)
    ap.add_argument("--vocab_size", type=int, default=1_000_000)
    ap.add_argument("--slab", action="store_true", help="per-slot tables (Criteo skew) in one slab")
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--steps_per_epoch", type=int, default=50)
    args = ap.parse_args(argv)
    from ..gemm_tuning import use_tuned_gemms

    use_tuned_gemms()  # committed TunableOp GEMM choices for the fixed dense shapes
    torch.manual_seed(args.seed)
    dev = torch.device("cuda")
    num_int_fea, num_cat_fea = 13, 26
    cards = criteo_cardinalities(args.vocab_size, num_cat_fea) if args.slab else [args.vocab_size] * num_cat_fea
    model = build_model(args.model_type, args.embedding_size, args.vocab_size, num_cat_fea,
                        num_int_fea, dev, slot_cardinalities=cards if args.slab else None)
    sched = DLRMScheduler(0.01, 100, 10000, 0.0001) if args.optimizer == "sgd" else None
    step = TrainStep(model, args.optimizer, loss_reduction=args.loss_reduction, sched=sched)
    rng = np.random.default_rng(args.seed)
    auc = AUC(num_thresholds=200)  # keras.metrics.AUC() default, ctr/train.py:86
    for epoch in range(1, args.epochs + 1):
        t0 = time.time()
        tot = 0.0
        auc.reset_states()
        for _ in range(args.steps_per_epoch):
            cat, dn, lb = criteo_batch(rng, args.train_batch_size, cards)
            if not args.slab:
                cat = cat % args.vocab_size
            batch = (torch.from_numpy(cat).to(dev), torch.from_numpy(dn).to(dev), torch.from_numpy(lb).to(dev))
            tot += float(step(batch))
            auc.update_state(batch[2], step.last_pred)
        torch.cuda.synchronize()
        dt = time.time() - t0
        print(f"epoch {epoch} loss {tot / args.steps_per_epoch:.4f} auc {auc.result():.4f} "
              f"{args.steps_per_epoch * args.train_batch_size / dt:.0f} ex/s")


if __name__ == "__main__":
    train()
