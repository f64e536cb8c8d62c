"""dien/train.py counterpart (reference dien/train.py:12-143): BASE / DIN / DIEN on synthetic
Amazon-shaped sequences. Flags and defaults as the reference (--gpus --gpu_memory_limit
--model_type --history_max_length --epochs --train_batch_size --test_batch_size --seed) plus
--item_vocab/--cat_vocab (default 63 001 / 801, Amazon-Electronics-shaped) and
--steps_per_epoch. train_step_dien (dien/train.py:13-24): loss = mean BCE + mean aux; Keras
Adam on every parameter (embedding tables: exact Keras Adam with the dense decay)."""
from __future__ import annotations

import argparse
import time

import numpy as np
import torch

from ..functional import binary_crossentropy
from ..metrics import AUC
from ..optim import GraphKerasAdam, KerasAdam, SparseAdam, _Workspace, densify_grad
from . import DIEN, DIN, BaseModel


def synthetic_batch(rng, batch, hist_len, item_vocab, cat_vocab, negatives=True):
    """Post-padded / pre-truncated histories (dien/data_loader.py:44,48) of length
    2 + Geometric(0.1) clipped to hist_len; items U[1, V) with a fixed item→cat map; uniform
    negative history (dien/data_loader.py:58); labels Bernoulli(0.5)."""
    item2cat = 1 + (np.arange(item_vocab) * 2654435761 % max(cat_vocab - 1, 1))
    lens = np.clip(2 + rng.geometric(0.1, batch), 2, hist_len)
    valid = np.arange(hist_len)[None, :] < lens[:, None]
    pos = np.where(valid, rng.integers(1, item_vocab, (batch, hist_len)), 0).astype(np.int32)
    feats = {
        "target_item": rng.integers(1, item_vocab, (batch, 1)).astype(np.int32),
        "pos_his_item": pos,
        "pos_his_cat": np.where(valid, item2cat[pos], 0).astype(np.int32),
    }
    feats["target_cat"] = item2cat[feats["target_item"]].astype(np.int32)
    if negatives:
        neg = rng.integers(1, item_vocab, (batch, hist_len)).astype(np.int32)
        feats["neg_his_item"] = neg
        feats["neg_his_cat"] = item2cat[neg].astype(np.int32)
    label = (rng.random((batch, 1)) < 0.5).astype(np.float32)
    return feats, label


class DIENStep:
    def __init__(self, model, lr=1e-3):
        self.model = model
        tables = [model.item_embedding, model.cat_embedding]
        dense = [p for n, p in model.named_parameters() if not n.endswith("grad_handle")]
        self.opt_dense = KerasAdam(dense, lr=lr)
        self.opt_sparse = SparseAdam(tables, lr=lr, mode="keras")
        self.is_dien = isinstance(model, DIEN)

    def __call__(self, feats, label):
        self.opt_dense.zero_grad(set_to_none=True)
        if self.is_dien:
            pred, aux = self.model(feats, training=True)
            self.last_pred = pred.detach()
            bce = binary_crossentropy(label, pred, reduction="mean")
            aux = aux.mean()
            total = bce + aux
        else:
            pred = self.model(feats, training=True)
            self.last_pred = pred.detach()
            total = aux = binary_crossentropy(label, pred, reduction="mean")
        total.backward()
        self.opt_dense.step()
        self.opt_sparse.step()
        return total, aux

    # -- graph-capturable step --------------------------------------------------------------
    def static_step(self, feats, label):
        """__call__ with no host-side per-step scalars, so it can sit in a HIP graph: the two
        tables' IndexedSlices gradients densified (densify_grad: the same sort + tiled
        segmented sum as the sparse apply, no sync) and Keras Adam over every variable with
        lr_t from device memory (GraphKerasAdam, a variable without a gradient skipped as Keras
        skips it). Keras' sparse Adam decays m / v and moves every row each step anyway, so the
        dense step is the same update (tests/test_dien_step_gpu.py: equal to __call__ bit for
        bit). Its Adam state is its own: do not interleave with __call__."""
        tables = [self.model.item_embedding, self.model.cat_embedding]
        if getattr(self, "opt_graph", None) is None:
            tw = {id(t.weight) for t in tables}
            self._gdense = [p for p in self.opt_dense.param_groups[0]["params"]
                            if id(p) not in tw and p.numel() > 0]
            self.opt_graph = GraphKerasAdam(self._gdense + [t.weight for t in tables],
                                            lr=self.opt_dense.param_groups[0]["lr"])
            self._ws = _Workspace()
            self.opt_sparse.release_state()  # the graph path's Adam state is opt_graph's
        for p in self._gdense:
            p.grad = None
        if self.is_dien:
            pred, aux = self.model(feats, training=True)
            aux = aux.mean()
            total = binary_crossentropy(label, pred, reduction="mean") + aux
        else:
            pred = self.model(feats, training=True)
            total = aux = binary_crossentropy(label, pred, reduction="mean")
        self.last_pred = pred.detach()
        total.backward()
        grads = [p.grad for p in self._gdense]  # None: Keras skips the variable
        nd = len(self._gdense)
        for i, t in enumerate(tables):  # densified straight into the flat gradient buffer
            got = t.take_grad(with_valid=True, segments=True)
            grads.append(densify_grad(t, got[0], got[1], self._ws, valid=got[2],
                                      out=self.opt_graph.grad_view(nd + i))
                         if got is not None else None)
        if not torch.cuda.is_current_stream_capturing():
            self.opt_graph.prepare()
            self.opt_graph.iterations += 1
        self.opt_graph.apply(grads)
        return total.detach(), aux.detach()

    def capture(self, feats, label):
        """Record one static_step on (feats, label) — static device tensors the caller refills
        before each replay — into a HIP graph; returns replay() -> (total, aux). Run at least
        one eager static_step first (it builds the optimizer state the graph reads)."""
        opt = self.opt_graph
        opt.prepare()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = self.static_step(feats, label)
        self._graph = g

        def replay():
            opt.prepare()
            g.replay()
            opt.iterations += 1
            return out
        return replay


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=str, default="0")
    ap.add_argument("--gpu_memory_limit", type=int, default=4096)
    ap.add_argument("--model_type", type=str, default="BASE")
    ap.add_argument("--history_max_length", type=int, default=100)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--train_batch_size", type=int, default=128)
    ap.add_argument("--test_batch_size", type=int, default=2048)
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--item_vocab", type=int, default=63001)
    ap.add_argument("--cat_vocab", type=int, default=801)
    ap.add_argument("--steps_per_epoch", type=int, default=50)
    ap.add_argument("--hip_graph", type=int, default=1,
                    help="1: the step captured once as a HIP graph (DIENStep.capture) and replayed "
                         "on each batch; 0: the eager step")
    args = ap.parse_args(argv)
    from ..gemm_tuning import use_tuned_gemms

    use_tuned_gemms()  # committed TunableOp GEMM choices for the fixed dense shapes
    torch.manual_seed(args.seed)
    kw = dict(item_vocab_size=args.item_vocab, item_embedding_size=18, cat_vocab_size=args.cat_vocab,
              cat_embedding_size=18, mlp_units=[200, 80, 1], device="cuda")
    if args.model_type == "DIEN":
        model = DIEN(36, 36, **kw)
    elif args.model_type == "DIN":
        model = DIN(**kw)
    else:
        model = BaseModel(**kw)
    step = DIENStep(model)
    rng = np.random.default_rng(args.seed)
    auc = AUC(num_thresholds=20000)  # dien/train.py:43-44
    static, replay = None, None
    for epoch in range(1, args.epochs + 1):
        t0, tot = time.time(), 0.0
        auc.reset_states()
        for _ in range(args.steps_per_epoch):
            f, lab = synthetic_batch(rng, args.train_batch_size, args.history_max_length,
                                     args.item_vocab, args.cat_vocab, args.model_type == "DIEN")
            feats = {k: torch.from_numpy(v).cuda() for k, v in f.items()}
            label = torch.from_numpy(lab).cuda()
            if args.hip_graph:
                # static input buffers refilled per batch; the first step runs eagerly (it builds
                # the optimizer state), the second captures the graph that later steps replay
                if static is None:
                    static = ({k: torch.empty_like(v) for k, v in feats.items()}, torch.empty_like(label))
                torch._foreach_copy_([static[0][k] for k in feats] + [static[1]],
                                     list(feats.values()) + [label])
                if getattr(step, "opt_graph", None) is None:
                    out = step.static_step(*static)
                else:
                    replay = replay or step.capture(*static)
                    out = replay()
                tot += float(out[0])
                auc.update_state(static[1], step.last_pred)
            else:
                tot += float(step(feats, label)[0])
                auc.update_state(label, step.last_pred)
        torch.cuda.synchronize()
        print(f"epoch {epoch} loss {tot / args.steps_per_epoch:.4f} auc {auc.result():.4f} "
              f"{args.steps_per_epoch * args.train_batch_size / (time.time() - t0):.0f} ex/s")


if __name__ == "__main__":
    main()
