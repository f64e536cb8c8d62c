"""esmm/train.py counterpart (reference esmm/train.py:153-255): BASE / ESMM / MMOE on
synthetic Ali-CCP-shaped data through the MI355X engine. Same flags and defaults as the
reference (--gpus --gpu_memory_limit --epochs --train_batch_size --test_batch_size
--auc_num_thresholds --train_ctr_tfrecord --model_type --test_steps --seed) plus
--rows (scale the 18 tables to this many rows, e.g. 40000000 for SURVEY cfg4) and
--steps_per_epoch. Multi-task loss: mean BCE over [ctr, ctcvr] (esmm/train.py:100-102);
Keras Adam (esmm/train.py:104,125) — dense KerasAdam + sparse Keras-exact Adam on the slab."""
from __future__ import annotations

import argparse
import time
from datetime import timedelta

import numpy as np
import torch

from ..functional import binary_crossentropy
from ..metrics import AUC
from ..optim import FusedKerasAdam, KerasAdam, SparseAdam, SparseSGD
from ..synthetic import aliccp_batch, scaled_vocab
from . import ESMM, FEAT_VOCAB, MMOE, BaseModel


def build(model_type, feat_vocab, embedding_size=18, device="cuda", generator=None, sharded_comm=None):
    mlp_units = [360, 200, 80, 1]  # esmm/train.py:217
    if model_type == "ESMM":
        return ESMM(mlp_units, feat_vocab, embedding_size, device, generator, sharded_comm)
    if model_type == "MMOE":  # esmm/train.py:245-253
        return MMOE(2, 8, [200, 80], [40, 1], feat_vocab, embedding_size, device, generator, sharded_comm)
    if model_type == "BASE":
        return BaseModel(mlp_units, "sigmoid", feat_vocab, embedding_size, device, generator, sharded_comm)
    raise ValueError(model_type)


class MultiTaskStep:
    """train_step of esmm/train.py:97-106: y_pred [B,2], mean BCE, Adam.

    comm (a recommender_amd.sharded.Comm, world > 1): data parallel over ranks — the dense
    gradients are all-reduced and averaged before the dense Adam (MirroredStrategy's sync), and a
    row-sharded slab applies its owners' update with the gradients scaled 1/W inside the backward,
    so both halves follow the mean loss over the global batch."""

    def __init__(self, model, optimizer="keras_adam", lr=1e-3, comm=None):
        """optimizer: "keras_adam" (the reference's tf.keras Adam, esmm/train.py:125: every
        slab row decays each step — a dense m / v sweep), "keras_adam_deferred" (the same update
        with each row's decay replayed when the row is next read, SparseAdam(defer_decay=True),
        fused into the step: bit-identical to "keras_adam" after materialize()), "lazy_adam"
        (touched rows only) or "sgd"."""
        self.model = model
        self.comm = comm
        dense = [p for n, p in model.named_parameters() if not n.endswith("grad_handle")]
        self.dense = dense
        slab = model.embedding_layer.slab
        table = getattr(slab, "shard", slab)
        if optimizer == "sgd":
            self.opt_dense = torch.optim.SGD(dense, lr=lr)
            self.opt_sparse = SparseSGD([table], lr=lr)
        elif optimizer == "keras_adam_deferred":
            if slab is not table:
                raise ValueError("keras_adam_deferred: one GPU (the row-sharded slab applies "
                                 "inside its exchange)")
            self.opt_dense = self._dense_adam(dense, lr)
            self.opt_sparse = SparseAdam([table], lr=lr, mode="keras", fused=True,
                                         defer_join=True, defer_decay=True)
        else:
            self.opt_dense = self._dense_adam(dense, lr)
            self.opt_sparse = SparseAdam([table], lr=lr, mode="keras" if optimizer == "keras_adam" else "lazy")
        self.sharded = slab is not table
        if self.sharded:
            slab.set_optimizer(self.opt_sparse)

    @staticmethod
    def _dense_adam(dense, lr):
        """Keras Adam of the dense parameters: the flat-buffer form on the GPU (one fused update
        launch, same roundings), the foreach form elsewhere."""
        if dense and all(p.is_cuda for p in dense):
            return FusedKerasAdam(dense, lr=lr)
        return KerasAdam(dense, lr=lr)

    def __call__(self, feats, label):
        self.opt_dense.zero_grad(set_to_none=True)
        y = self.model(feats)
        self.last_pred = y.detach()
        loss = binary_crossentropy(label, y, reduction="mean")
        loss.backward()
        if self.comm is not None and self.comm.world > 1:
            self._allreduce_dense()
        self.opt_dense.step()
        if self.sharded:
            self.model.embedding_layer.slab.join()
            self.opt_sparse.iterations += 1
        else:
            self.opt_sparse.step()
        return loss

    def materialize(self):
        """keras_adam_deferred: bring every slab row up to the last step (the dense sweep's
        state, bit for bit); a no-op otherwise."""
        if hasattr(self.opt_sparse, "materialize"):
            self.opt_sparse.materialize()

    def _allreduce_dense(self):
        grads = [p.grad for p in self.dense if p.grad is not None]
        flat = torch._utils._flatten_dense_tensors(grads)
        self.comm.all_reduce_(flat)
        flat.mul_(1.0 / self.comm.world)
        torch._foreach_copy_(grads, list(torch._utils._unflatten_dense_tensors(flat, grads)))


def train(argv=None):
    ap = argparse.ArgumentParser(description="ESMM model train config")
    ap.add_argument("--gpus", type=str, default="0")
    ap.add_argument("--gpu_memory_limit", type=int, default=4096)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--train_batch_size", type=int, default=512)
    ap.add_argument("--test_batch_size", type=int, default=2048)
    ap.add_argument("--auc_num_thresholds", type=int, default=10000)
    ap.add_argument("--train_ctr_tfrecord", type=str, default="(synthetic)")
    ap.add_argument("--model_type", type=str, default="MMOE")
    ap.add_argument("--test_steps", type=int, default=3000)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--steps_per_epoch", type=int, default=50)
    ap.add_argument("--optimizer", default="keras_adam", choices=["keras_adam", "lazy_adam", "sgd"])
    ap.add_argument("--sharded", action="store_true",
                    help="row-shard the slab over the torch.distributed ranks (RCCL all-to-all; "
                         "launch one process per GPU with torch.distributed.run)")
    args = ap.parse_args(argv)
    comm = None
    if args.sharded:
        import os

        import torch.distributed as dist

        from ..sharded import Comm

        if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not dist.is_initialized():
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                    timeout=timedelta(seconds=180))
        comm = Comm()
    from ..gemm_tuning import use_tuned_gemms

    use_tuned_gemms()  # committed TunableOp GEMM choices for the fixed dense shapes
    torch.manual_seed(args.seed)
    vocab = scaled_vocab(FEAT_VOCAB, args.rows) if args.rows else dict(FEAT_VOCAB)
    model = build(args.model_type, vocab, sharded_comm=comm)
    step = MultiTaskStep(model, args.optimizer, comm=comm)
    rng = np.random.default_rng([args.seed, comm.rank if comm else 0])
    # ctr and ctcvr AUCs over outputs [ctr, ctcvr] (esmm/train.py:58-61, 10000 thresholds)
    ctr_auc = AUC(num_thresholds=args.auc_num_thresholds)
    ctcvr_auc = AUC(num_thresholds=args.auc_num_thresholds)
    for epoch in range(1, args.epochs + 1):
        t0, tot = time.time(), 0.0
        ctr_auc.reset_states()
        ctcvr_auc.reset_states()
        for _ in range(args.steps_per_epoch):
            f, lab = aliccp_batch(rng, args.train_batch_size, vocab)
            feats = {k: torch.from_numpy(v).cuda() for k, v in f.items()}
            label = torch.from_numpy(lab).cuda()
            tot += float(step(feats, label))
            ctr_auc.update_state(label[:, 0], step.last_pred[:, 0])
            ctcvr_auc.update_state(label[:, 1], step.last_pred[:, 1])
        torch.cuda.synchronize()
        print(f"epoch {epoch} loss {tot / args.steps_per_epoch:.5f} ctr_auc {ctr_auc.result():.4f} "
              f"ctcvr_auc {ctcvr_auc.result():.4f} "
              f"{args.steps_per_epoch * args.train_batch_size / (time.time() - t0):.0f} ex/s")


if __name__ == "__main__":
    train()
