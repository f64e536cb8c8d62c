"""Training counterpart of eges/train.py (loop :14-24: sigmoid CE on the 1+num_ns skip-gram
logits, reduce_mean, Keras Adam on every table — IndexedSlices → SparseAdam(mode='keras')).

Data: the reference's pair pipeline (eges/data_loader.py:28-62: weighted walk → skipgrams →
log-uniform negatives) runs on the device (eges/sampler.py, EGESPairSampler) over a synthetic
weighted item graph (the JD session data is not available offline); `synthetic_batch` keeps
the i.i.d. batches of the same shapes for the model benchmarks.
Hyper-parameters from eges/train.py:45-54,75-92 (emb 160, num_ns 5, batch 1024, seed 4)."""
from __future__ import annotations

import argparse
import time

import numpy as np
import torch
import torch.nn.functional as F

from ..optim import GraphKerasAdam, SparseAdam, _Workspace, densify_grad
from .model import EGES, GES, DeepWalk
from .sampler import EGESPairSampler


def log_uniform(rng, n, range_max):
    """tf.random.log_uniform_candidate_sampler's distribution P(k) = log((k+2)/(k+1)) /
    log(range_max+1), by inverse CDF (without its uniqueness rejection)."""
    u = rng.random(n)
    return np.minimum((np.exp(u * np.log(range_max + 1.0)) - 1.0).astype(np.int64), range_max - 1)


def synthetic_item_graph(rng, n_items, n_edges):
    """Symmetric weighted co-occurrence CSR over items 1..n_items-1 (0 = OOV, no edges):
    popularity-skewed endpoints, integer session-count weights."""
    pop = rng.zipf(1.3, 2 * n_edges) % (n_items - 1) + 1
    src, dst = pop[:n_edges], pop[n_edges:]
    keep = src != dst
    s = np.concatenate([src[keep], dst[keep]])
    d = np.concatenate([dst[keep], src[keep]])
    w = rng.integers(1, 10, s.size).astype(np.float32)
    order = np.argsort(s, kind="stable")
    s, d, w = s[order], d[order], w[order]
    indptr = np.zeros(n_items + 1, np.int64)
    np.add.at(indptr, s + 1, 1)
    return np.cumsum(indptr), d.astype(np.int32), w


def synthetic_batch(rng, batch, n_items, n_cat, n_brand, num_ns=5):
    target = rng.integers(1, n_items, (batch, 1))
    pos = rng.integers(1, n_items, (batch, 1))
    neg = log_uniform(rng, batch * num_ns, n_items).reshape(batch, num_ns)
    context = np.concatenate([pos, neg], 1)
    item2cat = (np.arange(n_items) * 2654435761) % n_cat
    item2brand = (np.arange(n_items) * 40503) % n_brand
    label = np.zeros((batch, 1 + num_ns), np.float32)
    label[:, 0] = 1
    return (target.astype(np.int32), item2cat[target].astype(np.int32),
            item2brand[target].astype(np.int32), context.astype(np.int32), label)


class EGESStep:
    def __init__(self, model, lr=1e-3):
        self.model = model
        self.opt = SparseAdam(model.tables(), lr=lr, mode="keras")

    def __call__(self, inputs, labels):
        logits = self.model(inputs)
        loss = F.binary_cross_entropy_with_logits(logits, labels)  # sigmoid CE, reduce_mean
        loss.backward()
        self.opt.step()
        return loss.detach()

    # -- graph-capturable step --------------------------------------------------------------
    def static_step(self, inputs, labels):
        """The same step with no host-side per-step scalars, so it can sit in a HIP graph:
        every table's IndexedSlices gradient densified (densify_grad, no sync) and Keras Adam
        over all of them with lr_t from device memory (GraphKerasAdam, one launch). Keras'
        sparse Adam decays m / v and moves every row each step anyway (the dense sweep), so the
        dense step is the same update. Its Adam state is its own: do not interleave with
        __call__."""
        tables = self.model.tables()
        if getattr(self, "opt_graph", None) is None:
            self.opt_graph = GraphKerasAdam([t.weight for t in tables], lr=self.opt.lr)
            self._ws = _Workspace()
            self.opt.release_state()  # the graph path's Adam state is opt_graph's
        logits = self.model(inputs)
        loss = F.binary_cross_entropy_with_logits(logits, labels)
        loss.backward()
        grads = []
        for i, t in enumerate(tables):  # densified straight into the flat gradient buffer
            got = t.take_grad(segments=True)
            grads.append(densify_grad(t, got[0], got[1], self._ws,
                                      out=self.opt_graph.grad_view(i)) if got is not None
                         else None)
        if not torch.cuda.is_current_stream_capturing():
            self.opt_graph.prepare()
            self.opt_graph.iterations += 1
        self.opt_graph.apply(grads)
        return loss.detach()

    def capture(self, inputs, labels):
        """Record one static_step on (inputs, labels) — static device tensors the caller
        refills before each replay — into a HIP graph; returns replay() -> loss tensor. Run at
        least one eager static_step first."""
        opt = self.opt_graph
        opt.prepare()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            loss = self.static_step(inputs, labels)
        self._graph = g

        def replay():
            opt.prepare()
            g.replay()
            opt.iterations += 1
            return loss
        return replay


def build(model_type, n_items, n_cat, n_brand, embedding_size=160, device="cuda", generator=None):
    if model_type == "BGE":
        return DeepWalk(n_items, embedding_size, device=device, generator=generator)
    if model_type == "GES":
        return GES(n_items, n_cat, n_brand, embedding_size, device=device, generator=generator)
    if model_type == "EGES":
        return EGES(n_items, n_cat, n_brand, embedding_size, 3, device=device, generator=generator)
    raise ValueError(model_type)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model_type", default="BGE", choices=["BGE", "GES", "EGES"])
    ap.add_argument("--train_batch_size", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--n_items", type=int, default=63001)
    args = ap.parse_args(argv)
    rng = np.random.default_rng(args.seed)
    n_cat, n_brand = 801, 3000
    indptr, indices, weights = synthetic_item_graph(rng, args.n_items, 16 * args.n_items)
    items = np.arange(args.n_items)
    sampler = EGESPairSampler(indptr, indices, weights, args.n_items,
                              item2cat=(items * 2654435761) % n_cat,
                              item2brand=(items * 40503) % n_brand, seed=args.seed)
    model = build(args.model_type, args.n_items, n_cat, n_brand)
    step = EGESStep(model)
    t0 = time.perf_counter()
    for s in range(args.steps):
        *inp, lab = sampler.next_batch(args.train_batch_size, args.model_type)
        loss = step(tuple(inp), lab)
        if s % 50 == 0:
            print(f"step {s} loss {float(loss):.4f}")
    torch.cuda.synchronize()
    print(f"{args.steps * args.train_batch_size / (time.perf_counter() - t0):.0f} examples/s")


if __name__ == "__main__":
    main()
