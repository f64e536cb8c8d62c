"""Row-sharded embedding slab over W ranks (BASELINE north star "tables shard
row-wise across the 8 GPUs of one node with RCCL all-to-all over xGMI").

Layout: global row g lives on rank g % W at local row g // W (cyclic deal, so the Zipf-hot
rows of every slot spread over all ranks). Per step, on each rank:

  forward   sort ids by owner-major key (rs_sort_ids_sharded) → unique keys + inverse map +
            per-owner counts (rs_unique_inverse) → all-to-all of the unique local rows each
            owner must serve → owners gather them (rs_embedding_fwd on the shard) → all-to-all
            of the rows back. The step's kernels then read rows from the unique-row buffer by
            the inverse index, so nothing downstream changes.
  backward  grad rows (position order) → tiled segmented sum per unique row
            (rs_embedding_dedup_grad) → all-to-all to owners → each owner sorts the received
            (local row, source-rank-major) list and applies the optimizer with the same tiled
            fold (rs_sort_ids + rs_embedding_apply); the update is scaled 1/W (the global loss
            is the mean over W local batches).

The exchange chain runs on a side HIP stream; RCCL all-to-all runs on its own stream, so the
exchange overlaps the bottom MLP on the main stream. One host sync per step reads the W owner
counts (the all-to-all split sizes).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch import nn

from . import _lib as L
from .embedding import Embedding
from .optim import SortedIds, SparseOptimizer, _Workspace


class Comm:
    """All-to-all / all-reduce transport. gloo groups are staged through host memory (CPU tests
    and one-GPU multi-process tests); nccl (= RCCL on ROCm) runs device to device."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.staged = dist.is_initialized() and dist.get_backend(group) == "gloo"

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits):
        if self.world == 1:
            out.copy_(inp)
            return
        if self.staged:
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), list(out_splits), list(in_splits), group=self.group)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, inp, list(out_splits), list(in_splits), group=self.group)

    def all_reduce_(self, t: torch.Tensor):
        if self.world == 1:
            return
        if self.staged:
            c = t.cpu()
            dist.all_reduce(c, group=self.group)
            t.copy_(c)
        else:
            dist.all_reduce(t, group=self.group)


class _UniqueRows:
    """Duck-types Embedding for the kernels of recommender_amd.functional: weight = this step's
    unique rows [U, D]; ids handed to the kernels are the inverse indices into it."""

    def __init__(self, parent: "ShardedSlabEmbedding"):
        self.parent = parent
        self.weight = None
        self.input_dim = 0
        self.output_dim = parent.output_dim
        self.slot_offsets = None
        self.n_slots = 1
        self.err_flag = parent.err_flag
        self.grad_handle = parent.grad_handle
        self.fused_optimizer = None

    def presort(self, ids):
        pass

    def accumulate_grad(self, ids, grad_rows):
        self.parent.backward_exchange(grad_rows)


class ShardedSlabEmbedding(nn.Module):
    def __init__(self, cardinalities, dim: int, comm: Comm | None = None, device=None,
                 generator: torch.Generator | None = None, full_weight: torch.Tensor | None = None):
        super().__init__()
        self.comm = comm or Comm()
        W, r = self.comm.world, self.comm.rank
        device = torch.device(device) if device is not None else torch.device("cuda")
        card = torch.as_tensor(list(cardinalities), dtype=torch.int64)
        offs = torch.zeros(card.numel() + 1, dtype=torch.int64)
        offs[1:] = torch.cumsum(card, 0)
        self.input_dim = int(offs[-1])
        self.output_dim = int(dim)
        self.world, self.rank = W, r
        self.stride = -(-self.input_dim // W)
        self.key_space = self.input_dim if W == 1 else self.stride * W
        shard_rows = (self.input_dim - r + W - 1) // W
        w = None if full_weight is None else full_weight[r::W]
        self.shard = Embedding(shard_rows, dim, device=device, generator=generator, weight=w)
        self.register_buffer("slot_offsets", offs.to(device))
        self.register_buffer("err_flag", torch.zeros(1, dtype=torch.int32, device=device))
        self.grad_handle = nn.Parameter(torch.zeros(0, device=device), requires_grad=True)
        self.view = _UniqueRows(self)
        self.ws = _Workspace()
        self.side = torch.cuda.Stream(device=device) if device.type == "cuda" else None
        self.optimizer: SparseOptimizer | None = None
        self._st = None  # per-step exchange state
        self._prefetched: list = []  # exchange_begin states queued ahead, FIFO (prefetch)

    @property
    def n_slots(self):
        return self.slot_offsets.numel() - 1

    def set_optimizer(self, opt: SparseOptimizer):
        """opt must be built over [self.shard]; its learning rate is used as given (the 1/W
        scale of the global-mean loss is applied here)."""
        self.optimizer = opt

    # ---------------------------------------------------------------- forward
    def exchange_begin(self, ids: torch.Tensor):
        """Queue the owner-major sort, the unique / inverse pass and the split-size exchange on
        the side stream without blocking the host; DLRM calls this before it queues the bottom
        MLP, so the sort runs beside it (the side stream only waits for work queued so far)."""
        L.require_device(ids, "ids")
        dev = ids.device
        ids = ids.contiguous()
        main = torch.cuda.current_stream(dev)
        self.side.wait_stream(main)
        W = self.world
        with torch.cuda.stream(self.side):
            s = SortedIds(ids, self.input_dim, self.slot_offsets, self.err_flag, self.ws,
                          count_unique=False, world=W)
            n = ids.numel()
            uniq = torch.empty(n, dtype=torch.int32, device=dev)
            inverse = torch.empty(n, dtype=torch.int32, device=dev)
            n_unique = torch.zeros(1, dtype=torch.int32, device=dev)
            counts = torch.zeros(W, dtype=torch.int32, device=dev)
            w = self.ws.get("uniq", L.lib().rs_sort_ids_workspace_size(n), dev)
            L.call("rs_unique_inverse", L.ptr(s.rows), L.ptr(s.pos), n, self.input_dim, W,
                   L.ptr(uniq), L.ptr(inverse), L.ptr(n_unique), L.ptr(counts), L.ptr(w),
                   w.numel(), L.stream_ptr(dev))
            staged = self.comm.staged or not dist.is_initialized() or W == 1
            host = torch.empty(2 * W, dtype=torch.int32, pin_memory=True)
            if staged:
                host[:W].copy_(counts, non_blocking=True)
            else:
                # receive counts device to device, then ONE copy of both count vectors to the host
                recv = torch.empty_like(counts)
                dist.all_to_all_single(recv, counts, group=self.comm.group)
                host.copy_(torch.cat([counts, recv]), non_blocking=True)
            ready = torch.cuda.Event()
            ready.record(self.side)
        return dict(ids=ids, s=s, uniq=uniq, inverse=inverse, host=host, ready=ready,
                    staged=staged, dev=dev)

    @staticmethod
    def _ids_key(ids):
        return (ids.data_ptr(), tuple(ids.shape), ids.dtype)

    def prefetch(self, ids: torch.Tensor):
        """Queue the first half of a LATER step's exchange now (owner-major sort, unique /
        inverse, split sizes: exchange_begin) so that step's exchange_finish finds its split
        sizes already on the host: the one host sync of a sharded step then waits on work queued
        a step earlier instead of stalling the device. The split-size exchange is a collective,
        so every rank must prefetch the same steps in the same order. Entries are kept in queue
        order: a step takes its own entry and drops the older ones (steps that never ran), a
        step with no entry exchanges afresh, and a step whose entry's ids changed in place
        raises instead of re-exchanging (which one rank alone might do, pairing the ranks'
        collectives wrongly)."""
        if torch.cuda.is_current_stream_capturing():
            return
        if len(self._prefetched) >= 4:  # stale entries (steps that never ran)
            self._prefetched.pop(0)
        self._prefetched.append((self._ids_key(ids), ids._version, self.exchange_begin(ids)))

    def take_prefetched(self, ids: torch.Tensor):
        """The prefetched exchange_begin state of these ids (older entries dropped), or None."""
        key = self._ids_key(ids)
        for i, (k, version, st) in enumerate(self._prefetched):
            if k == key:
                del self._prefetched[: i + 1]
                if version != ids._version:
                    raise RuntimeError("ShardedSlabEmbedding: a prefetched batch's ids were "
                                       "changed in place before their step")
                return st
        return None

    def exchange_finish(self, st):
        """Wait (host) for the split sizes, then the two all-to-alls and the owner gather;
        returns (view, inverse ids [B, S] int32)."""
        dev, W = st["dev"], self.world
        main = torch.cuda.current_stream(dev)
        st["ready"].synchronize()  # the one host sync of the step (split sizes)
        send_counts = st["host"][:W].clone()
        with torch.cuda.stream(self.side):
            U = int(send_counts.sum())
            if W == 1:
                recv_counts = send_counts
            elif st["staged"]:
                recv_counts = torch.empty(W, dtype=torch.int32)
                self.comm_counts(recv_counts, send_counts)
            else:
                recv_counts = st["host"][W:].clone()
            R = int(recv_counts.sum())
            owner = torch.arange(W, device=dev, dtype=torch.int64).repeat_interleave(
                send_counts.to(dev, torch.int64), output_size=U)
            send_rows = (st["uniq"][:U].to(torch.int64) - owner * self.stride).to(torch.int32)
            recv_rows = torch.empty(R, dtype=torch.int32, device=dev)
            sc, rc = send_counts.tolist(), recv_counts.tolist()
            self.comm.all_to_all(recv_rows, send_rows, rc, sc)
            with torch.no_grad():
                served = self.shard(recv_rows) if R else torch.empty(0, self.output_dim, device=dev)
            rows = torch.empty(U, self.output_dim, device=dev)
            self.comm.all_to_all(rows, served.detach().contiguous(), sc, rc)
        inverse = st["inverse"]
        main.wait_stream(self.side)
        for t in (rows, inverse):
            t.record_stream(main)
        self.view.weight = rows
        self.view.input_dim = U
        self._st = dict(sorted=st["s"], U=U, R=R, send_counts=sc, recv_counts=rc,
                        recv_rows=recv_rows)
        return self.view, inverse.view(st["ids"].shape)

    def exchange(self, ids: torch.Tensor):
        """Fetch this step's unique rows; returns (view, inverse ids [B, S] int32)."""
        st = self.take_prefetched(ids.contiguous())
        return self.exchange_finish(st if st is not None else self.exchange_begin(ids))

    def comm_counts(self, recv_counts: torch.Tensor, send_counts: torch.Tensor):
        if self.comm.staged or not dist.is_initialized():
            dist.all_to_all_single(recv_counts, send_counts.clone(), group=self.comm.group)
        else:
            d = send_counts.to(self.slot_offsets.device)
            r = torch.empty_like(d)
            dist.all_to_all_single(r, d, group=self.comm.group)
            recv_counts.copy_(r.cpu())

    def forward(self, ids):
        """Plain lookup [.., D] (DeepFM / ESMM style): exchange, then expand by the inverse."""
        view, inv = self.exchange(ids)
        from .functional import embedding_lookup

        return embedding_lookup(view, inv)

    def presort(self, ids):
        pass

    # ---------------------------------------------------------------- backward
    def backward_exchange(self, grad_rows: torch.Tensor, global_grads: bool = False,
                          row_scale: torch.Tensor | None = None):
        """global_grads: the rows are gradients of the GLOBAL mean loss (the fused DLRM step's
        kernel scales by 1/(B·W)), so the owners apply them as they are; otherwise each rank's
        rows are of its local mean and the update is scaled 1/W. row_scale [B] (optional): the
        row of position p is row_scale[p // S] * grad_rows[p] (the fused step's unit rows and
        G[b]), formed inside the local segmented sum."""
        st = self._st
        if st is None:
            raise RuntimeError("backward without a forward exchange")
        dev = grad_rows.device
        main = torch.cuda.current_stream(dev)
        self.side.wait_stream(main)
        s = st["sorted"]
        with torch.cuda.stream(self.side):
            U, R, D = st["U"], st["R"], self.output_dim
            g = grad_rows.contiguous()
            uniq_rows = torch.empty(max(s.n, 1), dtype=torch.int32, device=dev)
            uniq_grad = torch.empty(max(s.n, 1), D, dtype=torch.float32, device=dev)
            if s.n:
                w = self.ws.get("dedup", L.lib().rs_dedup_workspace_size(s.n, D), dev)
                if row_scale is None:
                    L.call("rs_embedding_dedup_grad", L.ptr(s.rows), L.ptr(s.pos), s.n, L.ptr(g),
                           D, self.key_space, L.ptr(uniq_rows), L.ptr(uniq_grad), L.ptr(w),
                           w.numel(), L.stream_ptr(dev))
                else:
                    if row_scale.numel() * self.n_slots != s.n:
                        raise ValueError("row_scale must hold one value per example")
                    L.call("rs_embedding_dedup_grad_scaled", L.ptr(s.rows), L.ptr(s.pos), s.n,
                           L.ptr(g), L.ptr(row_scale), self.n_slots, D, self.key_space,
                           L.ptr(uniq_rows), L.ptr(uniq_grad), L.ptr(w), w.numel(),
                           L.stream_ptr(dev))
            recv_grad = torch.empty(R, D, dtype=torch.float32, device=dev)
            self.comm.all_to_all(recv_grad, uniq_grad[:U], st["recv_counts"], st["send_counts"])
            if self.optimizer is None:
                raise RuntimeError("ShardedSlabEmbedding has no optimizer (set_optimizer)")
            opt = self.optimizer
            params = opt._params()
            if R:
                if self.world > 1 and not global_grads:
                    if opt.kind == L.RS_OPT_SGD:
                        params.lr = params.lr / self.world  # same as scaling the gradient
                    else:
                        recv_grad.mul_(1.0 / self.world)
                opt.apply(self.shard, st["recv_rows"], recv_grad, params)
            elif opt.kind == L.RS_OPT_KERAS_ADAM:
                # no row of this shard was touched this step: Keras Adam still decays m / v and
                # moves every row (the dense half of _resource_apply_sparse)
                m, v, bitmap = opt._slots(self.shard)
                t = self.shard
                L.call("rs_keras_adam_dense_sweep", L.ptr(t.weight), L.ptr(m), L.ptr(v),
                       t.input_dim, t.output_dim, params, L.ptr(bitmap), L.stream_ptr(dev))
        g.record_stream(self.side)
        if row_scale is not None:
            row_scale.record_stream(self.side)
        self._st = None

    def join(self):
        """Make the current stream wait for the exchange / apply chain."""
        torch.cuda.current_stream(self.side.device).wait_stream(self.side)

    def full_weight(self) -> torch.Tensor:
        """Gather the whole slab (tests / checkpoints): [V, D] with row g from rank g % W."""
        W = self.world
        if W == 1:
            return self.shard.weight.clone()
        rows = -(-self.input_dim // W)
        pad = torch.zeros(rows, self.output_dim, device=self.shard.weight.device)
        pad[: self.shard.input_dim] = self.shard.weight
        parts = [torch.empty_like(pad) for _ in range(W)]
        if self.comm.staged:
            cp = [p.cpu() for p in parts]
            dist.all_gather(cp, pad.cpu(), group=self.comm.group)
            parts = cp
        else:
            dist.all_gather(parts, pad, group=self.comm.group)
        full = torch.stack(parts, 1).reshape(rows * W, self.output_dim)
        return full[: self.input_dim]
