"""Row-sharded embedding slab over W ranks (BASELINE north star "tables shard
row-wise across the 8 GPUs of one node with RCCL all-to-all over xGMI").

Layout: global row g lives on rank g % W at local row g // W (cyclic deal, so the Zipf-hot
rows of every slot spread over all ranks). Per step, on each rank:

  forward   sort ids by owner-major key (rs_sort_ids_sharded) → unique keys + inverse map +
            per-owner counts (rs_unique_inverse) → capacity-bounded packing (rs_exchange_pack:
            unique row u of owner o takes slot o·C + its rank among o's rows in a [W, C] block,
            every position the slot of its row) → all-to-all of the row ids (equal C-row blocks)
            → owners gather them (rs_gather_rows_padded; padding slots read zero rows) →
            all-to-all of the rows back. The step's kernels read rows from the [W·C, D] block
            by the slot index, so nothing downstream changes.
  backward  grad rows (position order) → tiled segmented sum per unique row written straight
            into its slot (rs_embedding_dedup_grad_mapped) → all-to-all to owners (equal
            blocks) → each owner sorts the received (local row, source-rank-major) slots,
            padding left out (masked sort), and applies the optimizer with the same tiled fold;
            rows of each rank's local mean are scaled 1/W, the fused DLRM step's rows (of the
            global mean) are applied as they are.

The capacity C (row slots per (rank, owner) pair) is calibrated once, on the first exchanged
batch (the largest per-owner unique count over all ranks x capacity_factor + 256), so every
all-to-all has fixed equal split sizes. A batch with more than C unique rows for some owner takes
a spill round instead of failing: each rank's largest excess over C is all-reduced (MAX) on the
device beside the row-id all-to-all, and when it is C2 > 0 every rank exchanges the excess rows in
a second pair of equal-split all-to-alls of [world, C2] blocks (slots after the capacity block),
so every rank issues the same collectives and no row is dropped. The host reads C2 when the step
needs its rows (exchange_finish): with the exchange prefetched a step ahead (the production
path) the value is long on the host; a step without prefetch waits for its own sort there.
The exchange runs on a side HIP stream (RCCL all-to-alls on their own), overlapping the bottom
MLP on the main stream; its first half (sort … row-id all-to-all) reads no table state and can
be queued a step ahead (prefetch).
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

    def __init__(self, group=None, force_collectives: bool = False):
        """force_collectives: run the collectives through the process group even at world 1
        (where they are copies): the RCCL path can then be exercised on a one-GPU box
        (tests/test_rccl_gpu.py). Off, world 1 short-circuits to device copies."""
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.staged = dist.is_initialized() and dist.get_backend(group) == "gloo"
        if force_collectives and not dist.is_initialized():
            raise RuntimeError("Comm(force_collectives=True) needs an initialised process group")
        self.force = bool(force_collectives)

    @property
    def collective(self) -> bool:
        """True when the collectives go through the process group (world > 1, or forced)."""
        return self.world > 1 or self.force

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None,
                   async_op: bool = False):
        """Splits None: equal blocks (the sharded slab's capacity-bounded exchange). async_op
        (RCCL): returns the work handle instead of ordering the current stream after it (gloo
        rehearsals stage through the host and return None)."""
        if not self.collective:
            out.copy_(inp)
            return None
        osp = None if out_splits is None else list(out_splits)
        isp = None if in_splits is None else list(in_splits)
        if self.staged:
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), osp, isp, group=self.group)
            out.copy_(o)
            return None
        return dist.all_to_all_single(out, inp, osp, isp, group=self.group, async_op=async_op)

    def all_reduce_(self, t: torch.Tensor, op=None):
        if not self.collective:
            return
        op = dist.ReduceOp.SUM if op is None else op
        if self.staged:
            c = t.cpu()
            dist.all_reduce(c, op=op, group=self.group)
            t.copy_(c)
        else:
            dist.all_reduce(t, op=op, group=self.group)


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
                 generator: torch.Generator | None = None, full_weight: torch.Tensor | None = None,
                 capacity: int | None = None, capacity_factor: float = 1.25):
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
        # exchange_begin's own stream: a later step's sort / unique / packing / row-id all-to-all
        # read no table state, so they run beside this step's exchange and apply instead of
        # queueing in front of them on the side stream
        self.pre = torch.cuda.Stream(device=device) if device.type == "cuda" else None
        self.optimizer: SparseOptimizer | None = None
        self._st = None  # per-step exchange state
        self._prefetched: list = []  # exchange_begin states queued ahead, FIFO (prefetch)
        # exchange capacity: row slots per (rank, owner) pair; None = calibrated on the first
        # batch (_calibrate), then fixed
        self.capacity = capacity
        self.capacity_factor = float(capacity_factor)
        self.spill_rounds = 0  # steps that exchanged rows past the capacity (a spill round)
        # the backward's dedup + gradient all-to-all in two owner halves (D = 128): the first
        # half's all-to-all runs while the second half is summed (RCCL); False: one of each
        self.split_halves = True
        # rows a step ahead (world > 1, SGD / lazy Adam): a prefetched step's capacity block is
        # gathered and sent while the step before it runs; after that step's apply only the rows
        # it updated (the ones both steps request, per owner stamps) are sent again
        self.rows_ahead = True
        self.rows_ahead_modes = {"fresh": 0, "late": 0, "full": 0}
        self.late_slots = [0, 0]  # late steps: (slots re-sent W·C_late, capacity slots W·C)
        self._overflow = None
        self._stamp = None  # int32 per local row: the last finished step (seq) that requested it
        self._seq = 0  # exchange_begin count (each step's seq)
        self._apply_count = 0
        self._last_applied = 0  # seq of the last applied step

    @property
    def n_slots(self):
        return self.slot_offsets.numel() - 1

    def set_optimizer(self, opt: SparseOptimizer):
        """opt must be built over [self.shard]; its learning rate is used as given (the 1/W
        scale of the global-mean loss is applied here)."""
        self.optimizer = opt

    # ---------------------------------------------------------------- forward
    def _calibrate(self, counts: torch.Tensor):
        """The exchange capacity (row slots per (rank, owner) pair, the same on every rank): the
        largest per-owner unique count of the first exchanged batch over all ranks, times
        capacity_factor, + 256, rounded up to 256. The only host sync of the exchange; every
        later step moves fixed [world, capacity] blocks."""
        mx = counts.max().to(torch.int64).reshape(1)
        if self.comm.collective:
            if self.comm.staged:
                c = mx.cpu()
                dist.all_reduce(c, op=dist.ReduceOp.MAX, group=self.comm.group)
                mx = c
            else:
                dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=self.comm.group)
        need = int(mx.item())
        self.capacity = -(-(int(need * self.capacity_factor) + 256) // 256) * 256

    def exchange_begin(self, ids: torch.Tensor):
        """Queue the first half of a step's exchange on its own stream: owner-major sort, unique
        / inverse + per-owner counts, the capacity-bounded packing (rs_exchange_pack: every
        unique row within the capacity gets a fixed slot in a [world, capacity] send block, each
        position the slot of its row) and each rank's largest excess over the capacity (the
        spill round's size, rs_exchange_excess). Nothing here reads the table, so it may run a
        step ahead (prefetch); no host sync once the capacity is known. Its collectives (the
        excess all-reduce, the row-id all-to-all: _begin_comm) are issued later — by the step
        before's exchange_finish once that step's own rows are on their way, or by this step's —
        so that RCCL, which runs collectives in issue order, never queues the current step's
        row transfer behind a later step's sort."""
        L.require_device(ids, "ids")
        dev = ids.device
        ids = ids.contiguous()
        main = torch.cuda.current_stream(dev)
        self.pre.wait_stream(main)
        W = self.world
        with torch.cuda.stream(self.pre):
            s = SortedIds(ids, self.input_dim, self.slot_offsets, self.err_flag, self.ws,
                          count_unique=False, world=W)
            n = ids.numel()
            uniq = torch.empty(n, dtype=torch.int32, device=dev)
            inverse = torch.empty(n, dtype=torch.int32, device=dev)
            # rs_unique_inverse zeroes the count and writes every owner's count: no fills here
            n_unique = torch.empty(1, dtype=torch.int32, device=dev)
            counts = torch.empty(W, dtype=torch.int32, device=dev)
            # this step's own workspace: its head is the segment index of every sorted key,
            # which the backward's dedup reuses (no second head-flag scan)
            w = torch.empty(L.lib().rs_unique_inverse_workspace_size(n), dtype=torch.uint8,
                            device=dev)
            L.call("rs_unique_inverse", L.ptr(s.rows), L.ptr(s.pos), n, self.input_dim, W,
                   L.ptr(uniq), L.ptr(inverse), L.ptr(n_unique), L.ptr(counts), L.ptr(w),
                   w.numel(), L.stream_ptr(dev))
            if self.capacity is None:
                self._calibrate(counts)
            C = self.capacity
            send_ids = torch.empty(W * C, dtype=torch.int32, device=dev)
            slot_of = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
            inv_slot = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
            # the packing's past-capacity flag is not read (the spill round sends those rows):
            # one persistent word, not a fill per step
            if self._overflow is None:
                self._overflow = torch.zeros(1, dtype=torch.int32, device=dev)
            L.call("rs_exchange_pack", L.ptr(uniq), L.ptr(n_unique), L.ptr(counts), W,
                   self.stride, C, L.ptr(inverse), n, L.ptr(send_ids), L.ptr(slot_of),
                   L.ptr(inv_slot), L.ptr(self._overflow), L.stream_ptr(dev))
            # the spill round's size: every rank's largest excess over C, all-reduced (MAX)
            excess = torch.empty(1, dtype=torch.int64, device=dev)
            L.call("rs_exchange_excess", L.ptr(counts), W, C, L.ptr(excess), L.stream_ptr(dev))
        self._seq += 1
        return dict(ids=ids, s=s, slot_of=slot_of, inv_slot=inv_slot, send_ids=send_ids,
                    capacity=C, dev=dev, uniq=uniq, n_unique=n_unique, counts=counts,
                    inverse=inverse, excess_dev=excess, seq=self._seq, early=None, late=None,
                    seg_excl=w, comm=False)

    def _begin_comm(self, st):
        """exchange_begin's collectives, on its stream: the spill round's size all-reduced (MAX)
        and copied to the host (read by the step's exchange_finish), the row-id all-to-all."""
        if st["comm"]:
            return
        dev, W, C = st["dev"], self.world, st["capacity"]
        with torch.cuda.stream(self.pre):
            excess = st["excess_dev"]
            self.comm.all_reduce_(excess, dist.ReduceOp.MAX)
            host = torch.empty(1, dtype=torch.int64, pin_memory=True)
            host.copy_(excess, non_blocking=True)
            excess_ready = torch.cuda.Event()
            excess_ready.record(self.pre)
            recv_ids = torch.empty(W * C, dtype=torch.int32, device=dev)
            self.comm.all_to_all(recv_ids, st["send_ids"])
            begun = torch.cuda.Event()
            begun.record(self.pre)
        st.update(excess=(excess_ready, host), recv_ids=recv_ids, begun=begun, comm=True)

    def _on_side(self, st):
        """Order the side stream after st's exchange_begin (its own stream) and mark st's device
        tensors as used there (their memory is not reused before the side stream's work on them
        has run)."""
        if st.get("on_side"):
            return
        self.side.wait_event(st["begun"])
        for v in list(st.values()) + [st["s"].rows, st["s"].pos]:
            if isinstance(v, torch.Tensor) and v.is_cuda:
                v.record_stream(self.side)
        st["on_side"] = True

    def _rows_ahead_ok(self) -> bool:
        """Rows a step ahead need an update that changes only the rows it receives (SGD, lazy
        Adam; Keras Adam's dense decay moves every row) and rows of a multiple-of-4 width."""
        opt = self.optimizer
        return (self.rows_ahead and self.comm.collective and self.output_dim % 4 == 0
                and opt is not None and opt.kind in (L.RS_OPT_SGD, L.RS_OPT_LAZY_ADAM))

    def _gather_send(self, ids: torch.Tensor, out: torch.Tensor):
        """Owners gather the requested rows (padding slots read zero rows) and send them back:
        out[...] = the rows this rank asked for, in its slot order. On the side stream."""
        dev = out.device
        served = torch.empty_like(out)
        L.call("rs_gather_rows_padded", L.ptr(self.shard.weight), self.shard.input_dim,
               self.output_dim, L.ptr(ids), ids.numel(), L.ptr(served), L.stream_ptr(dev))
        self.comm.all_to_all(out, served)

    def _issue_early(self, st):
        """The capacity block's rows, gathered now: final for every row the steps applied in
        between leave alone; exchange_finish re-sends the rest (on the side stream)."""
        W, C = self.world, st["capacity"]
        rows = torch.empty(W * C, self.output_dim, device=st["dev"])
        self._gather_send(st["recv_ids"], rows)
        st["early"] = (rows, self._apply_count)

    def _ahead(self, cur, nxt):
        """In exchange_finish of step `cur`, on the side stream: stamp cur's requested rows
        (capacity block and spill: the rows its apply will change), list the next step's slots
        whose rows are among them (rs_exchange_classify: re-sent after cur's apply), all-reduce the
        largest such list (the late round's size, read on the host at nxt's finish), send each
        requester its slot list, and gather + send nxt's capacity block now."""
        dev, W, C = nxt["dev"], self.world, nxt["capacity"]
        if self._stamp is None:
            self._stamp = torch.zeros(max(self.shard.input_dim, 1), dtype=torch.int32, device=dev)
        seq = cur["seq"]
        for ids in (cur["recv_ids"], cur.get("recv_spill")):
            if ids is not None:
                L.call("rs_exchange_mark", L.ptr(ids), ids.numel(), L.ptr(self._stamp),
                       self.shard.input_dim, seq, L.stream_ptr(dev))
        late_rows = torch.empty(W * C, dtype=torch.int32, device=dev)
        late_slot = torch.empty(W * C, dtype=torch.int32, device=dev)
        late_cnt = torch.empty(W, dtype=torch.int32, device=dev)
        L.call("rs_exchange_classify", L.ptr(nxt["recv_ids"]), W, C, L.ptr(self._stamp),
               self.shard.input_dim, seq, L.ptr(late_rows), L.ptr(late_slot), L.ptr(late_cnt),
               L.stream_ptr(dev))
        mx = torch.empty(1, dtype=torch.int64, device=dev)
        L.call("rs_exchange_excess", L.ptr(late_cnt), W, 0, L.ptr(mx), L.stream_ptr(dev))
        self.comm.all_reduce_(mx, dist.ReduceOp.MAX)
        host = torch.empty(1, dtype=torch.int64, pin_memory=True)
        host.copy_(mx, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(self.side)
        recv_slot = torch.empty(W * C, dtype=torch.int32, device=dev)
        self.comm.all_to_all(recv_slot, late_slot)
        nxt["late"] = dict(rows=late_rows, recv_slot=recv_slot, count=(ev, host), pred=seq)
        self._issue_early(nxt)

    def invalidate_rows_ahead(self):
        """The shard's rows were written by something other than the owner apply (a
        load_state_dict, a re-init, a manual edit): every queued step's early rows are stale, so
        each re-sends its whole block after the applies before it ('full' mode). The mode is
        decided from _apply_count alone, the same on every rank — call this on every rank."""
        self._apply_count += 2

    def _load_from_state_dict(self, *args, **kw):
        super()._load_from_state_dict(*args, **kw)
        self.invalidate_rows_ahead()

    @staticmethod
    def _ids_key(ids):
        return (ids.data_ptr(), tuple(ids.shape), ids.dtype)

    def prefetch(self, ids: torch.Tensor):
        """Queue the first half of a LATER step's exchange now (exchange_begin: sort, unique,
        packing, the row-id all-to-all) so it runs beside the current step; that step then
        starts from the owners' gather. The all-to-all is a collective, so every rank must
        prefetch the same steps in the same order. Entries are kept in queue order: a step
        takes its own entry and drops the older ones (steps that never ran), a step with no
        entry exchanges afresh, and a step whose entry's ids changed in place raises instead of
        re-exchanging (which one rank alone might do, pairing the ranks' collectives wrongly)."""
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
        """The second half, on the side stream after the previous step's owner apply: the spill
        round's ids when the all-reduced excess C2 is > 0 (rs_exchange_pack_spill: the rows past
        the capacity get slots world·C + o·C2 + j and their ids go in a second equal-split
        all-to-all), the owners gather the requested rows (rs_gather_rows_padded: padding slots
        read zero rows) and the rows go back in one all-to-all of equal [capacity, D] blocks (two
        with a spill round). Returns (view: the [world * (C + C2), D] rows, inverse ids [B, S]
        int32 = each position's slot)."""
        dev, W, C = st["dev"], self.world, st["capacity"]
        main = torch.cuda.current_stream(dev)
        D = self.output_dim
        self._begin_comm(st)  # issued here when no step before did (no prefetch)
        ev, host = st["excess"]
        ev.synchronize()  # prefetched a step ahead: long done
        C2 = int(host.item())
        n = st["ids"].numel()
        recv_spill = None
        with torch.cuda.stream(self.side):
            self._on_side(st)
            if st["early"] is None:  # not issued ahead: gathered now, after every queued apply
                self._issue_early(st)
            rows_c, count0 = st["early"]
            k = self._apply_count - count0
            late = st["late"]
            if k == 0:
                mode = "fresh"  # no apply since the gather
            elif k == 1 and late is not None and self._last_applied == late["pred"]:
                mode = "late"  # one apply since: the one of the step whose rows were stamped
            else:
                mode = "full"
            self.rows_ahead_modes[mode] += 1
            if mode == "late":
                lev, lhost = late["count"]
                lev.synchronize()  # recorded a step ago
                C_late = int(lhost.item())
                self.late_slots[0] += W * C_late
                self.late_slots[1] += W * C
                if C_late > 0:
                    ids_l = late["rows"].view(W, C)[:, :C_late].contiguous()
                    recv = torch.empty(W * C_late, D, device=dev)
                    self._gather_send(ids_l, recv)
                    L.call("rs_exchange_scatter_late", L.ptr(recv), L.ptr(late["recv_slot"]), W,
                           C, C_late, D, L.ptr(rows_c), L.stream_ptr(dev))
            elif mode == "full":
                self._gather_send(st["recv_ids"], rows_c)
            if C2 > 0:
                self.spill_rounds += 1
                spill_ids = torch.empty(W * C2, dtype=torch.int32, device=dev)
                L.call("rs_exchange_pack_spill", L.ptr(st["uniq"]), L.ptr(st["n_unique"]),
                       L.ptr(st["counts"]), W, self.stride, C, C2, L.ptr(st["inverse"]), n,
                       L.ptr(spill_ids), L.ptr(st["slot_of"]), L.ptr(st["inv_slot"]), None,
                       L.stream_ptr(dev))
                recv_spill = torch.empty(W * C2, dtype=torch.int32, device=dev)
                self.comm.all_to_all(recv_spill, spill_ids)
                rows = torch.empty(W * (C + C2), D, device=dev)
                rows[: W * C].copy_(rows_c)
                self._gather_send(recv_spill, rows[W * C:])
            else:
                rows = rows_c
            ready = torch.cuda.Event()
            ready.record(self.side)
            # the next prefetched step: its collectives now, behind this step's row transfers;
            # its rows (rows ahead) gathered and sent beside this step's train kernel
            st["recv_spill"] = recv_spill
            if self._prefetched:
                nxt = self._prefetched[0][2]
                self._begin_comm(nxt)
                if nxt["early"] is None and self._rows_ahead_ok():
                    self._on_side(nxt)
                    self._ahead(st, nxt)
        main.wait_event(ready)
        inverse = st["inv_slot"][:n]
        for t in (rows, inverse):
            t.record_stream(main)
        self.view.weight = rows
        self.view.input_dim = W * (C + C2)
        self._st = dict(sorted=st["s"], slot_of=st["slot_of"], recv_ids=st["recv_ids"],
                        recv_spill=recv_spill, capacity=C, spill=C2, seq=st["seq"],
                        seg_excl=st["seg_excl"])
        return self.view, inverse.view(st["ids"].shape)

    def exchange(self, ids: torch.Tensor):
        """Fetch this step's unique rows; returns (view, inverse ids [B, S] int32)."""
        st = self.take_prefetched(ids.contiguous())
        return self.exchange_finish(st if st is not None else self.exchange_begin(ids))

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
        G[b]), formed inside the local segmented sum. The per-unique-row sums go straight into
        their slots of the [world, capacity] send block (rs_embedding_dedup_grad_mapped), one
        all-to-all of equal blocks, then each owner applies the received rows in (source rank,
        slot) order, padding slots left out of its masked sort."""
        st = self._st
        if st is None:
            raise RuntimeError("backward without a forward exchange")
        dev = grad_rows.device
        main = torch.cuda.current_stream(dev)
        self.side.wait_stream(main)
        s = st["sorted"]
        W, C, C2, D = self.world, st["capacity"], st["spill"], self.output_dim
        with torch.cuda.stream(self.side):
            g = grad_rows.contiguous()
            send_grad = torch.empty(W * (C + C2), D, dtype=torch.float32, device=dev)
            uniq_rows = torch.empty(max(s.n, 1), dtype=torch.int32, device=dev)
            recv_grad = torch.empty(W * (C + C2), D, dtype=torch.float32, device=dev)
            if row_scale is not None and row_scale.numel() * self.n_slots != s.n:
                raise ValueError("row_scale must hold one value per example")
            w = self.ws.get("dedup", L.lib().rs_dedup_workspace_size(max(s.n, 1), D), dev)

            def dedup(lo, hi, seg_ready):
                # the segment ids come from exchange_begin's unique pass over the same keys
                if s.n:
                    L.call("rs_embedding_dedup_grad_mapped_range", L.ptr(s.rows), L.ptr(s.pos),
                           s.n, L.ptr(g), L.ptr(row_scale),
                           self.n_slots if row_scale is not None else 1, D, self.key_space, lo,
                           hi, seg_ready, L.ptr(st["seg_excl"]), L.ptr(st["slot_of"]),
                           L.ptr(uniq_rows), L.ptr(send_grad), L.ptr(w), w.numel(),
                           L.stream_ptr(dev))

            if W >= 2 and D == 128 and self.split_halves:
                # owner halves [0, W/2) and [W/2, W): keys are owner-major, so half A's rows are
                # the keys below (W/2)·stride. Each half: its dedup, then an all-to-all in which
                # only that half's owners receive (every rank sends them C rows); with RCCL the
                # first all-to-all runs while the second half is summed
                h = W // 2
                K = h * self.stride
                mine_a = self.rank < h
                none = torch.empty(0, D, dtype=torch.float32, device=dev)
                dedup(0, K, 0)
                work_a = self.comm.all_to_all(recv_grad[: W * C] if mine_a else none,
                                              send_grad[: h * C],
                                              [C] * W if mine_a else [0] * W,
                                              [C] * h + [0] * (W - h), async_op=True)
                dedup(K, self.key_space, 1)
                work_b = self.comm.all_to_all(none if mine_a else recv_grad[: W * C],
                                              send_grad[h * C: W * C],
                                              [0] * W if mine_a else [C] * W,
                                              [0] * h + [C] * (W - h), async_op=True)
                for wk in (work_a, work_b):
                    if wk is not None:
                        wk.wait()
            else:
                dedup(0, self.key_space, 0)
                self.comm.all_to_all(recv_grad[: W * C], send_grad[: W * C])
            recv_ids = st["recv_ids"]
            if C2 > 0:
                self.comm.all_to_all(recv_grad[W * C:], send_grad[W * C:])
                # source-rank-major [world, C + C2]: each row's terms stay in source-rank order,
                # the order the owner's fold has without a spill round (the oracle's)
                recv_grad = torch.cat([recv_grad[: W * C].view(W, C, D),
                                       recv_grad[W * C:].view(W, C2, D)], 1).view(-1, D)
                recv_ids = torch.cat([recv_ids.view(W, C), st["recv_spill"].view(W, C2)],
                                     1).view(-1)
            if self.optimizer is None:
                raise RuntimeError("ShardedSlabEmbedding has no optimizer (set_optimizer)")
            opt = self.optimizer
            params = opt._params()
            if self.world > 1 and not global_grads:
                if opt.kind == L.RS_OPT_SGD:
                    params.lr = params.lr / self.world  # same as scaling the gradient
                else:
                    recv_grad.mul_(1.0 / self.world)
            # the received slots are W runs (one per source rank), each its source's rows in
            # key order with the padding at the end: merged, not radix-sorted (same order as the
            # masked sort: source-rank-major among equal rows, padding left out)
            sorted_ids = SortedIds.from_runs(recv_ids, W, self.shard.input_dim, self.err_flag)
            # every owner applies (an owner no rank sent a row to still runs Keras' dense decay)
            opt.apply(self.shard, recv_ids, recv_grad, params, sorted_ids=sorted_ids)
        self._apply_count += 1
        self._last_applied = st["seq"]
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
