"""Embedding tables — the keras.layers.Embedding surface backed by librecsys_hip.

`Embedding(input_dim, output_dim, mask_zero)` mirrors keras.layers.Embedding [3p] as used at
ctr/model.py:10, dien/model.py:11-12, esmm/esmm.py:10-11: weight [input_dim, output_dim] fp32,
initialised U(-0.05, 0.05) (Keras 'uniform'), `compute_mask(ids) = ids != 0` (mask_zero).

`SlabEmbedding(cardinalities, dim)` packs one table per slot into a single HBM slab with row
offsets ("one slab with slot offsets"); a lookup takes ids [B, n_slots].

Gradients: the table is not an autograd leaf. A lookup's backward hands (ids, grad rows) to
`accumulate_grad`; a sparse optimizer (recommender_amd.optim) drains them with `take_grad`.
"""
from __future__ import annotations

import torch
from torch import nn

from . import _lib as L
from .functional import embedding_lookup


class Embedding(nn.Module):
    def __init__(self, input_dim: int, output_dim: int, mask_zero: bool = False, device=None,
                 slot_offsets: torch.Tensor | None = None, init_range: float = 0.05,
                 generator: torch.Generator | None = None, weight: torch.Tensor | None = None):
        super().__init__()
        device = torch.device(device) if device is not None else torch.device("cuda")
        self.input_dim = int(input_dim)
        self.output_dim = int(output_dim)
        self.mask_zero = bool(mask_zero)
        if weight is not None:
            if tuple(weight.shape) != (self.input_dim, self.output_dim):
                raise ValueError("weight shape mismatch")
            # always a private copy: the table is updated in place by the sparse optimizers
            w = weight.detach().to(device=device, dtype=torch.float32).clone().contiguous()
        else:
            w = torch.empty(self.input_dim, self.output_dim, device=device, dtype=torch.float32)
            w.uniform_(-init_range, init_range, generator=generator)
        self.register_buffer("weight", w)
        self.register_buffer("slot_offsets",
                             None if slot_offsets is None else slot_offsets.to(device, torch.int64))
        # the largest slot's row count, host-side (the sort picks its form from it); derived
        # again whenever the slot_offsets buffer is reloaded (_load_from_state_dict)
        self._set_max_slot_rows(slot_offsets)
        self.register_buffer("err_flag", torch.zeros(1, dtype=torch.int32, device=device))
        # zero-size leaf that keeps the lookup inside the autograd graph
        self.grad_handle = nn.Parameter(torch.zeros(0, device=device), requires_grad=True)
        self._pending: list[tuple[torch.Tensor, torch.Tensor]] = []
        # fused sparse optimizer (set by SparseOptimizer(..., fused=True)): the sort runs on
        # its side stream ahead of the dense forward, the apply inside the backward
        self.fused_optimizer = None
        self._presorted = None
        # sorts queued ahead for later steps (Embedding.prefetch), keyed by the ids' storage
        self._prefetched: dict = {}
        self._prefetch_queue: list = []  # prefetched ids whose sort is not launched yet
        self._prefetch_gen: list = []  # the presort count when each queued entry arrived
        self._presort_gen = 0
        # deferred join (SparseOptimizer(defer_join=True)): the event the next table read waits on
        self._pending_update = None
        # deferred-decay Keras Adam: the step this table's rows were last caught up for
        self._catchup_step = 0

    def wait_update(self):
        """Order the current stream after a deferred sparse update of this table (no-op when
        none is pending). Every kernel that reads the table calls this first. With a
        deferred-decay Keras Adam, the rows must have been caught up for this step
        (Embedding.presort) or the optimizer materialized."""
        opt = self.fused_optimizer
        if opt is not None and getattr(opt, "defer_decay", False):
            if self._catchup_step != opt.iterations + 1 and opt._materialized != opt.iterations:
                raise RuntimeError("deferred-decay Keras Adam: rows read without presort() for "
                                   "this step; call the optimizer's materialize() first")
        self.wait_update_raw()

    def wait_update_raw(self):
        ev, self._pending_update = self._pending_update, None
        if ev is not None:
            L.stream_wait_event(torch.cuda.current_stream(self.weight.device), ev)

    @property
    def n_slots(self) -> int:
        return 1 if self.slot_offsets is None else self.slot_offsets.numel() - 1

    def forward(self, ids: torch.Tensor, grad_mask=None) -> torch.Tensor:
        """grad_mask: see functional.embedding_lookup (masked positions carry no gradient)."""
        return embedding_lookup(self, ids, grad_mask)

    def compute_mask(self, ids: torch.Tensor):
        return ids != 0 if self.mask_zero else None

    # ---- fused-optimizer plumbing ----
    @staticmethod
    def _ids_key(ids: torch.Tensor):
        return (ids.data_ptr(), tuple(ids.shape), ids.dtype, ids.device)

    def prefetch(self, ids: torch.Tensor):
        """Queue the radix sort of a LATER step's ids now, on the fused optimizer's sort stream
        (ordered after everything queued so far on the current stream, so `ids` must already be
        written or queued). Call it before the step that precedes the one using `ids`: the sort
        then runs beside this step's kernels instead of delaying the next one. The ids must not
        change until their step has run; a step whose ids match a prefetched sort (same storage,
        shape and dtype) uses it, any other step sorts as usual."""
        opt = self.fused_optimizer
        if opt is None or not torch.is_grad_enabled() or torch.cuda.is_current_stream_capturing():
            return
        key = self._ids_key(ids)
        if key in self._prefetched or any(self._ids_key(q) == key for q in self._prefetch_queue):
            return
        if len(self._prefetch_queue) >= 4:  # bounded like _prefetched: launch what waits
            self.flush_prefetch()
        self._prefetch_queue.append(ids)
        self._prefetch_gen.append(self._presort_gen)
        if not opt.prefetch_after_kernel:
            self.flush_prefetch()

    def flush_prefetch(self):
        """Launch the sorts Embedding.prefetch queued. The fused DLRM step calls this right
        after its train kernel, so the next batch's sort runs beside this step's sparse update
        and dense tail (the train kernel's resident grid leaves no CU slots for it, and a sort
        queued at the next step's start would delay that step's kernel); presort() calls it too,
        when the queue holds its own ids, so a queued sort is never lost."""
        q, self._prefetch_queue, self._prefetch_gen = self._prefetch_queue, [], []
        opt = self.fused_optimizer
        for ids in q:
            key = self._ids_key(ids)
            if len(self._prefetched) >= 4:  # stale entries (steps that never ran)
                self._prefetched.pop(next(iter(self._prefetched)))
            # the entry holds the ids (their storage cannot be reused while it waits) and their
            # version counter (an in-place change before the step voids it)
            self._prefetched[key] = (ids, ids._version, opt.sort_ahead(self, ids))

    def presort(self, ids: torch.Tensor):
        """Queue the radix sort of this step's ids on the fused optimizer's side stream. Call it
        after the step's forward kernels are queued: the host then issues the sort while the
        GPU is busy with the forward, and the sort runs beside it. The lookup's backward reuses
        it (or sorts on the spot when no presort was issued)."""
        if self.fused_optimizer is not None and torch.is_grad_enabled():
            self._presort_gen += 1
            if self._prefetch_queue and (
                    any(self._ids_key(q) == self._ids_key(ids) for q in self._prefetch_queue)
                    or self._prefetch_gen[0] < self._presort_gen - 1):
                # this step's own ids were queued but not sorted yet, or an entry has waited a
                # whole step: paths without the fused DLRM kernel (which flushes right after its
                # train kernel) flush here, so a queued sort never waits more than one step
                self.flush_prefetch()
            e = self._prefetched.pop(self._ids_key(ids), None) if self._prefetched else None
            ahead = e[2] if e is not None and e[1] == ids._version else None
            opt = self.fused_optimizer
            if ahead is None:
                ahead = (opt.sort_ahead(self, ids) if opt.presort_own_stream
                         else opt.sort_async(self, ids))
            self._presorted = (ids, ahead)
            if getattr(opt, "defer_decay", False):
                # replay the step's rows' skipped decay on the stream the sort ran on
                on_sort = getattr(ahead, "ready", None) is not None
                if on_sort:
                    L.stream_wait_event(opt.sort_stream, ahead.ready)
                opt.catch_up(self, ahead, opt.sort_stream if on_sort else opt.side)

    def take_presorted(self, ids: torch.Tensor):
        p, self._presorted = self._presorted, None
        if p is not None and p[0] is ids:
            return p[1]
        return self.fused_optimizer.sort_async(self, ids)

    # ---- sparse gradient plumbing ----
    def accumulate_grad(self, ids: torch.Tensor, grad_rows: torch.Tensor, valid=None):
        """valid (ids' shape, optional): positions flagged 0 carry no gradient (left out by
        take_grad(with_valid=True)'s consumers)."""
        v = None if valid is None else valid.reshape(-1).to(torch.uint8)
        self._pending.append((ids.reshape(-1), grad_rows.reshape(-1, self.output_dim), v))

    def has_grad(self) -> bool:
        return bool(self._pending)

    def take_grad(self, with_valid: bool = False, segments: bool = False):
        """(ids [N] flattened in position order, grad rows [N, dim]) of every lookup since the
        last call, concatenated in call order; clears the pending list. with_valid: a third
        entry, the uint8 [N] flags of positions that carry gradient (None when every lookup
        registered all its positions). segments: the grad rows of 2-4 lookups stay a list of the
        lookups' own [N_i, dim] row views (densify_grad reads them in place, no concatenation)."""
        p, self._pending = self._pending, []
        if not p:
            return None
        if len(p) == 1:
            ids, g, v = p[0]
        else:
            # every lookup holds a multiple of n_slots ids, so position % n_slots stays the slot
            same = all(i.dtype == p[0][0].dtype for i, _, _ in p)
            ids = torch.cat([i if same else i.to(torch.int64) for i, _, _ in p])
            if segments and len(p) <= 4 and all(g.stride(-1) == 1 for _, g, _ in p):
                g = [g for _, g, _ in p]
            else:
                g = torch.cat([g for _, g, _ in p])
            v = None
            if any(x is not None for _, _, x in p):
                v = torch.cat([x if x is not None else torch.ones(i.numel(), dtype=torch.uint8,
                                                                   device=i.device)
                               for i, _, x in p])
        return (ids, g, v) if with_valid else (ids, g)

    def _set_max_slot_rows(self, slot_offsets):
        if slot_offsets is None:
            self.max_slot_rows = self.input_dim
        else:
            so = torch.as_tensor(slot_offsets).to("cpu", torch.int64)
            self.max_slot_rows = max(1, int((so[1:] - so[:-1]).max())) if so.numel() > 1 else 1

    def _load_from_state_dict(self, state_dict, prefix, *args, **kw):
        super()._load_from_state_dict(state_dict, prefix, *args, **kw)
        # the slot-segmented sort trusts max_slot_rows to bound every slot: keep it the
        # loaded offsets' own (a kernel-side guard flags RS_ERRBIT_RANGE if it ever is not)
        self._set_max_slot_rows(self.slot_offsets)

    def zero_grad_pending(self):
        self._pending = []

    def oob_detected(self) -> bool:
        """True if any lookup since the last reset saw an out-of-range id (synchronises)."""
        return bool(self.err_flag.item() & L.RS_ERRBIT_OOB)

    def reset_oob(self):
        self.err_flag.zero_()

    def extra_repr(self):
        return f"{self.input_dim}, {self.output_dim}, mask_zero={self.mask_zero}, slots={self.n_slots}"


class SlabEmbedding(Embedding):
    """Per-slot tables of `cardinalities[s]` rows packed in one slab; ids [..., n_slots]."""

    def __init__(self, cardinalities, dim: int, device=None, **kw):
        card = torch.as_tensor(list(cardinalities), dtype=torch.int64)
        offs = torch.zeros(card.numel() + 1, dtype=torch.int64)
        offs[1:] = torch.cumsum(card, 0)
        super().__init__(int(offs[-1]), dim, device=device, slot_offsets=offs, **kw)
        self.cardinalities = card.tolist()
