"""Optimizers: sparse appliers for embedding tables (fused HIP segmented-sum + update) and
Keras-semantics dense optimizers for the MLP parameters.

Embedding (a-2):
  SparseSGD        var[u] -= lr * Σ g           (the DLRM SGD path, ctr/train.py:77-79)
  SparseAdam(lazy) Adam on touched rows only     (roofline mode)
  SparseAdam(keras) Keras OptimizerV2 Adam exactly: dense decay of m/v and dense var update of
                   every row (ctr/train.py:80,84 `tf.keras.optimizers.Adam()` defaults)
Dense:
  KerasAdam        Keras Adam update rule on torch tensors (lr_t folding, eps outside sqrt)
  DLRMScheduler    warmup-linear then cosine decay (ctr/util.py:7-37)
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np
import torch

from . import _lib as L
from .embedding import Embedding


def keras_adam_coefficients(step: int, lr=1e-3, beta1=0.9, beta2=0.999, epsilon=1e-7):
    """Keras Adam._prepare_local [3p TF 2.2] in float32; `step` = iterations + 1."""
    f = np.float32
    t = f(step)
    b1p = np.power(f(beta1), t, dtype=np.float32)
    b2p = np.power(f(beta2), t, dtype=np.float32)
    lr_t = f(f(lr) * (np.sqrt(f(f(1) - b2p), dtype=np.float32) / f(f(1) - b1p)))
    return L.AdamParams(float(lr_t), float(f(beta1)), float(f(beta2)), float(f(f(1) - f(beta1))),
                        float(f(f(1) - f(beta2))), float(f(epsilon)))


class _Workspace:
    """Grow-only device scratch buffers keyed by name."""

    def __init__(self):
        self.bufs: dict[str, torch.Tensor] = {}

    def get(self, name, nbytes, device):
        b = self.bufs.get(name)
        if b is None or b.numel() < nbytes or b.device != device:
            b = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
            self.bufs[name] = b
        return b


class SortedIds:
    """Radix-sorted ids of one step (rs_sort_ids_slots / rs_sort_ids_sharded): sorted rows
    (uint32 bits in int32), original positions, device count of distinct valid rows."""

    def __init__(self, ids: torch.Tensor, n_rows: int, slot_offsets: torch.Tensor | None = None,
                 err_flag: torch.Tensor | None = None, ws: _Workspace | None = None,
                 count_unique: bool = True, world: int = 1, valid: torch.Tensor | None = None,
                 max_slot_rows: int | None = None):
        """valid (uint8 [n], optional): positions with 0 are left out (sentinel key, no flag).
        max_slot_rows: the largest slot's row count (host-known; Embedding.max_slot_rows) — it
        lets a slab whose slots are all < 2^24 rows take the slot-segmented sort."""
        ws = ws or _Workspace()
        ids = ids.contiguous()
        L.require_device(ids, "ids")
        n = ids.numel()
        dev = ids.device
        self.n = n
        self.rows = torch.empty(n, dtype=torch.int32, device=dev)
        self.pos = torch.empty(n, dtype=torch.int32, device=dev)
        self.n_unique = torch.zeros(1, dtype=torch.int32, device=dev) if count_unique else None
        n_slots = 1 if slot_offsets is None else slot_offsets.numel() - 1
        nbytes = L.lib().rs_sort_ids_workspace_size(n)
        w = ws.get("sort", nbytes, dev)
        if valid is not None and (world != 1 or valid.numel() != n or valid.dtype != torch.uint8):
            raise ValueError("valid: a uint8 flag per id, one GPU")
        if world == 1:
            msr = int(n_rows) if max_slot_rows is None else int(max_slot_rows)
            L.call("rs_sort_ids_slots", L.ptr(ids), L.id_dtype_code(ids), n,
                   L.ptr(None if valid is None else valid.contiguous()), L.ptr(slot_offsets),
                   n_slots, int(n_rows), msr, L.ptr(self.rows), L.ptr(self.pos),
                   L.ptr(self.n_unique), L.ptr(err_flag), L.ptr(w), w.numel(), L.stream_ptr(dev))
        else:
            L.call("rs_sort_ids_sharded", L.ptr(ids), L.id_dtype_code(ids), n, L.ptr(slot_offsets),
                   n_slots, int(n_rows), int(world), L.ptr(self.rows), L.ptr(self.pos),
                   L.ptr(self.n_unique), L.ptr(err_flag), L.ptr(w), w.numel(), L.stream_ptr(dev))

    @classmethod
    def from_runs(cls, ids: torch.Tensor, n_runs: int, n_rows: int,
                  err_flag: torch.Tensor | None = None) -> "SortedIds":
        """The sort of n_runs equal runs of int32 rows, each ascending with its padding (< 0) at
        the end (a row-sharded owner's received slots, one run per source rank), as the masked
        sort would give it: a merge (rs_sort_ids_runs), one launch."""
        ids = ids.contiguous()
        L.require_device(ids, "ids")
        if ids.dtype != torch.int32:
            raise ValueError("from_runs: int32 rows")
        self = cls.__new__(cls)
        n = ids.numel()
        self.n = n
        self.rows = torch.empty(n, dtype=torch.int32, device=ids.device)
        self.pos = torch.empty(n, dtype=torch.int32, device=ids.device)
        self.n_unique = None
        L.call("rs_sort_ids_runs", L.ptr(ids), n, int(n_runs), int(n_rows), L.ptr(self.rows),
               L.ptr(self.pos), L.ptr(err_flag), L.stream_ptr(ids.device))
        return self

    @classmethod
    def for_table(cls, table: Embedding, ids: torch.Tensor, ws: _Workspace | None = None,
                  count_unique: bool = True, valid: torch.Tensor | None = None):
        return cls(ids, table.input_dim, table.slot_offsets, table.err_flag, ws, count_unique,
                   valid=valid, max_slot_rows=getattr(table, "max_slot_rows", None))


def dedup_grad(table: Embedding, ids: torch.Tensor, grad_rows: torch.Tensor,
               ws: _Workspace | None = None, sorted_ids: SortedIds | None = None):
    """(uniq_rows int64 [U], uniq_grad [U, dim]) — the deduplicated IndexedSlices gradient.
    Synchronises once to read U."""
    ws = ws or _Workspace()
    dev = table.weight.device
    s = sorted_ids or SortedIds.for_table(table, ids, ws)
    n, dim = s.n, table.output_dim
    g = grad_rows.contiguous()
    uniq_rows = torch.empty(n, dtype=torch.int32, device=dev)
    uniq_grad = torch.empty(n, dim, dtype=torch.float32, device=dev)
    nbytes = L.lib().rs_dedup_workspace_size(n, dim)
    w = ws.get("dedup", nbytes, dev)
    L.call("rs_embedding_dedup_grad", L.ptr(s.rows), L.ptr(s.pos), n, L.ptr(g), dim,
           table.input_dim, L.ptr(uniq_rows), L.ptr(uniq_grad), L.ptr(w), w.numel(),
           L.stream_ptr(dev))
    u = int(s.n_unique.item())
    return uniq_rows[:u].to(torch.int64) & 0xFFFFFFFF, uniq_grad[:u]


class SparseOptimizer:
    """Sparse appliers for Embedding tables.

    fused=False: lookups hand (ids, grad rows) to the table; step() sorts and applies.
    fused=True (one lookup per table per step): the ids are radix-sorted on a side HIP stream
    as soon as the lookup (or Embedding.presort) sees them, and the segmented-sum + update runs
    on that stream right after the lookup's backward kernel — overlapping the rest of the
    dense backward. step() joins the side stream into the current one."""
    kind = L.RS_OPT_SGD

    def __init__(self, tables, lr=0.01, fused=False, defer_join=False):
        """defer_join (fused only): step() does not make the current stream wait for the side
        stream; the tables' next readers do (Embedding.wait_update), so the update overlaps
        whatever the next step runs before its first table read (e.g. the bottom MLP). Readers
        outside the engine's kernels must call torch.cuda.synchronize() (or wait_update())."""
        if isinstance(tables, Embedding):
            tables = [tables]
        self.tables = list(tables)
        self.lr = lr
        self.iterations = 0
        self.ws = _Workspace()
        self.fused = fused
        self.defer_join = bool(defer_join) and fused
        self.side = None
        self._applied = set()
        self.sort_stream, self.sort_ws = None, None
        self._dev_events, self._ready_i = {}, 0
        # the step's presort runs on the sort stream (ordered after the current stream only), so
        # it overlaps the previous step's update instead of queueing behind it on the side
        # stream (north star with the early apply: 0.862 -> 0.841 ms/step; RS_PRESORT_STREAM=0
        # restores the side-stream presort)
        self.presort_own_stream = os.environ.get("RS_PRESORT_STREAM", "1") == "1"
        # Embedding.prefetch: launch the later batch's sort right after the current step's train
        # kernel (Embedding.flush_prefetch) instead of at the prefetch call
        self.prefetch_after_kernel = os.environ.get("RS_PREFETCH_AFTER_KERNEL", "1") == "1"
        if fused:
            dev = self.tables[0].weight.device
            self.side = torch.cuda.Stream(device=dev)
            for t in self.tables:
                t.fused_optimizer = self
                # sorts another optimizer prefetched belong to its streams and scratch
                t._prefetched, t._prefetch_queue, t._presorted = {}, [], None

    def _dev_event(self, name):
        """A persistent device-scope event of this optimizer's stream plumbing (None when device
        events are off: the callers then use torch events)."""
        if not L.DEVICE_EVENTS:
            return None
        e = self._dev_events.get(name)
        if e is None:
            e = self._dev_events[name] = L.DeviceEvent()
        return e

    # ---- fused path ----
    def sort_async(self, table: Embedding, ids: torch.Tensor) -> SortedIds:
        main = torch.cuda.current_stream(ids.device)
        self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            s = SortedIds.for_table(table, ids, self.ws, count_unique=False)
        ids.record_stream(self.side)
        return s

    def sort_ahead(self, table: Embedding, ids: torch.Tensor) -> SortedIds:
        """Embedding.prefetch: the sort of a later step's ids on a stream of its own (its own
        scratch), so it can run while this step's update still reads the current sort."""
        dev = ids.device
        if self.sort_stream is None:
            self.sort_stream = torch.cuda.Stream(device=dev)
            self.sort_ws = _Workspace()
        ss = self.sort_stream
        L.stream_wait_stream(ss, torch.cuda.current_stream(dev), self._dev_event("sort_in"))
        with torch.cuda.stream(ss):
            s = SortedIds.for_table(table, ids, self.sort_ws, count_unique=False)
            # a ring of device events: a sort's ready event is waited for within a few steps,
            # and waiting on a later record of this in-order stream only orders more work
            self._ready_i = (self._ready_i + 1) % 4
            s.ready = L.record_event(ss, self._dev_event(f"ready{self._ready_i}"))
        ids.record_stream(ss)
        return s

    def apply_async(self, table: Embedding, ids, grad_rows, sorted_ids: SortedIds, row_scale=None):
        """row_scale [B] (optional): the gradient row of position p is row_scale[p // S] *
        grad_rows[p] with S = ids.shape[-1] (the fused DLRM step's unit rows and G[b])."""
        if id(table) in self._applied:
            raise RuntimeError("fused sparse optimizer: a table was looked up twice in one step")
        self._launch_apply(table, ids, grad_rows, sorted_ids, row_scale)
        self._applied.add(id(table))

    def _launch_apply(self, table, ids, grad_rows, sorted_ids, row_scale=None):
        main = torch.cuda.current_stream(grad_rows.device)
        L.stream_wait_stream(self.side, main, self._dev_event("apply_in"))
        ready = getattr(sorted_ids, "ready", None)
        if ready is not None:  # sorted ahead on the sort stream (Embedding.prefetch)
            L.stream_wait_event(self.side, ready)
            sorted_ids.rows.record_stream(self.side)
            sorted_ids.pos.record_stream(self.side)
        with torch.cuda.stream(self.side):
            self.apply(table, ids, grad_rows, self._params(), sorted_ids=sorted_ids,
                       row_scale=row_scale)
        grad_rows.record_stream(self.side)
        if row_scale is not None:
            row_scale.record_stream(self.side)

    def _params(self) -> L.AdamParams:
        lr = self.lr(self.iterations) if callable(self.lr) else self.lr
        return L.AdamParams(float(np.float32(lr)), 0.0, 0.0, 0.0, 0.0, 0.0)

    def _slots(self, t: Embedding):
        return None, None, None

    def apply(self, table: Embedding, ids: torch.Tensor, grad_rows: torch.Tensor, params,
              sorted_ids: SortedIds | None = None, row_scale: torch.Tensor | None = None,
              valid: torch.Tensor | None = None):
        """valid (uint8 per id, optional): positions flagged 0 carry no gradient and are left out
        of the segmented sums (Embedding.take_grad(with_valid=True))."""
        dev = table.weight.device
        s = sorted_ids or SortedIds.for_table(table, ids, self.ws, count_unique=False, valid=valid)
        g = grad_rows.contiguous()
        m, v, bitmap = self._slots(table)
        nbytes = L.lib().rs_apply_workspace_size(s.n, table.output_dim)
        w = self.ws.get("apply", nbytes, dev)
        group = 1
        if row_scale is not None:
            row_scale = row_scale.contiguous()
            group = ids.shape[-1] if ids.dim() > 1 else s.n // max(row_scale.numel(), 1)
            if row_scale.numel() * group != s.n:
                raise ValueError("row_scale must hold one value per example")
        L.call("rs_embedding_apply_scaled", self.kind, L.ptr(table.weight), L.ptr(m), L.ptr(v),
               table.input_dim, table.output_dim, L.ptr(s.rows), L.ptr(s.pos), s.n, L.ptr(g),
               L.ptr(row_scale), group, params, L.ptr(bitmap), L.ptr(w), w.numel(),
               L.stream_ptr(dev))
        if self.kind == L.RS_OPT_KERAS_ADAM and not getattr(self, "defer_decay", False):
            L.call("rs_keras_adam_dense_sweep", L.ptr(table.weight), L.ptr(m), L.ptr(v),
                   table.input_dim, table.output_dim, params, L.ptr(bitmap), L.stream_ptr(dev))
        elif getattr(self, "defer_decay", False):
            # the step's rows are now current through it (the catch-up left them one behind)
            L.call("rs_keras_adam_mark", L.ptr(self.last[id(table)]), table.input_dim,
                   L.ptr(s.rows), s.n, self.iterations + 1, L.stream_ptr(dev))

    def step(self):
        applied = set()
        if self.fused:
            if self.defer_join:
                ev = L.record_event(self.side, self._dev_event("join"))
                for t in self.tables:
                    t._pending_update = ev
            else:
                torch.cuda.current_stream(self.tables[0].weight.device).wait_stream(self.side)
            applied, self._applied = self._applied, set()
        params = self._params()
        for t in self.tables:
            got = t.take_grad(with_valid=True)
            if got is None:
                if (self.kind == L.RS_OPT_KERAS_ADAM and id(t) not in applied
                        and not getattr(self, "defer_decay", False)):
                    # Keras still decays m/v and moves var densely when the slice is empty
                    m, v, bitmap = self._slots(t)
                    L.call("rs_keras_adam_dense_sweep", L.ptr(t.weight), L.ptr(m), L.ptr(v),
                           t.input_dim, t.output_dim, params, L.ptr(bitmap),
                           L.stream_ptr(t.weight.device))
                continue
            ids, g, valid = got
            if valid is None:
                self.apply(t, ids, g, params)
            else:
                self.apply(t, ids, g, params, valid=valid)
        self.iterations += 1

    def zero_grad(self):
        for t in self.tables:
            t.zero_grad_pending()


class SparseSGD(SparseOptimizer):
    """var[u] -= lr * Σ_{p: id_p = u} g_p. lr may be a float or a schedule step → lr."""
    kind = L.RS_OPT_SGD


class SparseAdam(SparseOptimizer):
    """mode='keras': exact Keras Adam (dense m/v decay + dense var update, 24·V·D bytes/step);
    mode='lazy': the same update restricted to touched rows.

    defer_decay=True (mode='keras', fused=True): the dense decay of rows without a gradient is
    not swept over all V rows each step; each row records the last step applied to it and
    replays the skipped steps, with the sweep's own arithmetic, right before a step reads it
    (Embedding.presort → rs_keras_adam_catchup). `materialize()` brings every row up to date:
    table, m and v then equal the per-step dense sweep's bit for bit. Reading a table outside
    the engine's step (evaluation, checkpoints, tests) needs materialize() first;
    Embedding.wait_update raises otherwise."""

    def __init__(self, tables, lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7, mode="keras",
                 fused=False, defer_join=False, defer_decay=False):
        super().__init__(tables, lr, fused=fused, defer_join=defer_join)
        self.beta_1, self.beta_2, self.epsilon = beta_1, beta_2, epsilon
        if mode not in ("keras", "lazy"):
            raise ValueError("mode must be 'keras' or 'lazy'")
        self.kind = L.RS_OPT_KERAS_ADAM if mode == "keras" else L.RS_OPT_LAZY_ADAM
        self.defer_decay = bool(defer_decay)
        if self.defer_decay and (self.kind != L.RS_OPT_KERAS_ADAM or not fused):
            raise ValueError("defer_decay needs mode='keras' and fused=True")
        self.state = {}
        self.last = {}
        for t in self.tables:
            w = t.weight
            m = torch.zeros_like(w)
            v = torch.zeros_like(w)
            bitmap = (torch.zeros((t.input_dim + 31) // 32, dtype=torch.int32, device=w.device)
                      if self.kind == L.RS_OPT_KERAS_ADAM else None)
            self.state[id(t)] = (m, v, bitmap)
            if self.defer_decay:
                self.last[id(t)] = torch.zeros(t.input_dim, dtype=torch.int32, device=w.device)
                t._catchup_step = 0
        self._lr_host = [0.0]  # lr_t of step s at index s (host mirror of _lr_dev)
        self._lr_dev = None
        self._materialized = 0

    def _slots(self, t):
        if self.state is None:
            raise RuntimeError("SparseAdam state released (the step's graph path owns the Adam "
                               "state: GraphKerasAdam); do not interleave the two paths")
        return self.state[id(t)]

    def release_state(self):
        """Free m / v / bitmaps: a static (graph-capturable) step keeps its own Keras Adam state
        (GraphKerasAdam), so these would be 2x the tables' memory held for nothing."""
        self.state = None
        self.last = {}

    def _lr_of_step(self, s):
        lr = self.lr(s - 1) if callable(self.lr) else self.lr
        return keras_adam_coefficients(s, lr, self.beta_1, self.beta_2, self.epsilon).lr

    def _lr_hist(self, upto, device):
        """Device lr_t history covering steps 1..upto (extended 1024 steps at a time)."""
        if len(self._lr_host) <= upto:
            end = max(upto + 1, len(self._lr_host) + 1024)
            self._lr_host += [self._lr_of_step(s) for s in range(len(self._lr_host), end)]
            self._lr_dev = torch.tensor(self._lr_host, dtype=torch.float32, device=device)
        return self._lr_dev

    def catch_up(self, table, sorted_ids, stream):
        """Queue on `stream` (after the sort of this step's ids) the replay of the decay the
        step's rows skipped; the table's next reader waits for it."""
        step = self.iterations + 1
        dev = table.weight.device
        lr = self._lr_hist(step, dev)
        m, v, _ = self._slots(table)
        if self.fused:
            stream.wait_stream(self.side)  # after the previous step's update of these rows
        with torch.cuda.stream(stream):
            L.call("rs_keras_adam_catchup", L.ptr(table.weight), L.ptr(m), L.ptr(v),
                   L.ptr(self.last[id(table)]), table.input_dim, table.output_dim,
                   L.ptr(sorted_ids.rows), sorted_ids.n, L.ptr(lr), step, self._params(),
                   L.stream_ptr(dev))
            ev = torch.cuda.Event()
            ev.record(stream)
        table._pending_update = ev
        table._catchup_step = step

    def materialize(self):
        """Bring every row of every table up to the last applied step (bit-identical to the
        per-step dense sweep); a no-op without defer_decay."""
        if not self.defer_decay or self._materialized == self.iterations:
            return
        for t in self.tables:
            t.wait_update_raw()
            dev = t.weight.device
            cur = torch.cuda.current_stream(dev)
            if self.fused:
                cur.wait_stream(self.side)
                if self.sort_stream is not None:
                    cur.wait_stream(self.sort_stream)
            lr = self._lr_hist(max(self.iterations, 1), dev)
            m, v, _ = self._slots(t)
            L.call("rs_keras_adam_materialize", L.ptr(t.weight), L.ptr(m), L.ptr(v),
                   L.ptr(self.last[id(t)]), t.input_dim, t.output_dim, L.ptr(lr),
                   self.iterations, self._params(), L.stream_ptr(dev))
        self._materialized = self.iterations

    def _params(self):
        lr = self.lr(self.iterations) if callable(self.lr) else self.lr
        return keras_adam_coefficients(self.iterations + 1, lr, self.beta_1, self.beta_2,
                                       self.epsilon)


class KerasAdam(torch.optim.Optimizer):
    """Keras OptimizerV2 Adam update for dense tensors [3p TF 2.2 _resource_apply_dense]:
    m = b1*m + (1-b1)*g; v = b2*v + (1-b2)*g*g; var -= lr_t*m/(sqrt(v)+eps)."""

    def __init__(self, params, lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        super().__init__(params, dict(lr=lr, beta_1=beta_1, beta_2=beta_2, epsilon=epsilon))
        self.iterations = 0

    @torch.no_grad()
    def step(self, closure=None):
        self.iterations += 1
        for group in self.param_groups:
            c = keras_adam_coefficients(self.iterations, group["lr"], group["beta_1"],
                                        group["beta_2"], group["epsilon"])
            ps = [p for p in group["params"] if p.grad is not None and p.numel() > 0]
            if not ps:
                continue
            ms, vs, gs = [], [], []
            for p in ps:
                st = self.state[p]
                if not st:
                    st["m"] = torch.zeros_like(p)
                    st["v"] = torch.zeros_like(p)
                ms.append(st["m"])
                vs.append(st["v"])
                gs.append(p.grad)
            torch._foreach_mul_(ms, c.beta1)
            torch._foreach_add_(ms, torch._foreach_mul(gs, c.one_minus_beta1))
            torch._foreach_mul_(vs, c.beta2)
            torch._foreach_add_(vs, torch._foreach_mul(torch._foreach_mul(gs, gs), c.one_minus_beta2))
            den = torch._foreach_add(torch._foreach_sqrt(vs), c.epsilon)
            upd = torch._foreach_div(torch._foreach_mul(ms, c.lr), den)
            torch._foreach_sub_(ps, upd)


class GraphKerasAdam:
    """KerasAdam's update (same roundings) over a fixed list of dense tensors, with lr_t read
    from device memory: a window of lr_t values indexed by a device step counter that the
    update advances itself. KerasAdam passes lr_t as a host scalar, which a HIP graph would
    freeze at its capture step; this one can sit inside a graph and be replayed step after
    step (PinSageStep.capture). The tensors are re-pointed to views of one flat buffer (the
    Parameter objects stay), so a step is one gradient concat + one rs_keras_adam_flat launch.
    Call prepare() on the host before each step (it rolls the window, outside any graph);
    gradients are passed to apply() explicitly."""

    def __init__(self, params, lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7, window=4096):
        self.params = list(params)
        self.lr, self.beta_1, self.beta_2, self.epsilon = lr, beta_1, beta_2, epsilon
        dev = self.params[0].device
        sizes = [p.numel() for p in self.params]
        pads = [(-n) % 4 for n in sizes]  # each view 16-byte aligned
        self._segs = []
        off = 0
        for n, pad in zip(sizes, pads):
            self._segs.append((off, n, pad))
            off += n + pad
        self.flat = torch.zeros(off, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p, (o, n, _) in zip(self.params, self._segs):
                self.flat[o:o + n].copy_(p.reshape(-1))
                p.data = self.flat[o:o + n].view_as(p)
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        # the step's gradients in the same layout (padding stays 0): a table's densified gradient
        # is written straight into its view (densify_grad(out=grad_view(i))), other gradients
        # are copied in — no per-step concat of every gradient
        self.grad_flat = torch.zeros_like(self.flat)
        self.iterations = 0
        self.window = int(window)
        self._lr = torch.empty(self.window, dtype=torch.float32, device=dev)
        self._idx = torch.zeros(1, dtype=torch.int64, device=dev)
        self._base = 0
        self._fill()

    def _fill(self):
        vals = [keras_adam_coefficients(self._base + i + 1, self.lr, self.beta_1, self.beta_2,
                                        self.epsilon).lr for i in range(self.window)]
        self._lr.copy_(torch.tensor(vals, dtype=torch.float32))
        self._idx.zero_()

    def prepare(self):
        """Host side, before a step: start a new lr_t window when this one is used up."""
        if self.iterations - self._base >= self.window:
            self._base = self.iterations
            self._fill()

    def grad_view(self, i: int) -> torch.Tensor:
        """Parameter i's slice of the flat gradient buffer, shaped like the parameter."""
        o, n, _ = self._segs[i]
        return self.grad_flat[o:o + n].view_as(self.params[i])

    @torch.no_grad()
    def collect(self, grads):
        """Copy the given gradients (None skipped) into their views of grad_flat, those not
        already written there, in one multi-tensor copy: one launch where per-tensor copies were
        one ~4 us memcpy node each (~25 per DIEN step)."""
        dsts, srcs = [], []
        for i, g in enumerate(grads):
            if g is None:
                continue
            dst = self.grad_view(i)
            if g.data_ptr() != dst.data_ptr():
                dsts.append(dst)
                srcs.append(g.reshape(dst.shape))
        if dsts:
            torch._foreach_copy_(dsts, srcs)

    @torch.no_grad()
    def apply(self, grads):
        """One Keras Adam step of every tensor with `grads` (same order); graph-capturable.
        A None gradient skips its tensor, as Keras' apply_gradients skips a variable without a
        gradient (no m / v decay, no move); a zero gradient still decays m and v and moves the
        variable by lr_t·m/(√v + ε). The tensors with gradients are updated in runs of
        contiguous segments, one rs_keras_adam_flat launch per run."""
        c = keras_adam_coefficients(1, self.lr, self.beta_1, self.beta_2, self.epsilon)
        dev = self.flat.device
        runs, cur = [], None
        for i, g in enumerate(grads):
            if g is None:
                cur = None
                continue
            if cur is None:
                cur = [i, i]
                runs.append(cur)
            cur[1] = i
        self.collect(grads)
        for a, b in runs:
            o = self._segs[a][0]
            ob, nb, pb = self._segs[b]
            n = ob + nb + pb - o
            L.call("rs_keras_adam_flat", L.ptr(self.flat[o:]), L.ptr(self.m[o:]),
                   L.ptr(self.v[o:]), L.ptr(self.grad_flat[o:]), n, L.ptr(self._lr),
                   L.ptr(self._idx), c, L.stream_ptr(dev))
        self._idx.add_(1)


class FusedKerasAdam(GraphKerasAdam):
    """KerasAdam's optimizer interface (zero_grad / step, host-side step count) over
    GraphKerasAdam's flat buffers: a step is one multi-tensor gradient copy and one
    rs_keras_adam_flat launch per run of tensors with gradients, where KerasAdam's nine foreach
    ops launch ≈ 30 multi-tensor kernels (≈ 0.2 ms per cfg4 step). Same roundings as KerasAdam;
    the parameters become views of the flat buffer (the Parameter objects stay)."""

    def zero_grad(self, set_to_none: bool = True):
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    @torch.no_grad()
    def step(self):
        self.prepare()
        self.apply([p.grad for p in self.params])
        self.iterations += 1

    @property
    def state(self) -> dict:
        """KerasAdam's per-parameter state view: {param: {"m", "v"}} (views of the flat moment
        buffers) once a step has run, empty before."""
        if self.iterations == 0:
            return {}
        out = {}
        for p, (o, n, _) in zip(self.params, self._segs):
            out[p] = {"m": self.m[o:o + n].view_as(p), "v": self.v[o:o + n].view_as(p)}
        return out


def densify_grad(table: Embedding, ids: torch.Tensor, grad_rows: torch.Tensor,
                 ws: _Workspace | None = None, valid: torch.Tensor | None = None,
                 out: torch.Tensor | None = None) -> torch.Tensor:
    """The IndexedSlices gradient as a dense [input_dim, dim] tensor with no host sync. Small
    tables (input_dim·dim <= 16384): rs_embedding_grad_dense_small (one pass, fixed block /
    lane order); others: deterministic segmented sum (rs_embedding_grad_dense: position order
    per row, each row's sum stored in place, untouched rows 0). valid (uint8 per id, optional):
    positions flagged 0 are left out — for lookups whose masked positions carry no gradient
    (Embedding.accumulate_grad's valid). out (optional, contiguous fp32 [input_dim, dim]): the
    gradient is written there (every element) instead of into a new tensor. grad_rows may be a
    list of 1-4 [N_i, dim] row views (Embedding.take_grad(segments=True): one per lookup, row
    stride free, unit column stride), read in place as if concatenated."""
    ws = ws or _Workspace()
    dev = table.weight.device
    dim, V = table.output_dim, table.input_dim
    if out is not None and (tuple(out.shape) != (V, dim) or out.dtype != torch.float32
                            or not out.is_contiguous()):
        raise ValueError("out must be a contiguous fp32 [input_dim, dim] tensor")
    if isinstance(grad_rows, (list, tuple)):
        segs = list(grad_rows)
        if (len(segs) > 4 or (valid is None and V * dim <= 16384)
                or any(g.dim() != 2 or g.shape[1] != dim or g.stride(1) != 1
                       or (g.shape[0] > 1 and g.stride(0) < dim) for g in segs)):
            grad_rows = torch.cat([g.reshape(-1, dim) for g in segs])  # the one-array paths
        else:
            s = SortedIds.for_table(table, ids, ws, count_unique=False, valid=valid)
            dense = out if out is not None else torch.empty(V, dim, dtype=torch.float32, device=dev)
            w = ws.get("dense", L.lib().rs_apply_workspace_size(s.n, dim), dev)
            k = len(segs)
            ptrs = (C.c_void_p * 4)(*[g.data_ptr() for g in segs])
            ns = (C.c_int64 * 4)(*[g.shape[0] for g in segs])
            lds = (C.c_int64 * 4)(*[g.stride(0) if g.shape[0] > 1 else dim for g in segs])
            L.call("rs_embedding_grad_dense_segs", L.ptr(s.rows), L.ptr(s.pos), s.n, k,
                   C.cast(ptrs, C.c_void_p), C.cast(ns, C.c_void_p), C.cast(lds, C.c_void_p), dim,
                   V, L.ptr(dense), L.ptr(w), w.numel(), L.stream_ptr(dev))
            return dense
    if valid is None and V * dim <= 16384 and dim <= 256 and dim & (dim - 1) == 0:
        # small table (PinSage year / genre): one pass, per-block LDS copies, no sort
        ids = ids.reshape(-1).contiguous()
        n = ids.numel()
        dense = out if out is not None else torch.empty(V, dim, dtype=torch.float32, device=dev)
        w = ws.get("dense_small", L.lib().rs_embedding_grad_dense_small_workspace_size(n, V, dim),
                   dev)
        L.call("rs_embedding_grad_dense_small", L.ptr(ids), L.id_dtype_code(ids), n,
               L.ptr(grad_rows.contiguous()), dim, V, L.ptr(dense), L.ptr(table.err_flag),
               L.ptr(w), w.numel(), L.stream_ptr(dev))
        return dense
    s = SortedIds.for_table(table, ids, ws, count_unique=False, valid=valid)
    n = s.n
    dense = out if out is not None else torch.empty(V, dim, dtype=torch.float32, device=dev)
    w = ws.get("dense", L.lib().rs_apply_workspace_size(n, dim), dev)
    L.call("rs_embedding_grad_dense", L.ptr(s.rows), L.ptr(s.pos), n, L.ptr(grad_rows.contiguous()),
           dim, V, L.ptr(dense), L.ptr(w), w.numel(), L.stream_ptr(dev))
    return dense


class DLRMScheduler:
    """ctr/util.py:7-37: lr = initial*step/warmup for step <= warmup, else cosine decay to
    alpha over decay_steps."""

    def __init__(self, initial_learning_rate, warmup_steps, decay_steps, alpha):
        self.initial_learning_rate = initial_learning_rate
        self.warmup_steps = warmup_steps
        self.decay_steps = decay_steps
        self.alpha = alpha

    def __call__(self, step):
        f = np.float32
        step = f(step)
        warm = f(self.warmup_steps)
        if step <= warm:
            return float(f(step / warm) * f(self.initial_learning_rate))
        g = min(step, f(warm + f(self.decay_steps)))
        frac = f((g - warm) / f(self.decay_steps))
        cos = f(0.5) * (f(1.0) + f(math.cos(f(math.pi) * frac)))
        decayed = f((f(1) - f(self.alpha)) * cos + f(self.alpha))
        return float(f(self.initial_learning_rate) * decayed)
