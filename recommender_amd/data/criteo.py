"""Criteo TSV → device-resident DLRM/DeepFM batches (ctr/tfrecord_io.py).

The reference builds a joint vocabulary over the 26 categorical columns of the training TSV
(tokens seen more than 10 times get ids 0, 1, .. in first-appearance order; empty fields get a
per-column imputation token; OOV → 0, colliding with the first token), then writes TFRecords
of (log(x + 1) dense features, categorical ids, label). Here the raw text is copied to HBM once
and parsed, hashed, counted, numbered and looked up by the kernels of csrc/criteo.hip; the
result is the (cat_features [n, 26] int64, int_features [n, 13] float32, label [n] float32)
the reference's read_tfrecord yields (tfrecord_io.py:78-96), already on the device.

    vocab = CriteoVocab.build("train.txt")          # build_vocab (tfrecord_io.py:15-36)
    cat, dense, label = vocab.encode("test.txt")     # write_tfrecord + read_tfrecord
"""
from __future__ import annotations

import torch

from .. import _lib as L
from ..optim import SortedIds
from .text import line_index, pow2_at_least, text_to_device

NUM_INT, NUM_CAT = 13, 26
MIN_COUNT = 10  # count > 10 (tfrecord_io.py:33)


def read_criteo_tsv(src, device="cuda"):
    """Parse a Criteo TSV (path, bytes, or a uint8 tensor, possibly already on the device):
    (label [n] f32, dense [n, 13] f32, token hashes [n, 26] uint64 as int64, n_lines).
    One host sync sizes the line index (the newline count)."""
    dev = torch.device(device)
    text = text_to_device(src, dev)
    n_bytes = text.numel()
    if n_bytes == 0:
        z = torch.zeros(0, device=dev)
        return z, z.view(0, NUM_INT), torch.zeros(0, NUM_CAT, dtype=torch.int64, device=dev), 0
    starts, n_lines = line_index(text)
    st = L.stream_ptr(dev)
    label = torch.empty(n_lines, device=dev)
    dense = torch.empty(n_lines, NUM_INT, device=dev)
    hashes = torch.empty(n_lines, NUM_CAT, dtype=torch.int64, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    L.call("rs_criteo_parse", L.ptr(text), n_bytes, L.ptr(starts), n_lines, NUM_INT, NUM_CAT,
           L.ptr(label), L.ptr(dense), L.ptr(hashes), L.ptr(err), st)
    if int(err.item()):
        raise ValueError("malformed Criteo line (field count != 40)")
    return label, dense, hashes, n_lines


class CriteoVocab:
    """The joint categorical vocabulary as a device hash table (key = token hash)."""

    def __init__(self, keys, ids, capacity, size):
        self.keys, self.ids, self.capacity, self.size = keys, ids, capacity, size

    @classmethod
    def build(cls, train_src, min_count: int = MIN_COUNT, device="cuda"):
        dev = torch.device(device)
        _, _, hashes, n_lines = read_criteo_tsv(train_src, dev)
        n_tok = n_lines * NUM_CAT
        if n_tok >= (1 << 31):
            raise ValueError("train file too large for one pass (positions are int32 keys)")
        cap = pow2_at_least(max(2 * n_tok, 1024))
        keys = torch.full((cap,), -1, dtype=torch.int64, device=dev)  # 0xFF.. = empty slot
        counts = torch.zeros(cap, dtype=torch.int32, device=dev)
        first = torch.full((cap,), -1, dtype=torch.int64, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        st = L.stream_ptr(dev)
        L.call("rs_vocab_count", L.ptr(hashes), n_tok, 0, L.ptr(keys), L.ptr(counts), L.ptr(first),
               cap, L.ptr(err), st)
        first_out = torch.empty(cap, dtype=torch.int64, device=dev)
        slot_out = torch.empty(cap, dtype=torch.int32, device=dev)
        n_kept = torch.zeros(1, dtype=torch.int32, device=dev)
        ws = torch.empty(L.lib().rs_vocab_collect_workspace_size(cap), dtype=torch.uint8, device=dev)
        L.call("rs_vocab_collect", L.ptr(keys), L.ptr(counts), L.ptr(first), cap, min_count,
               L.ptr(first_out), L.ptr(slot_out), L.ptr(n_kept), L.ptr(ws), ws.numel(), st)
        if int(err.item()):
            raise RuntimeError("vocabulary hash table overflow")
        k = int(n_kept.item())
        ids = torch.full((cap,), -1, dtype=torch.int32, device=dev)
        if k:
            # first-appearance order: stable radix sort of the kept slots by first position
            s = SortedIds(first_out[:k].contiguous(), max(n_tok, 1), count_unique=False)
            order = s.pos.to(torch.int64)
            sorted_slots = slot_out[:k].index_select(0, order).contiguous()
            L.call("rs_vocab_assign", L.ptr(sorted_slots), k, L.ptr(ids), st)
        return cls(keys, ids, cap, k)

    def lookup(self, hashes: torch.Tensor) -> torch.Tensor:
        out = torch.empty(hashes.shape, dtype=torch.int64, device=hashes.device)
        L.call("rs_vocab_lookup", L.ptr(hashes.contiguous()), hashes.numel(), L.ptr(self.keys),
               L.ptr(self.ids), self.capacity, L.ptr(out), L.stream_ptr(hashes.device))
        return out

    def encode(self, src, device="cuda"):
        """write_tfrecord + read_tfrecord (tfrecord_io.py:39-96): (cat_features [n, 26] int64,
        int_features [n, 13] float32, label [n] float32) on the device."""
        label, dense, hashes, _ = read_criteo_tsv(src, device)
        return self.lookup(hashes), dense, label
