"""Raw text in HBM and its line index (rs_line_index) — shared by the ingestion pipelines."""
from __future__ import annotations

import os

import numpy as np
import torch

from .. import _lib as L

FNV_BASIS, FNV_PRIME = 1469598103934665603, 1099511628211


def fnv1a64(data: bytes) -> int:
    """The token hash the kernels use (csrc/hashtab.hpp), as a signed int64 (torch storage)."""
    h = FNV_BASIS
    for b in data:
        h = ((h ^ b) * FNV_PRIME) & 0xFFFFFFFFFFFFFFFF
    return h - (1 << 64) if h >= (1 << 63) else h


def text_to_device(src, device) -> torch.Tensor:
    """A path, bytes / str, or uint8 array or tensor → a uint8 tensor on `device`."""
    if isinstance(src, torch.Tensor):
        return src.to(device=device, dtype=torch.uint8).contiguous()
    if isinstance(src, str) and not os.path.exists(src) and ("\n" in src or "\t" in src or "," in src):
        src = src.encode()
    if isinstance(src, (str, os.PathLike)):
        data = np.fromfile(src, dtype=np.uint8)
    elif isinstance(src, (bytes, bytearray)):
        data = np.frombuffer(bytearray(src), dtype=np.uint8)
    else:
        data = np.asarray(src, dtype=np.uint8)
    t = torch.from_numpy(data)
    if torch.device(device).type == "cuda":
        t = t.pin_memory()
    return t.to(device, non_blocking=True)


def line_index(text: torch.Tensor):
    """(line_starts int64 [n_newlines + 1], n_lines): one host sync sizes the index. A final
    line without '\\n' counts; an empty text has no lines."""
    dev = text.device
    n_bytes = text.numel()
    if n_bytes == 0:
        return torch.zeros(1, dtype=torch.int64, device=dev), 0
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = torch.empty(L.lib().rs_line_index_workspace_size(n_bytes), dtype=torch.uint8, device=dev)
    st = L.stream_ptr(dev)
    L.call("rs_line_index", L.ptr(text), n_bytes, None, L.ptr(cnt), L.ptr(ws), ws.numel(), st)
    info = torch.stack([cnt[0], text[-1].to(torch.int32)]).cpu()
    n_nl, last_byte = int(info[0]), int(info[1])
    n_lines = n_nl if last_byte == 10 else n_nl + 1
    starts = torch.empty(n_nl + 1, dtype=torch.int64, device=dev)
    L.call("rs_line_index", L.ptr(text), n_bytes, L.ptr(starts), L.ptr(cnt), L.ptr(ws), ws.numel(), st)
    return starts, n_lines


def pow2_at_least(n: int) -> int:
    c = 2
    while c < n:
        c <<= 1
    return c


class HashTable:
    """An open-addressing device table (keys ~0 = empty) with per-slot ids (-1 = none)."""

    def __init__(self, keys: torch.Tensor, ids: torch.Tensor, size: int):
        self.keys, self.ids, self.size = keys, ids, size
        self.capacity = keys.numel()

    def lookup_i32(self, hashes: torch.Tensor, oov_id: int = 0, err: torch.Tensor | None = None):
        out = torch.empty(hashes.shape, dtype=torch.int32, device=hashes.device)
        L.call("rs_vocab_lookup_i32", L.ptr(hashes.contiguous()), hashes.numel(), L.ptr(self.keys),
               L.ptr(self.ids), self.capacity, int(oov_id), int(err is not None), L.ptr(out),
               L.ptr(err), L.stream_ptr(hashes.device))
        return out


def count_tokens(hashes: torch.Tensor, present: torch.Tensor | None, capacity: int):
    """rs_vocab_count(_masked): (keys, counts, first positions) of every (present) token."""
    dev = hashes.device
    keys = torch.full((capacity,), -1, dtype=torch.int64, device=dev)
    counts = torch.zeros(capacity, dtype=torch.int32, device=dev)
    first = torch.full((capacity,), -1, dtype=torch.int64, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    L.call("rs_vocab_count_masked", L.ptr(hashes), L.ptr(present), hashes.numel(), 0, L.ptr(keys),
           L.ptr(counts), L.ptr(first), capacity, L.ptr(err), L.stream_ptr(dev))
    return keys, counts, first, err


def collect(keys, counts, first, min_count: int):
    """Slots with count > min_count: (first positions, slots) in slot order; one sync for the size."""
    dev = keys.device
    cap = keys.numel()
    first_out = torch.empty(cap, dtype=torch.int64, device=dev)
    slot_out = torch.empty(cap, dtype=torch.int32, device=dev)
    n_kept = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = torch.empty(L.lib().rs_vocab_collect_workspace_size(cap), dtype=torch.uint8, device=dev)
    L.call("rs_vocab_collect", L.ptr(keys), L.ptr(counts), L.ptr(first), cap, int(min_count),
           L.ptr(first_out), L.ptr(slot_out), L.ptr(n_kept), L.ptr(ws), ws.numel(),
           L.stream_ptr(dev))
    k = int(n_kept.item())
    return first_out[:k].contiguous(), slot_out[:k].contiguous()
