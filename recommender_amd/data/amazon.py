"""Amazon (DIEN) text → device-resident DIEN/DIN/BASE batches (SURVEY §8f rank 4;
dien/util.py:4-37 build_vocab, dien/data_loader.py:27-75 parse_line / example_generator).

Line format `label \\t user \\t item \\t cat \\t his_items \\t his_cats`, histories separated by
'\\x02'. The reference builds item / cat vocabularies (ids 1..n, 'mask' 0, 'unk' n + 1) and
item_id2cat_id over the train file in Python, then parses every line per example with
pad_sequences(maxlen, padding='post', truncating='pre') and, for DIEN, draws a negative history
of maxlen uniform items in [1, len(item_vocab)) with their cats. Here the text sits in HBM and
csrc/textpipe.hip does every step:

    vocab = DienVocab.build(train_text)                 # util.build_vocab
    feats, label = vocab.encode(text, maxlen=100, sample_negative=True, seed=4)

`feats` matches the reference's feature dict batched: target_item / target_cat [n, 1],
pos_his_item / pos_his_cat (and neg_his_item / neg_his_cat) [n, maxlen], all int32; label
[n, 1] float32. Differences, both unspecified in the reference: ids are numbered in first-
appearance order (the reference enumerates a Python set), and the negative draws come from
Philox keyed by (seed, line, position) instead of NumPy's global stream.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .. import _lib as L
from ..optim import SortedIds
from .text import HashTable, collect, count_tokens, line_index, pow2_at_least, text_to_device


@dataclass
class DienTokens:
    """Line-major ragged token streams of one file: per line the target token, then history."""
    label: torch.Tensor      # [n] f32
    n_hi: torch.Tensor       # [n] int32 history item tokens
    n_hc: torch.Tensor       # [n] int32 history cat tokens
    item_off: torch.Tensor   # [n] int64 stream offset of the line's target item
    cat_off: torch.Tensor
    item_hash: torch.Tensor  # [Σ (1 + n_hi)] int64
    cat_hash: torch.Tensor

    @property
    def n(self) -> int:
        return self.label.numel()


def read_dien_text(src, device="cuda") -> DienTokens:
    dev = torch.device(device)
    text = text_to_device(src, dev)
    starts, n = line_index(text)
    st = L.stream_ptr(dev)
    n_hi = torch.empty(n, dtype=torch.int32, device=dev)
    n_hc = torch.empty(n, dtype=torch.int32, device=dev)
    label = torch.empty(n, dtype=torch.float32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    L.call("rs_dien_parse", L.ptr(text), text.numel(), L.ptr(starts), n, None, None, L.ptr(n_hi),
           L.ptr(n_hc), L.ptr(label), None, None, L.ptr(err), st)
    # stream offsets (exclusive scans of 1 + count) and the two totals in one sync
    ci = torch.cumsum(n_hi.to(torch.int64) + 1, 0)
    cc = torch.cumsum(n_hc.to(torch.int64) + 1, 0)
    zero = torch.zeros(1, dtype=torch.int64, device=dev)
    info = torch.cat([ci[-1:] if n else zero, cc[-1:] if n else zero, err.to(torch.int64)]).cpu()
    if int(info[2]):
        raise ValueError("malformed DIEN line (expected 6 tab-separated fields)")
    item_off = torch.cat([zero, ci[:-1]]) if n else zero[:0]
    cat_off = torch.cat([zero, cc[:-1]]) if n else zero[:0]
    item_hash = torch.empty(int(info[0]), dtype=torch.int64, device=dev)
    cat_hash = torch.empty(int(info[1]), dtype=torch.int64, device=dev)
    L.call("rs_dien_parse", L.ptr(text), text.numel(), L.ptr(starts), n, L.ptr(item_off),
           L.ptr(cat_off), L.ptr(n_hi), L.ptr(n_hc), L.ptr(label), L.ptr(item_hash),
           L.ptr(cat_hash), L.ptr(err), st)
    return DienTokens(label, n_hi, n_hc, item_off, cat_off, item_hash, cat_hash)


def _first_appearance_table(hashes: torch.Tensor) -> HashTable:
    """Every distinct token, ids 1..n in order of first appearance in the stream."""
    dev = hashes.device
    n = hashes.numel()
    cap = pow2_at_least(max(2 * n, 1024))
    keys, counts, first, err = count_tokens(hashes, None, cap)
    first_out, slot_out = collect(keys, counts, first, 0)
    if int(err.item()):
        raise RuntimeError("vocabulary hash table overflow")
    k = first_out.numel()
    ids = torch.full((cap,), -1, dtype=torch.int32, device=dev)
    if k:
        s = SortedIds(first_out, max(n, 1), count_unique=False)
        L.call("rs_vocab_assign_grouped", L.ptr(s.pos), L.ptr(slot_out), None, k, 1, L.ptr(ids),
               L.stream_ptr(dev))
    return HashTable(keys, ids, k)


class DienVocab:
    """item_vocab / cat_vocab / item_id2cat_id of dien/util.py as device tables."""

    def __init__(self, items: HashTable, cats: HashTable, cat_of_item: torch.Tensor):
        self.items, self.cats, self.cat_of_item = items, cats, cat_of_item

    @property
    def n_item_ids(self) -> int:
        """len(item_vocab): the items, 'mask' and 'unk' (the item embedding's vocab size)."""
        return self.items.size + 2

    @property
    def n_cat_ids(self) -> int:
        return self.cats.size + 2

    @property
    def unk_item(self) -> int:
        return self.items.size + 1

    @property
    def unk_cat(self) -> int:
        return self.cats.size + 1

    @classmethod
    def build(cls, train_src, device="cuda"):
        toks = train_src if isinstance(train_src, DienTokens) else read_dien_text(train_src, device)
        dev = toks.label.device
        items = _first_appearance_table(toks.item_hash)
        cats = _first_appearance_table(toks.cat_hash)
        cat_of_item = torch.full((items.size + 2,), -1, dtype=torch.int32, device=dev)
        ws = torch.empty(L.lib().rs_dien_item_cat_workspace_size(items.capacity), dtype=torch.uint8,
                         device=dev)
        L.call("rs_dien_item_cat", L.ptr(toks.item_hash), L.ptr(toks.cat_hash), L.ptr(toks.item_off),
               L.ptr(toks.cat_off), L.ptr(toks.n_hi), L.ptr(toks.n_hc), toks.n, L.ptr(items.keys),
               L.ptr(items.ids), items.capacity, L.ptr(cats.keys), L.ptr(cats.ids), cats.capacity,
               L.ptr(cat_of_item), L.ptr(ws), ws.numel(), L.stream_ptr(dev))
        cat_of_item[0] = 0                      # 'mask' (never drawn)
        cat_of_item[items.size + 1] = cats.size + 1  # item_id2cat_id['unk'] = 'unk'
        return cls(items, cats, cat_of_item)

    def encode(self, src, maxlen: int = 100, sample_negative: bool = False, seed: int = 0,
               line_base: int = 0, device="cuda"):
        """parse_line over every line: (feats, label [n, 1] f32). Raises KeyError for a cat the
        vocabulary lacks (index_cat_id, data_loader.py:31-32) or a drawn item without a cat."""
        toks = src if isinstance(src, DienTokens) else read_dien_text(src, device)
        dev = toks.label.device
        n = toks.n
        i32 = dict(dtype=torch.int32, device=dev)
        ti, tc = torch.empty(n, 1, **i32), torch.empty(n, 1, **i32)
        hi, hc = torch.empty(n, maxlen, **i32), torch.empty(n, maxlen, **i32)
        ni = torch.empty(n, maxlen, **i32) if sample_negative else None
        nc = torch.empty(n, maxlen, **i32) if sample_negative else None
        err = torch.zeros(1, **i32)
        L.call("rs_dien_encode", L.ptr(toks.item_hash), L.ptr(toks.cat_hash), L.ptr(toks.item_off),
               L.ptr(toks.cat_off), L.ptr(toks.n_hi), L.ptr(toks.n_hc), n, L.ptr(self.items.keys),
               L.ptr(self.items.ids), self.items.capacity, self.unk_item, L.ptr(self.cats.keys),
               L.ptr(self.cats.ids), self.cats.capacity, maxlen, L.ptr(self.cat_of_item),
               self.n_item_ids, seed & 0xFFFFFFFFFFFFFFFF, line_base, L.ptr(ti), L.ptr(tc),
               L.ptr(hi), L.ptr(hc), L.ptr(ni), L.ptr(nc), L.ptr(err), L.stream_ptr(dev))
        if n and int(err.item()):
            raise KeyError("cat id not in the vocabulary (index_cat_id)")
        feats = {"target_item": ti, "target_cat": tc, "pos_his_item": hi, "pos_his_cat": hc}
        if sample_negative:
            feats["neg_his_item"], feats["neg_his_cat"] = ni, nc
        return feats, toks.label.view(n, 1)
