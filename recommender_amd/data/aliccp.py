"""Ali-CCP text → device-resident ESMM/MMOE batches (SURVEY §8f rank 4;
esmm/process_public_dataset.py:40-153, esmm/tfrecord_io.py:25-134).

The reference joins sample_skeleton_{train,test}.csv with common_features_{train,test}.csv in
Python (one dict per common line), counts per-column values, keeps values seen at least 12
times (`v1 > 10` on a count that starts at 0, :70-81), numbers them 1..n and writes
ctr_cvr.{train,test} (`click,purchase,<18 ids>`, '0' for OOV), which tfrecord_io.py turns into
TFRecords. Here both raw files are copied to HBM once; csrc/textpipe.hip parses the kv strings,
joins through a device hash map, counts and numbers the vocabulary and encodes the ids:

    rows = aliccp_join(skeleton_train, common_train)          # process_train :42-64
    vocab = AliCCPVocab.build(rows)                            # :65-96
    feats, labels = vocab.encode(rows)                         # ctr_cvr.train → read_tfrecord
    feats_t, labels_t = vocab.encode(aliccp_join(skeleton_test, common_test))   # process_test

`feats` is the model input dict {column: [n, 1] int32} in the reference's `cols` order
(esmm/tfrecord_io.py:4-22), `labels` [n, 2] int32 = [click, purchase]. Id numbering inside a
column is first-appearance order; the reference enumerates a Python set (unspecified order), so
the vocabulary *sets*, counts and OOV behaviour are the parity surface.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .. import _lib as L
from ..optim import SortedIds
from .text import HashTable, collect, count_tokens, fnv1a64, line_index, pow2_at_least, text_to_device

ALICCP_COLUMNS = ['101', '121', '122', '124', '125', '126', '127', '128', '129', '205', '206',
                  '207', '216', '508', '509', '702', '853', '301']  # process_public_dataset.py:21-39
MIN_SEEN = 10  # `v1 > 10` (:81) on the reference's count, which starts at 0 on first sight


@dataclass
class KvLines:
    """rs_kv_parse output for one CSV file."""
    key_hash: torch.Tensor   # [n] int64
    vals: torch.Tensor       # [n, C] int64 (value token hashes)
    present: torch.Tensor    # [n, C] uint8
    keep: torch.Tensor | None
    labels: torch.Tensor | None


def parse_kv_csv(src, key_field: int, kv_field: int, with_labels: bool, columns=ALICCP_COLUMNS,
                 device="cuda") -> KvLines:
    dev = torch.device(device)
    text = text_to_device(src, dev)
    starts, n = line_index(text)
    C = len(columns)
    col_hashes = torch.tensor([fnv1a64(c.encode()) for c in columns], dtype=torch.int64, device=dev)
    key_hash = torch.empty(n, dtype=torch.int64, device=dev)
    vals = torch.empty(n, C, dtype=torch.int64, device=dev)
    present = torch.empty(n, C, dtype=torch.uint8, device=dev)
    keep = torch.empty(n, dtype=torch.int32, device=dev) if with_labels else None
    labels = torch.empty(n, 2, dtype=torch.int32, device=dev) if with_labels else None
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    L.call("rs_kv_parse", L.ptr(text), text.numel(), L.ptr(starts), n, key_field, kv_field,
           int(with_labels), L.ptr(col_hashes), C, L.ptr(key_hash), L.ptr(keep), L.ptr(labels),
           L.ptr(vals), L.ptr(present), L.ptr(err), L.stream_ptr(dev))
    if n and int(err.item()):
        raise ValueError("malformed Ali-CCP line (too few comma fields)")
    return KvLines(key_hash, vals, present, keep, labels)


@dataclass
class JoinedRows:
    """Kept skeleton lines after the common-feature overlay."""
    keys: torch.Tensor     # [n, C] int64 (column, value) hashes; '0' for an absent column
    present: torch.Tensor  # [n, C] uint8
    labels: torch.Tensor   # [n, 2] int32 [click, purchase]

    @property
    def n(self) -> int:
        return self.keys.shape[0]


def aliccp_join(skeleton_src, common_src, columns=ALICCP_COLUMNS, device="cuda") -> JoinedRows:
    """process_train / process_test up to the .tmp file (:42-64, :121-137)."""
    dev = torch.device(device)
    C = len(columns)
    common = parse_kv_csv(common_src, 0, 2, False, columns, dev)       # common_id,count,kv
    skel = parse_kv_csv(skeleton_src, 3, 5, True, columns, dev)        # id,click,buy,common,n,kv
    n_common, n = common.key_hash.numel(), skel.key_hash.numel()
    cap = pow2_at_least(max(2 * n_common, 16))
    mkeys = torch.full((cap,), -1, dtype=torch.int64, device=dev)
    mvals = torch.full((cap,), -1, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    st = L.stream_ptr(dev)
    L.call("rs_map_insert", L.ptr(common.key_hash), n_common, L.ptr(mkeys), L.ptr(mvals), cap,
           L.ptr(err), st)
    out_keys = torch.empty(n, C, dtype=torch.int64, device=dev)
    out_present = torch.empty(n, C, dtype=torch.uint8, device=dev)
    out_labels = torch.empty(n, 2, dtype=torch.int32, device=dev)
    n_kept = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = torch.empty(L.lib().rs_aliccp_join_workspace_size(n), dtype=torch.uint8, device=dev)
    L.call("rs_aliccp_join", L.ptr(skel.keep), n, C, L.ptr(skel.key_hash), L.ptr(skel.vals),
           L.ptr(skel.present), L.ptr(skel.labels), L.ptr(mkeys), L.ptr(mvals), cap,
           L.ptr(common.vals), L.ptr(common.present), L.ptr(out_keys), L.ptr(out_present),
           L.ptr(out_labels), L.ptr(n_kept), L.ptr(err), L.ptr(ws), ws.numel(), st)
    info = torch.cat([n_kept, err]).cpu()
    if int(info[1]):
        raise KeyError("skeleton line refers to an unknown common_feature_index (or map overflow)")
    k = int(info[0])
    return JoinedRows(out_keys[:k], out_present[:k], out_labels[:k])


class AliCCPVocab:
    """The 18 per-column vocabularies as one device hash table keyed by (column, value)."""

    def __init__(self, table: HashTable, sizes: list[int], columns):
        self.table, self.sizes, self.columns = table, sizes, list(columns)

    @property
    def feat_vocab(self) -> dict:
        """{column: number of kept values} — what esmm/train.py:197-215 hard-codes."""
        return dict(zip(self.columns, self.sizes))

    @classmethod
    def build(cls, rows: JoinedRows, min_seen: int = MIN_SEEN, columns=ALICCP_COLUMNS):
        dev = rows.keys.device
        n, C = rows.keys.shape
        cap = pow2_at_least(max(2 * n * C, 1024))
        if n * C >= (1 << 31) or C * max(n, 1) >= (1 << 32):
            raise ValueError("too many rows for one vocabulary pass")
        keys, counts, first, err = count_tokens(rows.keys.reshape(-1), rows.present.reshape(-1), cap)
        # seen ≥ min_seen + 2 ⇔ the reference's count (seen - 1) > min_seen
        first_out, slot_out = collect(keys, counts, first, min_seen + 1)
        if int(err.item()):
            raise RuntimeError("vocabulary hash table overflow")
        k = first_out.numel()
        ids = torch.full((cap,), -1, dtype=torch.int32, device=dev)
        sizes = [0] * C
        if k:
            st = L.stream_ptr(dev)
            sort_key = torch.empty(k, dtype=torch.int64, device=dev)
            group = torch.empty(k, dtype=torch.int32, device=dev)
            L.call("rs_vocab_regroup", L.ptr(first_out), k, C, max(n, 1), L.ptr(sort_key),
                   L.ptr(group), st)
            s = SortedIds(sort_key, C * max(n, 1), count_unique=False)
            L.call("rs_vocab_assign_grouped", L.ptr(s.pos), L.ptr(slot_out), L.ptr(group), k, 1,
                   L.ptr(ids), st)
            sizes = torch.bincount(group, minlength=C).cpu().tolist()
        return cls(HashTable(keys, ids, k), sizes, columns)

    def encode(self, rows: JoinedRows):
        """ctr_cvr rows as the model input: ({column: [n, 1] int32}, labels [n, 2] int32);
        an unseen value (or '0' for an absent column) → 0 (:104, :151)."""
        ids = self.table.lookup_i32(rows.keys, 0)
        return {c: ids[:, i:i + 1] for i, c in enumerate(self.columns)}, rows.labels


def subsample_impressions(labels: torch.Tensor, ratio: int = 5) -> torch.Tensor:
    """Row indices write_impression_tfrecord_with_subsample keeps (esmm/tfrecord_io.py:53-64):
    every click, and the non-clicks whose running non-click count is a multiple of `ratio`."""
    nonclick = labels[:, 0] == 0
    run = torch.cumsum(nonclick.to(torch.int64), 0)
    keep = ~nonclick | (run % ratio == 0)
    return keep.nonzero().squeeze(1)


def click_rows(labels: torch.Tensor) -> torch.Tensor:
    """Row indices write_click_tfrecord keeps (clicked impressions, esmm/tfrecord_io.py:83-86)."""
    return (labels[:, 0] == 1).nonzero().squeeze(1)
