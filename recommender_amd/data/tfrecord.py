"""The reference's Criteo TFRecord files (ctr/tfrecord_io.py:39-96) without TensorFlow.

read_tfrecord  ← read_tfrecord (tfrecord_io.py:78-96: TFRecordDataset → parse_single_example →
                 parse_tensor): the framing is indexed on the host by rs_tfrecord_index (each
                 record's offset depends on every earlier length), the file is copied to HBM once
                 and rs_tfrecord_parse_criteo decodes every Example on the device (one wave per
                 record). Returns the dataset's element structure batched over the whole file:
                 ({'int_features': [n, 13] f32, 'cat_features': [n, 26] i64}, label [n] i64).
write_tfrecord ← write_tfrecord's record layout (tfrecord_io.py:66-75): one Example per row with
                 serialize_tensor blobs and an int64 label (host encoding, CRC32C in C).
encode_tsv     ← write_tfrecord end to end: Criteo TSV → device vocabulary ids, log(x + 1) dense
                 features, labels (recommender_amd.data.criteo) → TFRecord file.
"""
from __future__ import annotations

import ctypes as C
import os
import struct

import numpy as np
import torch

from .. import _lib as L
from .text import text_to_device

NUM_INT, NUM_CAT = 13, 26


def _host_bytes(src) -> np.ndarray:
    if isinstance(src, (str, os.PathLike)):
        return np.fromfile(src, dtype=np.uint8)
    if isinstance(src, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(src), dtype=np.uint8)
    if isinstance(src, np.ndarray):
        return np.ascontiguousarray(src.view(np.uint8).reshape(-1))
    raise TypeError("src must be a path, bytes or a uint8 array")


def index_records(data: np.ndarray, verify_crc: bool = True):
    """(offsets int64 [n], payload lengths int32 [n]) of the records in a host buffer."""
    n_bytes = data.size
    cap = n_bytes // 16 + 1
    offs = np.empty(cap, np.int64)
    lens = np.empty(cap, np.int32)
    n = C.c_int64(0)
    ptr = data.ctypes.data if n_bytes else None
    L.check(L.lib().rs_tfrecord_index(ptr, n_bytes, int(verify_crc), offs.ctypes.data,
                                       lens.ctypes.data, cap, C.byref(n)), "rs_tfrecord_index")
    return offs[: n.value], lens[: n.value]


def read_tfrecord(src, device="cuda", verify_crc: bool = True, n_int: int = NUM_INT,
                  n_cat: int = NUM_CAT):
    """({'int_features', 'cat_features'}, label) of every record, on the device. Raises on
    corrupt framing; a malformed Example raises after the parse (its row is zeroed)."""
    dev = torch.device(device)
    host = _host_bytes(src)
    offs, lens = index_records(host, verify_crc)
    n = offs.size
    text = text_to_device(host, dev)
    dense = torch.empty(n, n_int, dtype=torch.float32, device=dev)
    cat = torch.empty(n, n_cat, dtype=torch.int64, device=dev)
    label = torch.empty(n, dtype=torch.int64, device=dev)
    if n:
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        o = torch.from_numpy(offs).to(dev)
        ln = torch.from_numpy(lens).to(dev)
        L.call("rs_tfrecord_parse_criteo", L.ptr(text), L.ptr(o), L.ptr(ln), n, n_int, n_cat,
               int(verify_crc), L.ptr(dense), L.ptr(cat), L.ptr(label), L.ptr(err),
               L.stream_ptr(dev))
        if int(err.item()) & L.RS_ERRBIT_FORMAT:
            raise ValueError("malformed tf.train.Example record(s) (CRC, key, dtype or shape)")
    return {"int_features": dense, "cat_features": cat}, label


# ---- writer ------------------------------------------------------------------------------
def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _ld(num: int, payload: bytes) -> bytes:
    return _varint((num << 3) | 2) + _varint(len(payload)) + payload


def _tensor(raw: bytes, dtype_code: int, n: int) -> bytes:
    return (_varint(1 << 3) + _varint(dtype_code) + _ld(2, _ld(2, _varint(1 << 3) + _varint(n)))
            + _ld(4, raw))


def _masked_crc(b: bytes) -> int:
    out = C.c_uint32(0)
    buf = np.frombuffer(b, np.uint8)
    L.check(L.lib().rs_crc32c_masked(buf.ctypes.data if buf.size else None, buf.size,
                                      C.byref(out)), "rs_crc32c_masked")
    return out.value


def encode_records(int_features, cat_features, labels) -> bytes:
    """TFRecord bytes: per row an Example {'int_features': serialize_tensor(float32 [13]),
    'cat_features': serialize_tensor(int64 [26]), 'label': int64} (tfrecord_io.py:66-75)."""
    ints = np.ascontiguousarray(np.asarray(int_features, "<f4"))
    cats = np.ascontiguousarray(np.asarray(cat_features, "<i8"))
    labs = np.asarray(labels, np.int64).reshape(-1)
    if ints.ndim != 2 or cats.ndim != 2 or not (ints.shape[0] == cats.shape[0] == labs.size):
        raise ValueError("int_features [n, a], cat_features [n, b], labels [n]")
    out = []
    for i in range(labs.size):
        feats = (_ld(1, _ld(1, b"int_features") + _ld(2, _ld(1, _ld(1, _tensor(ints[i].tobytes(), 1, ints.shape[1])))))
                 + _ld(1, _ld(1, b"cat_features") + _ld(2, _ld(1, _ld(1, _tensor(cats[i].tobytes(), 9, cats.shape[1])))))
                 + _ld(1, _ld(1, b"label") + _ld(2, _ld(3, _ld(1, _varint(int(labs[i])))))))
        payload = _ld(1, feats)
        ln = struct.pack("<Q", len(payload))
        out.append(ln + struct.pack("<I", _masked_crc(ln)) + payload
                   + struct.pack("<I", _masked_crc(payload)))
    return b"".join(out)


def _crc32c_table() -> np.ndarray:
    t = np.arange(256, dtype=np.uint32)
    for _ in range(8):
        t = np.where(t & 1, (t >> 1) ^ np.uint32(0x82F63B78), t >> 1).astype(np.uint32)
    return t


_CRC_TABLE = None


def _masked_crc_rows(rows: np.ndarray) -> np.ndarray:
    """Masked CRC32C (the TFRecord framing checksum) of every row of a [n, m] uint8 array,
    vectorised over the rows: the byte loop runs over the m columns."""
    global _CRC_TABLE
    if _CRC_TABLE is None:
        _CRC_TABLE = _crc32c_table()
    crc = np.full(rows.shape[0], 0xFFFFFFFF, np.uint32)
    for j in range(rows.shape[1]):
        crc = _CRC_TABLE[(crc ^ rows[:, j]) & 0xFF] ^ (crc >> np.uint32(8))
    crc ^= np.uint32(0xFFFFFFFF)
    return (((crc >> np.uint32(15)) | (crc << np.uint32(17))) + np.uint32(0xA282EAD8)).astype(np.uint32)


def encode_records_fixed(int_features, cat_features, labels) -> bytes:
    """encode_records for a whole batch at once, bit-identical: with n_int floats, n_cat int64
    ids and a label in 0..127 every record has the same byte layout, so one template record is
    tiled and the data bytes and payload CRCs are filled column-wise (a 1M-row file in seconds
    instead of a per-record Python loop)."""
    ints = np.ascontiguousarray(np.asarray(int_features, "<f4"))
    cats = np.ascontiguousarray(np.asarray(cat_features, "<i8"))
    labs = np.asarray(labels, np.int64).reshape(-1)
    n = labs.size
    if ints.ndim != 2 or cats.ndim != 2 or not (ints.shape[0] == cats.shape[0] == n):
        raise ValueError("int_features [n, a], cat_features [n, b], labels [n]")
    if n == 0:
        return b""
    if labs.min() < 0 or labs.max() > 127:
        return encode_records(ints, cats, labs)  # varint labels of other widths
    a, b = ints.shape[1], cats.shape[1]
    # a template whose data fields are findable: distinct sentinel values, label 0 vs 1
    si = (np.arange(a, dtype=np.float32) + np.float32(0.3141)).reshape(1, a)
    sc = (np.arange(b, dtype=np.int64) + 0x5EED_0000_0000).reshape(1, b)
    t0 = np.frombuffer(encode_records(si, sc, [0]), np.uint8)
    t1 = np.frombuffer(encode_records(si, sc, [1]), np.uint8)
    rec = t0.size
    io = bytes(t0).find(si.tobytes())
    co = bytes(t0).find(sc.tobytes())
    lo = int(np.flatnonzero(t0[12:rec - 4] != t1[12:rec - 4])[0]) + 12
    out = np.tile(t0, (n, 1))
    out[:, io:io + 4 * a] = ints.view(np.uint8).reshape(n, 4 * a)
    out[:, co:co + 8 * b] = cats.view(np.uint8).reshape(n, 8 * b)
    out[:, lo] = labs.astype(np.uint8)
    out[:, rec - 4:] = _masked_crc_rows(out[:, 12:rec - 4]).astype("<u4").view(np.uint8).reshape(n, 4)
    return out.tobytes()


def write_tfrecord(path, int_features, cat_features, labels):
    with open(path, "wb") as f:
        f.write(encode_records_fixed(int_features, cat_features, labels))


def encode_tsv(vocab, tsv_src, out_path, device="cuda"):
    """write_tfrecord (tfrecord_io.py:39-75): a Criteo TSV through the device vocabulary
    (recommender_amd.data.criteo.CriteoVocab) into the reference's TFRecord layout."""
    cat, dense, label = vocab.encode(tsv_src, device)
    write_tfrecord(out_path, dense.cpu().numpy(), cat.cpu().numpy(),
                   label.cpu().numpy().astype(np.int64))
