"""Oracle: the reference's Criteo TFRecord format (ctr/tfrecord_io.py:39-96) restated in pure
Python — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

TensorFlow is not in this image, so the format is restated from its public specifications:
TFRecord framing (uint64 length, masked CRC32C of the length, payload, masked CRC32C of the
payload; mask(c) = ((c >> 15) | (c << 17)) + 0xa282ead8), the tf.train.Example / Features /
Feature protobufs (example.proto, feature.proto; proto3, so repeated scalars are packed) and
tf.io.serialize_tensor's TensorProto (dtype 1, tensor_shape 2 {dim 2 {size 1}}, tensor_content
4; DT_FLOAT = 1, DT_INT64 = 9). PARITY: pinned only by the CRC32C known answer
(crc32c(b"123456789") = 0xE3069283, RFC 3720 B.4) — no TFRecord file ships with the reference.
"""
from __future__ import annotations

import struct

import numpy as np

_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def varint(v: int) -> bytes:
    v &= (1 << 64) - 1  # int64 two's complement, as protobuf encodes negative int64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def field(num: int, wt: int, payload: bytes) -> bytes:
    tag = varint((num << 3) | wt)
    if wt == 2:
        return tag + varint(len(payload)) + payload
    return tag + payload


def tensor_proto(arr: np.ndarray) -> bytes:
    """tf.io.serialize_tensor of a 1-D float32 / int64 array."""
    dtype = {np.dtype(np.float32): 1, np.dtype(np.int64): 9}[arr.dtype]
    shape = field(2, 2, field(1, 0, varint(arr.shape[0])))
    return (field(1, 0, varint(dtype)) + field(2, 2, shape)
            + field(4, 2, arr.astype(arr.dtype.newbyteorder("<")).tobytes()))


def example(int_features: np.ndarray, cat_features: np.ndarray, label: int) -> bytes:
    """ctr/tfrecord_io.py:69-74: {'int_features': bytes, 'cat_features': bytes, 'label': int64}."""
    def entry(key, feature):
        return field(1, 2, field(1, 2, key.encode()) + field(2, 2, feature))

    bl = lambda b: field(1, 2, field(1, 2, b))            # Feature.bytes_list.value[0]
    il = lambda v: field(3, 2, field(1, 2, varint(v)))    # Feature.int64_list (packed)
    feats = (entry("int_features", bl(tensor_proto(np.asarray(int_features, np.float32))))
             + entry("cat_features", bl(tensor_proto(np.asarray(cat_features, np.int64))))
             + entry("label", il(int(label))))
    return field(1, 2, feats)


def frame(payload: bytes) -> bytes:
    ln = struct.pack("<Q", len(payload))
    return ln + struct.pack("<I", masked_crc(ln)) + payload + struct.pack("<I", masked_crc(payload))


def write_records(int_features, cat_features, labels) -> bytes:
    return b"".join(frame(example(i, c, l)) for i, c, l in zip(int_features, cat_features, labels))


# ---- reader -----------------------------------------------------------------------------
def _rd_varint(b: bytes, p: int):
    v, sh = 0, 0
    while True:
        x = b[p]
        p += 1
        v |= (x & 0x7F) << sh
        if not x & 0x80:
            return v, p
        sh += 7


def _fields(b: bytes):
    """(field number, wire type, value) of one message; value = int or bytes."""
    p = 0
    while p < len(b):
        tag, p = _rd_varint(b, p)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, p = _rd_varint(b, p)
        elif wt == 2:
            n, p = _rd_varint(b, p)
            v, p = b[p:p + n], p + n
        elif wt == 1:
            v, p = b[p:p + 8], p + 8
        elif wt == 5:
            v, p = b[p:p + 4], p + 4
        else:
            raise ValueError("bad wire type")
        yield f, wt, v


def _tensor(b: bytes):
    dtype, dims, content = None, [], None
    for f, wt, v in _fields(b):
        if f == 1:
            dtype = v
        elif f == 2:
            for f2, _, d in _fields(v):
                if f2 == 2:
                    dims.append(dict((ff, vv) for ff, _, vv in _fields(d)).get(1, 0))
        elif f == 4:
            content = v
    dt = {1: "<f4", 9: "<i8"}[dtype]
    return np.frombuffer(content, dt).reshape(dims)


def read_records(data: bytes):
    """(int_features [n, 13] f32, cat_features [n, 26] i64, label [n] i64); raises on a bad CRC."""
    p, ints, cats, labels = 0, [], [], []
    while p < len(data):
        (n,) = struct.unpack_from("<Q", data, p)
        (lc,) = struct.unpack_from("<I", data, p + 8)
        if masked_crc(data[p:p + 8]) != lc:
            raise ValueError("length crc")
        payload = data[p + 12:p + 12 + n]
        (dc,) = struct.unpack_from("<I", data, p + 12 + n)
        if masked_crc(payload) != dc:
            raise ValueError("data crc")
        p += 16 + n
        feats = {}
        for f, _, v in _fields(payload):
            if f == 1:
                for f2, _, e in _fields(v):
                    if f2 == 1:
                        kv = {ff: vv for ff, _, vv in _fields(e)}
                        feats[kv[1].decode()] = kv[2]
        for key in ("int_features", "cat_features"):
            (_, _, bl), = [x for x in _fields(feats[key]) if x[0] == 1]
            (_, _, val), = [x for x in _fields(bl) if x[0] == 1]
            feats[key] = _tensor(val)
        (_, wt, il), = [x for x in _fields(feats["label"]) if x[0] == 3]
        (_, wt2, lv), = [x for x in _fields(il) if x[0] == 1]
        label = _rd_varint(lv, 0)[0] if wt2 == 2 else lv
        ints.append(feats["int_features"])
        cats.append(feats["cat_features"])
        labels.append(label - (1 << 64) if label >= 1 << 63 else label)
    return (np.array(ints, np.float32).reshape(-1, 13), np.array(cats, np.int64).reshape(-1, 26),
            np.array(labels, np.int64))
