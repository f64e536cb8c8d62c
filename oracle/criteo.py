"""Oracle: ctr/tfrecord_io.py build_vocab / write_tfrecord restated on text — TEST
INFRASTRUCTURE ONLY (see oracle/__init__.py).

build_vocab (:15-36): count every categorical token of the train text jointly over the 26
columns (empty → the column's imputation token), keep count > 10, ids in first-appearance
order. write_tfrecord (:39-75): ints ''/negative → 0, log(x + 1) in float32; tokens → id or 0.
The reference's imputation tokens are random strings (unseeded); any per-column token no real
token equals gives the same ids, so `<null:c>` is used. Lines keep their '\\n' as Python's
text-mode iteration gives them (the last token carries it)."""
from __future__ import annotations

import numpy as np

NUM_INT, NUM_CAT, TOTAL = 13, 26, 40
IMPUTE = [f"<null:{c}>" for c in range(NUM_CAT)]


def _lines(text: str):
    return text.replace("\r\n", "\n").splitlines(keepends=True)


def _cats(fields):
    out = []
    for i in range(NUM_INT + 1, TOTAL):
        v = fields[i]
        out.append(IMPUTE[i - NUM_INT - 1] if v in ("", "\n") else v)
    return out


def build_vocab(text: str, min_count: int = 10) -> dict:
    counts = {}
    for line in _lines(text):
        for v in _cats(line.split("\t")):
            counts[v] = counts.get(v, 0) + 1
    vocab, idx = {}, 0
    for key, c in counts.items():
        if c > min_count:
            vocab[key] = idx
            idx += 1
    return vocab


def encode(text: str, vocab: dict):
    cats, dense, label = [], [], []
    for line in _lines(text):
        f = line.split("\t")
        ints = [0 if (s == "" or int(s) < 0) else int(s) for s in f[1:1 + NUM_INT]]
        dense.append(np.log(np.array(ints, np.float32) + np.float32(1)))
        cats.append([vocab.get(v, 0) for v in _cats(f)])
        label.append(float(int(f[0])))
    return (np.array(cats, np.int64).reshape(-1, NUM_CAT), np.array(dense, np.float32).reshape(-1, NUM_INT),
            np.array(label, np.float32))
