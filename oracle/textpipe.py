"""Oracle: the Ali-CCP and Amazon (DIEN) text → id pipelines restated on text — TEST
INFRASTRUCTURE ONLY (see oracle/__init__.py). SURVEY §8f rank 4.

Ali-CCP (esmm/process_public_dataset.py:40-153):
  * common features (:42-50): line `common_id,count,kv` → {field: value} from
    re.split('\\x01|\\x02|\\x03', kv) read as (field, value, weight) triples (dict(zip): the last
    occurrence of a field wins).
  * join (:52-64, :121-137): skeleton line `sample_id,click,purchase,common_id,count,kv`; lines
    with click == '0' and purchase == '1' are dropped; the sample's dict is updated by its common
    dict (common wins); the 18 use_columns values, '0' when absent.
  * vocabulary (:65-90): per column, counting every PRESENT (field, value) of the joined dict; the
    reference's count starts at 0 on first sight (:70-71), so `v1 > 10` keeps values seen at least
    12 times. Ids 1..n per column (:95-96) enumerate a Python set, whose order is unspecified
    (string hashing is salted per process); the build numbers them in first-appearance order
    (first joined line carrying the value) — a deterministic member of the same family.
  * encode (:97-106, :139-153): value (or '0' when absent) → id, 0 when not in the vocabulary.

Amazon / DIEN (dien/util.py:4-37, dien/data_loader.py:27-63):
  * line `label \\t user \\t item \\t cat \\t his_items \\t his_cats` (line.strip().split('\\t')),
    histories split on '\\x02' (an empty field is one empty token).
  * build_vocab: item ids = {target} ∪ history items, cat ids likewise, numbered 1..n (a Python
    set again: first-appearance order here, over the token stream target, h_1, .., h_n per line);
    'mask' = 0, 'unk' = n + 1; item_id2cat_id: the LAST (item, cat) pair in that stream wins
    (dict assignment order), plus 'unk' → 'unk'.
  * parse_line: target item → id or unk; target / history cats → id (unknown raises KeyError:
    index_cat_id tests `cat_id in cat_id`, always true); histories → ids, pad_sequences(maxlen=L,
    padding='post', truncating='pre'): the LAST L tokens, zero-padded at the end.
  * DIEN negatives (:51-55): L items uniform in [1, len(item_vocab)) = [1, n_items + 1] (unk
    included), cat = cat id of item_id2cat_id of the item. The reference draws from NumPy's
    global stream; the build draws Philox keyed by (seed, line, position) — same distribution,
    draw stream unpinned; the oracle takes the draws as input and checks the cat mapping.
"""
from __future__ import annotations

import re

import numpy as np

ALICCP_COLUMNS = ['101', '121', '122', '124', '125', '126', '127', '128', '129', '205', '206',
                  '207', '216', '508', '509', '702', '853', '301']
ALICCP_MIN_SEEN = 10  # `v1 > 10` on a count that starts at 0 (:70-71, :81)


def _lines(text: str):
    return text.replace("\r\n", "\n").splitlines()


def _kv(s: str) -> dict:
    kv = re.split("\x01|\x02|\x03", s)
    return dict(zip(kv[0::3], kv[1::3]))


def aliccp_join(skeleton: str, common: str, cols=ALICCP_COLUMNS):
    """[(click, purchase, values[18] with None when absent)] for the kept skeleton lines."""
    common_d = {}
    for line in _lines(common):
        ll = line.strip().split(",")
        common_d[ll[0]] = _kv(ll[2])
    rows = []
    for line in _lines(skeleton):
        ll = line.strip().split(",")
        if ll[1] == "0" and ll[2] == "1":
            continue
        fd = _kv(ll[5])
        fd.update(common_d[ll[3]])
        rows.append((int(ll[1]), int(ll[2]), [fd.get(k) for k in cols]))
    return rows


def aliccp_vocab(rows, n_cols=len(ALICCP_COLUMNS), min_seen=ALICCP_MIN_SEEN):
    """Per column {value: id} with ids 1.. in first-appearance order."""
    seen = [dict() for _ in range(n_cols)]
    for _, _, vals in rows:
        for c, v in enumerate(vals):
            if v is not None:
                d = seen[c]
                d[v] = d[v] + 1 if v in d else 0
    vocab = []
    for d in seen:
        m, nxt = {}, 1
        for v, c in d.items():  # dict order = first appearance
            if c > min_seen:
                m[v] = nxt
                nxt += 1
        vocab.append(m)
    return vocab


def aliccp_encode(rows, vocab):
    """(ids [n, 18] int32, labels [n, 2] int32 = [click, purchase])."""
    ids = np.array([[vocab[c].get("0" if v is None else v, 0) for c, v in enumerate(vals)]
                    for _, _, vals in rows], np.int32).reshape(-1, len(vocab))
    lab = np.array([[a, b] for a, b, _ in rows], np.int32).reshape(-1, 2)
    return ids, lab


# ---- Amazon / DIEN ------------------------------------------------------------------------


def _dien_fields(line: str):
    f = line.strip().split("\t")
    label, _user, item, cat, his_items, his_cats = f
    return label, item, cat, his_items.split("\x02"), his_cats.split("\x02")


def dien_vocab(text: str):
    """(item_vocab, cat_vocab, item_id2cat_id) as build_vocab makes them (first-appearance
    numbering in place of set order)."""
    items, cats, i2c = {}, {}, {"unk": "unk"}
    for line in _lines(text):
        _, item, cat, hi, hc = _dien_fields(line)
        for it in [item] + hi:
            items.setdefault(it, len(items) + 1)
        for ct in [cat] + hc:
            cats.setdefault(ct, len(cats) + 1)
        i2c[item] = cat
        for it, ct in zip(hi, hc):
            i2c[it] = ct
    items["mask"] = 0
    items["unk"] = len(items)
    cats["mask"] = 0
    cats["unk"] = len(cats)
    return items, cats, i2c


def _pad(seq, maxlen):
    s = seq[-maxlen:]  # truncating='pre'
    return s + [0] * (maxlen - len(s))  # padding='post'


def dien_encode(text: str, items: dict, cats: dict, maxlen: int):
    """{target_item [n,1], target_cat [n,1], pos_his_item [n,L], pos_his_cat [n,L]} int32 and
    label [n, 1] float32; KeyError for an unknown cat, as the reference."""
    ti, tc, hi, hc, lab = [], [], [], [], []
    unk = items["unk"]
    for line in _lines(text):
        label, item, cat, his_i, his_c = _dien_fields(line)
        lab.append([float(label)])
        ti.append([items.get(item, unk)])
        tc.append([cats[cat]])
        hi.append(_pad([items.get(x, unk) for x in his_i], maxlen))
        hc.append(_pad([cats[x] for x in his_c], maxlen))
    n = len(lab)
    return ({"target_item": np.array(ti, np.int32).reshape(n, 1),
             "target_cat": np.array(tc, np.int32).reshape(n, 1),
             "pos_his_item": np.array(hi, np.int32).reshape(n, maxlen),
             "pos_his_cat": np.array(hc, np.int32).reshape(n, maxlen)},
            np.array(lab, np.float32).reshape(n, 1))


def dien_cat_of_item(items: dict, cats: dict, i2c: dict) -> np.ndarray:
    """cat id of every item id 0..n_items+1 (0 for the mask id): the map the negative sampler
    reads (index_cat_id(item_id2cat_id[reverse_vocab[idx]]), data_loader.py:54)."""
    out = np.zeros(len(items), np.int32)
    for it, idx in items.items():
        if it != "mask":
            out[idx] = cats[i2c[it]]
    return out
