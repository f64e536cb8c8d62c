"""CPU checks of the PinSage evaluation restatement (oracle/pinsage.py eval section,
recommender_amd/pinsage/evaluation.py host helpers) against the reference's own formulas
(pinsage/train/util.py:5-39 with pandas, evaluation.py:54-65 with scipy), re-expressed here."""
import numpy as np
import pandas as pd
from scipy import sparse as ssp

from oracle import pinsage as O
from recommender_amd.pinsage.evaluation import build_val_test_matrix, train_test_split_by_time


def pandas_split(users, ts):
    df = pd.DataFrame({"user": users, "ts": ts})
    df["train_mask"] = True
    df["val_mask"] = False
    df["test_mask"] = False

    def per_user(d):
        d = d.sort_values(["ts"])
        if d.shape[0] > 1:
            d.iloc[-1, -3], d.iloc[-1, -1] = False, True
        if d.shape[0] > 2:
            d.iloc[-2, -3], d.iloc[-2, -2] = False, True
        return d

    df = df.groupby("user", group_keys=False).apply(per_user).sort_index()
    return tuple(df[c].to_numpy().nonzero()[0] for c in ("train_mask", "val_mask", "test_mask"))


def test_split_matches_pandas_formulation():
    rng = np.random.default_rng(3)
    users = rng.integers(0, 60, 800)
    ts = rng.permutation(800)  # distinct times (pandas' sort is not stable)
    ref = pandas_split(users, ts)
    for got in (train_test_split_by_time(users, ts), O.split_by_time(users, ts)):
        assert all(np.array_equal(a, b) for a, b in zip(got, ref))


def test_hit_rate_matches_scipy_formulation():
    rng = np.random.default_rng(1)
    U, I, K = 200, 90, 10
    users = rng.integers(0, U, 300)
    items = rng.integers(0, I, 300)
    val, _ = build_val_test_matrix(users, items, np.arange(300), np.arange(0), U, I)
    gt = val.tocsr()
    recs = np.stack([rng.choice(I, K, replace=False) for _ in range(U)])
    rel = np.asarray(gt[np.repeat(np.arange(U), K), recs.flatten()]).reshape(U, K)
    ref = (rel != 0).any(axis=1).mean()
    got, _ = O.hit_rate(recs, gt.indptr, gt.indices)
    assert got == ref


def test_masked_topk_oracle_ties_and_exclusion():
    s = np.array([[1.0, 3.0, 3.0, 2.0, 3.0]], np.float32)
    assert O.masked_topk(s, 3).tolist() == [[1, 2, 4]]
    assert O.masked_topk(s, 3, np.array([0, 2]), np.array([2, 1])).tolist() == [[4, 3, 0]]
    ip = np.array([0, 5])
    assert O.masked_topk(s, 5, ip, np.arange(5)).tolist() == [[0, 1, 2, 3, 4]]  # all -inf


def test_latest_item_ties():
    ip = np.array([0, 3, 3, 5])
    u2i = np.array([4, 7, 9, 2, 1])
    ts = np.array([5, 9, 9, 1, 0])
    assert O.latest_item(ip, u2i, ts).tolist() == [7, -1, 2]
