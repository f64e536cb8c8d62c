"""CPU: the bucket-histogram AUC (recommender_amd.metrics.auc_from_counts) equals the literal
keras.metrics.AUC restatement (oracle/metrics.py), and both agree with known answers."""
import numpy as np
import pytest

from oracle.metrics import keras_auc
from recommender_amd.metrics import auc_from_counts, keras_thresholds


def bucket_counts(y, p, T):
    thr = keras_thresholds(T)
    b = np.searchsorted(thr, np.asarray(p, np.float32), side="left")  # #thresholds < p
    y = np.asarray(y) != 0
    return (np.bincount(b[~y], minlength=T + 1), np.bincount(b[y], minlength=T + 1))


@pytest.mark.parametrize("T", [3, 200, 20000])
def test_bucket_formulation_matches_keras(rng, T):
    y = rng.random(5000) < 0.3
    p = np.clip(rng.random(5000) * 0.6 + y * 0.3, 0, 1).astype(np.float32)
    p[:10] = [0, 1, 0.5, 1e-8, 1 - 1e-8, 0.25, 0.75, 0.1, 0.9, 0.5]  # exact grid / end points
    ref, _, _ = keras_auc(y, p, T)
    neg, pos = bucket_counts(y, p, T)
    assert abs(auc_from_counts(neg, pos) - ref) < 1e-12


def test_known_answers(rng):
    y = np.r_[np.zeros(500), np.ones(500)]
    assert abs(auc_from_counts(*bucket_counts(y, np.r_[np.full(500, .2), np.full(500, .8)], 200)) - 1.0) < 1e-12
    assert abs(auc_from_counts(*bucket_counts(y, np.r_[np.full(500, .8), np.full(500, .2)], 200))) < 1e-12
    # random scores: close to sklearn's exact AUC at a fine grid
    from sklearn.metrics import roc_auc_score

    y = rng.random(20000) < 0.4
    p = rng.random(20000).astype(np.float32)
    assert abs(auc_from_counts(*bucket_counts(y, p, 20000)) - roc_auc_score(y, p)) < 1e-3


def test_pr_curve_interpolation_runs(rng):
    y = rng.random(2000) < 0.5
    p = np.clip(y * 0.5 + rng.random(2000) * 0.5, 0, 1)
    v = auc_from_counts(*bucket_counts(y, p, 200), curve="PR")
    assert 0.5 < v <= 1.0
