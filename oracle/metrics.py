"""Oracle: keras.metrics.AUC [3p TF 2.2] restated literally — TEST INFRASTRUCTURE ONLY.

metrics_utils.update_confusion_matrix_variables compares every prediction with every
threshold (pred > t_i); result() integrates the ROC curve with the trapezoid ('interpolation')
rule. Counts are kept exact (Keras: float32 variables). Callers: ctr/train.py:86,
dien/train.py:43-44, esmm/train.py:164."""
from __future__ import annotations

import numpy as np


def keras_auc(y_true, y_pred, num_thresholds=200):
    eps = 1e-7
    thr = np.array([0.0 - eps] + [(i + 1) * 1.0 / (num_thresholds - 1)
                                  for i in range(num_thresholds - 2)] + [1.0 + eps], np.float32)
    p = np.asarray(y_pred, np.float32).reshape(-1)
    y = np.asarray(y_true).reshape(-1) != 0
    above = p[None, :] > thr[:, None]                      # [T, n]
    tp = (above & y[None]).sum(1).astype(np.float64)
    fp = (above & ~y[None]).sum(1).astype(np.float64)
    fn = y.sum() - tp
    tn = (~y).sum() - fp
    recall = np.divide(tp, tp + fn, out=np.zeros_like(tp), where=(tp + fn) != 0)
    fpr = np.divide(fp, fp + tn, out=np.zeros_like(fp), where=(fp + tn) != 0)
    T = num_thresholds
    return float(np.sum((fpr[: T - 1] - fpr[1:]) * (recall[: T - 1] + recall[1:]) / 2.0)), tp, fp
