"""Device metrics: Keras' thresholded AUC.

AUC(num_thresholds=200, curve='ROC', summation_method='interpolation') mirrors
keras.metrics.AUC [3p TF 2.2] as the reference uses it (ctr/train.py:86 default 200,
dien/train.py:43-44 20000, esmm/train.py:164 10000): update_state(y_true, y_pred) on device
(rs_auc_update: one bucket histogram pass), result() from the exact int64 counts, reset_states().
Curves: ROC (interpolation / minoring / majoring) and PR (interpolation, Davis & Goadrich)."""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L

EPSILON = 1e-7  # keras backend epsilon


def keras_thresholds(num_thresholds: int) -> np.ndarray:
    """metrics.AUC.__init__: [0 - eps] + [(i + 1) / (T - 1) for i in range(T - 2)] + [1 + eps],
    stored as float32."""
    t = [(i + 1) * 1.0 / (num_thresholds - 1) for i in range(num_thresholds - 2)]
    return np.array([0.0 - EPSILON] + t + [1.0 + EPSILON], dtype=np.float32)


def auc_from_counts(neg: np.ndarray, pos: np.ndarray, curve: str = "ROC",
                    summation_method: str = "interpolation") -> float:
    """AUC.result() from per-bucket counts (bucket b = #thresholds < prediction)."""
    T = neg.size - 1
    # TP_i = Σ_{b > i} pos[b] (prediction above threshold i)
    tp = np.cumsum(pos[::-1])[::-1][1:].astype(np.float64)
    fp = np.cumsum(neg[::-1])[::-1][1:].astype(np.float64)
    fn = pos.sum() - tp
    tn = neg.sum() - fp

    def div(a, b):
        return np.divide(a, b, out=np.zeros_like(a), where=b != 0)

    if curve == "PR" and summation_method == "interpolation":
        dtp = tp[: T - 1] - tp[1:]
        p = tp + fp
        dp = p[: T - 1] - p[1:]
        prec_slope = div(dtp, np.maximum(dp, 0))
        intercept = tp[1:] - prec_slope * p[1:]
        safe_p_ratio = np.where((p[: T - 1] > 0) & (p[1:] > 0), div(p[: T - 1], np.maximum(p[1:], 0)),
                                np.ones_like(p[1:]))
        pr_auc_increment = div(prec_slope * (dtp + intercept * np.log(safe_p_ratio)),
                               np.maximum(tp[1:] + fn[1:], 0))
        return float(np.sum(pr_auc_increment))
    recall = div(tp, tp + fn)
    if curve == "ROC":
        x, y = div(fp, fp + tn), recall
    else:  # PR with riemann sums
        x, y = recall, div(tp, tp + fp)
    if summation_method == "interpolation":
        heights = (y[: T - 1] + y[1:]) / 2.0
    elif summation_method == "minoring":
        heights = np.minimum(y[: T - 1], y[1:])
    else:
        heights = np.maximum(y[: T - 1], y[1:])
    return float(np.sum((x[: T - 1] - x[1:]) * heights))


class AUC:
    def __init__(self, num_thresholds: int = 200, curve: str = "ROC",
                 summation_method: str = "interpolation", name: str | None = None, device="cuda"):
        if num_thresholds <= 1:
            raise ValueError("num_thresholds must be > 1")
        self.num_thresholds = num_thresholds
        self.curve = curve.upper()
        self.summation_method = summation_method.lower()
        self.name = name
        self.device = torch.device(device)
        self.thresholds = torch.from_numpy(keras_thresholds(num_thresholds)).to(self.device)
        self.counts = torch.zeros(2, num_thresholds + 1, dtype=torch.int64, device=self.device)
        self.err_flag = torch.zeros(1, dtype=torch.int32, device=self.device)

    def update_state(self, y_true, y_pred, sample_weight=None):
        if sample_weight is not None:
            raise NotImplementedError("sample_weight is not used by the reference")
        p = torch.as_tensor(y_pred, device=self.device).reshape(-1).float().contiguous()
        y = torch.as_tensor(y_true, device=self.device).reshape(-1).float().contiguous()
        if p.numel() != y.numel():
            raise ValueError("y_true and y_pred sizes differ")
        L.call("rs_auc_update", L.ptr(p), L.ptr(y), p.numel(), L.ptr(self.thresholds),
               self.num_thresholds, L.ptr(self.counts), L.ptr(self.err_flag),
               L.stream_ptr(self.device))

    def result(self) -> float:
        c = self.counts.cpu().numpy()
        if int(self.err_flag.item()):
            raise ValueError("predictions must be in [0, 1] (keras.metrics.AUC asserts this)")
        return auc_from_counts(c[0], c[1], self.curve, self.summation_method)

    def reset_states(self):
        self.counts.zero_()
        self.err_flag.zero_()
