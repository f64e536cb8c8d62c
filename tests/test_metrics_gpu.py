"""GPU: rs_auc_update bucket counts bit-exact vs the CPU searchsorted counts; AUC.result()
equals the literal keras.metrics.AUC restatement; accumulation / reset / range check."""
import numpy as np
import pytest
import torch

from oracle.metrics import keras_auc
from recommender_amd.metrics import AUC, keras_thresholds

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T", [200, 10000, 20000])
def test_auc_matches_keras(rng, T):
    y = (rng.random(30000) < 0.25).astype(np.float32)
    p = np.clip(rng.random(30000) * 0.7 + y * 0.3, 0, 1).astype(np.float32)
    m = AUC(num_thresholds=T)
    for a, b in ((0, 10000), (10000, 30000)):  # two update_state calls accumulate
        m.update_state(torch.from_numpy(y[a:b]).cuda(), torch.from_numpy(p[a:b]).cuda())
    thr = keras_thresholds(T)
    bkt = np.searchsorted(thr, p, side="left")
    np.testing.assert_array_equal(m.counts[0].cpu().numpy(), np.bincount(bkt[y == 0], minlength=T + 1))
    np.testing.assert_array_equal(m.counts[1].cpu().numpy(), np.bincount(bkt[y != 0], minlength=T + 1))
    ref, _, _ = keras_auc(y, p, T)
    assert abs(m.result() - ref) < 1e-12
    m.reset_states()
    assert int(m.counts.sum()) == 0


def test_auc_rejects_out_of_range():
    m = AUC()
    m.update_state(torch.tensor([1.0, 0.0]).cuda(), torch.tensor([1.5, 0.2]).cuda())
    with pytest.raises(ValueError):
        m.result()
