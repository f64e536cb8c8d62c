"""GPU parity: the DeepFM train step at SURVEY cfg1's shape (shared 1M x 16 table, batch 1024,
26 slots + 13 dense, MLP [512, 256, 1], Keras Adam; ctr/model.py:6-31, ctr/train.py:81-85)
against oracle/ctr.py over 3 chained steps (oracle/check_deepfm.py states the tolerances:
logits 1e-5, table / m / v bit-exact from the kernel's gradient rows)."""
import numpy as np
import pytest
import torch

from oracle.check_deepfm import checked_deepfm_adam_step
from recommender_amd.ctr.train import TrainStep, build_model
from recommender_amd.synthetic import criteo_batch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("fused", [True, False])
def test_deepfm_cfg1_keras_adam_three_steps(fused):
    V, D, B, S = 1_000_000, 16, 1024, 26
    g = torch.Generator(device=DEV)
    g.manual_seed(4)
    model = build_model("DeepFM", D, V, S, 13, torch.device(DEV), generator=g)
    step = TrainStep(model, "keras_adam", fused=fused)
    rng = np.random.default_rng(4)
    for i in range(3):
        cat, dn, lb = criteo_batch(rng, B, [V] * S)
        r = checked_deepfm_adam_step(model, step, cat % V, dn, lb)
        print(f"step {i}: {r}")
