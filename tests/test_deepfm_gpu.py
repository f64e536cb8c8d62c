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


def test_deepfm_static_and_graph_step_equal_eager():
    """TrainStep.static_step (the table's gradient densified, Keras Adam over every variable
    with lr_t from device memory: graph-capturable) equals the eager Keras-Adam step (KerasAdam
    + SparseAdam(keras) with its dense sweep) bit for bit over 3 steps at cfg1's shape, and the
    step captured into a HIP graph and replayed on refilled input buffers stays within 1e-5 of
    the eager static steps (the library GEMMs may pick another algorithm under capture)."""
    V, D, B, S = 1_000_000, 16, 1024, 26
    rng = np.random.default_rng(9)
    batches = []
    for _ in range(3):
        cat, dn, lb = criteo_batch(rng, B, [V] * S)
        batches.append(tuple(torch.from_numpy(x).to(DEV) for x in (cat % V, dn, lb)))

    def run(mode):
        g = torch.Generator(device=DEV)
        g.manual_seed(4)
        m = build_model("DeepFM", D, V, S, 13, torch.device(DEV), generator=g)
        st = TrainStep(m, "keras_adam", fused=False)
        static = tuple(torch.empty_like(t) for t in batches[0])
        replay, losses = None, []
        for i, b in enumerate(batches):
            if mode == "eager":
                losses.append(float(st(b)))
            elif mode == "static" or i == 0:
                losses.append(float(st.static_step(b)))
            else:
                for d, s in zip(static, b):
                    d.copy_(s)
                replay = replay or st.capture_static(static)
                losses.append(float(replay()))
        torch.cuda.synchronize()
        params = {n: p.detach().cpu().numpy().copy() for n, p in m.named_parameters()
                  if not n.endswith("grad_handle")}
        params["table"] = m.embedding_layer.weight.detach().cpu().numpy().copy()
        return losses, params

    (le, pe), (ls, ps), (lg, pg) = run("eager"), run("static"), run("graph")
    assert le == ls, (le, ls)
    for n in pe:
        np.testing.assert_array_equal(ps[n], pe[n], err_msg=f"static vs eager: {n}")
    np.testing.assert_allclose(lg, ls, rtol=1e-5)
    for n in ps:
        np.testing.assert_allclose(pg[n], ps[n], rtol=1e-5, atol=1e-7, err_msg=f"graph: {n}")
