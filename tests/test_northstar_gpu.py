"""Full-size parity of the north-star step (BASELINE.json: Criteo DLRM, 26 slots over a 40M x 128
fp32 slab, batch 65 536) — the exact production path bench.py times: composed bottom/top MLP
forward with the top chain fused into the interaction kernel, factored MLP backward, rank-one
interaction backward, fused side-stream radix sort + tiled segmented-sum SGD apply with the
deferred join (ctr/model.py:45-57, ctr/train.py:77-79 SGD path).

oracle/check_dlrm.py states the checks and their tolerances (loss and per-example logits 1e-5,
grad rows 1e-5 of their magnitude bound, sort bit-exact, touched table rows bit-exact against
the oracle's dedup + apply of the kernel's grad rows). Here they run at full size, where the
checked rows include slab rows >= 2^32 / 128 (64-bit row offsets), on three consecutive steps
(after a deferred update, so each forward reads the updated rows). The dense half is checked too:
the twelve MLP parameter gradients per element against the oracle's, and the SGD apply, with the
oracle carrying its own MLP state across the steps. cfg2 (26 x 10M per-slot slab, D 64, B 8192)
runs the same checks; and a step whose batch-deep sum A_top is perturbed by 1 % must fail them.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.timeout(900)
def test_northstar_step_full_size():
    from oracle.check_dlrm import checked_dlrm_sgd_step
    from recommender_amd.ctr.layers import MLP
    from recommender_amd.ctr.train import TrainStep, build_model
    from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

    assert MLP.factored_backward and MLP.composed_forward  # the production defaults
    S, D, B, V, lr = 26, 128, 65536, 40_000_000, 0.01
    dev = torch.device(DEV)
    cards = criteo_cardinalities(V, S)
    g = torch.Generator(device=dev)
    g.manual_seed(4)
    model = build_model("DLRM", D, V, S, 13, dev, slot_cardinalities=cards,
                        bottom=[512, 256, D], top=[512, 256, 1], generator=g)
    step = TrainStep(model, "sgd", lr=lr, fused=True, defer_sparse_join=True)
    assert step.fused_step_ready((torch.zeros(B, S, dtype=torch.int64, device=dev),
                                  torch.zeros(B, 13, device=dev), None))
    rng = np.random.default_rng(4)
    state = {}
    for it in range(3):
        cat, dn, lb = criteo_batch(rng, B, cards)
        r = checked_dlrm_sgd_step(model, step, cat, dn, lb, lr, state)
        print(f"step {it}: {r}")
        assert r["rows_beyond_2^32_elems"] > 0, "no checked row beyond 2^32 elements"
        assert r["touched_rows"] > 200_000


@pytest.mark.timeout(900)
def test_cfg2_step():
    """SURVEY cfg2: DLRM over 26 per-slot tables x 10M rows (one 66.6 GB slab), D 64, B 8192,
    bottom [512, 256, 64], top [512, 256, 1] (ctr/train.py:74-75), SGD; three checked steps."""
    from oracle.check_dlrm import checked_dlrm_sgd_step
    from recommender_amd.ctr.train import TrainStep, build_model
    from recommender_amd.synthetic import criteo_batch

    S, D, B, per, lr = 26, 64, 8192, 10_000_000, 0.01
    dev = torch.device(DEV)
    cards = [per] * S
    g = torch.Generator(device=dev)
    g.manual_seed(4)
    model = build_model("DLRM", D, per * S, S, 13, dev, slot_cardinalities=cards,
                        bottom=[512, 256, D], top=[512, 256, 1], generator=g)
    step = TrainStep(model, "sgd", lr=lr, fused=True, defer_sparse_join=True)
    rng = np.random.default_rng(4)
    state = {}
    try:
        for it in range(3):
            cat, dn, lb = criteo_batch(rng, B, cards)
            r = checked_dlrm_sgd_step(model, step, cat, dn, lb, lr, state)
            print(f"cfg2 step {it}: {r}")
            assert r["rows_beyond_2^32_elems"] > 0
    finally:
        del step, model
        torch.cuda.empty_cache()


def test_dense_half_check_trips_on_perturbed_sum(monkeypatch):
    """The dense-half check can fail: the production step with one entry of its batch-deep sum
    A_top (the factored top-MLP backward's operand) scaled by 1.01 before the dense tail reads it."""
    from oracle.check_dlrm import checked_dlrm_sgd_step
    from recommender_amd import functional
    from recommender_amd.ctr.layers import MLP
    from recommender_amd.ctr.train import TrainStep, build_model
    from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

    monkeypatch.setattr(MLP, "factored_min_batch", 0)
    S, D, B, lr = 26, 128, 2048, 0.05
    dev = torch.device(DEV)
    cards = criteo_cardinalities(400_000, S)
    g = torch.Generator(device=dev)
    g.manual_seed(4)
    model = build_model("DLRM", D, sum(cards), S, 13, dev, slot_cardinalities=cards,
                        bottom=[128, 64, D], top=[128, 64, 1], generator=g)
    step = TrainStep(model, "sgd", lr=lr, fused=True, defer_sparse_join=True)
    rng = np.random.default_rng(4)
    state = {}
    cat, dn, lb = criteo_batch(rng, B, cards)
    checked_dlrm_sgd_step(model, step, cat, dn, lb, lr, state)  # unperturbed: passes
    orig = functional._dense_tail_sgd
    calls = []

    def perturbed(tl, rows, bl, A_top, s_top, P_bot, lr_):
        j = A_top.reshape(-1).abs().argmax()
        A_top.reshape(-1)[j] *= 1.01
        calls.append(1)
        return orig(tl, rows, bl, A_top, s_top, P_bot, lr_)

    monkeypatch.setattr(functional, "_dense_tail_sgd", perturbed)
    cat, dn, lb = criteo_batch(rng, B, cards)
    with pytest.raises(AssertionError, match="top MLP layer"):
        checked_dlrm_sgd_step(model, step, cat, dn, lb, lr, state)
    assert calls, "the production step did not run the dense tail"


@pytest.mark.timeout(900)
def test_northstar_keras_adam_deferred_decay():
    """The reference's active ctr optimizer (ctr/train.py:80,84: Keras Adam on every variable)
    at full north-star size, with the deferred exact decay: three checked steps
    (oracle/check_dlrm.py checked_dlrm_keras_step: every row the steps touched bit-exact in
    table / m / v after materialize(), MLP Keras Adam of its own gradients bit for bit)."""
    from oracle.check_dlrm import checked_dlrm_keras_step
    from recommender_amd.ctr.train import TrainStep, build_model
    from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

    S, D, B, V = 26, 128, 65536, 40_000_000
    dev = torch.device(DEV)
    cards = criteo_cardinalities(V, S)
    g = torch.Generator(device=dev)
    g.manual_seed(4)
    model = build_model("DLRM", D, V, S, 13, dev, slot_cardinalities=cards,
                        bottom=[512, 256, D], top=[512, 256, 1], generator=g)
    step = TrainStep(model, "keras_adam", lr=1e-3, fused=True, defer_sparse_join=True,
                     defer_decay=True)
    assert step.fused_step_ready((torch.zeros(B, S, dtype=torch.int64, device=dev), None, None))
    rng = np.random.default_rng(4)
    state = {}
    try:
        for it in range(3):
            cat, dn, lb = criteo_batch(rng, B, cards)
            r = checked_dlrm_keras_step(model, step, cat, dn, lb, state)
            print(f"keras step {it}: {r}")
            assert r["rows_beyond_2^32_elems"] > 0
    finally:
        del step, model
        torch.cuda.empty_cache()
