"""Full-size parity of the north-star step (BASELINE.json: Criteo DLRM, 26 slots over a 40M x 128
fp32 slab, batch 65 536) — the exact production path bench.py times: composed bottom/top MLP
forward with the top chain fused into the interaction kernel, factored MLP backward, rank-one
interaction backward, fused side-stream radix sort + tiled segmented-sum SGD apply with the
deferred join (ctr/model.py:45-57, ctr/train.py:77-79 SGD path).

oracle/check_dlrm.py states the checks and their tolerances (loss and per-example logits 1e-5,
grad rows 1e-5 of their magnitude bound, sort bit-exact, touched table rows bit-exact against
the oracle's dedup + apply of the kernel's grad rows). Here they run at full size, where the
checked rows include slab rows >= 2^32 / 128 (64-bit row offsets), on the second step too
(after a deferred update, so the second forward reads the updated rows).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.timeout(600)
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
    rng = np.random.default_rng(4)
    for it in range(2):
        cat, dn, lb = criteo_batch(rng, B, cards)
        r = checked_dlrm_sgd_step(model, step, cat, dn, lb, lr)
        print(f"step {it}: {r}")
        assert r["rows_beyond_2^32_elems"] > 0, "no checked row beyond 2^32 elements"
        assert r["touched_rows"] > 200_000
