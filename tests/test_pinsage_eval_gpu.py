"""GPU parity for the PinSage evaluation (pinsage/train/evaluation.py):
latest item per user, masked top-k, hit flags — bit-exact against oracle/pinsage.py. The
end-to-end recommend() uses small-integer item representations, so the fp32 similarity GEMM
is exact and the top-k (with its many ties) must match the oracle exactly too."""
import numpy as np
import pytest
import torch

from oracle import pinsage as O
from recommender_amd.pinsage import PinSageModel, PinSageSampler
from recommender_amd.pinsage.evaluation import (build_val_test_matrix, get_item_reprs,
                                                hit_rate_eval, latest_items, masked_topk,
                                                recommend, train_test_split_by_time)
from recommender_amd.pinsage.graph import HeteroGraph

pytestmark = pytest.mark.gpu
DEV = "cuda"


def graph_with_time(seed=0, n_users=80, n_items=150, n_edges=1500):
    rng = np.random.default_rng(seed)
    u = np.concatenate([np.arange(n_users), rng.integers(0, n_users, n_edges)])
    i = rng.integers(0, n_items, u.size)
    key = np.unique(u * n_items + i)
    u, i = key // n_items, key % n_items
    ts = rng.integers(0, 40, u.size)  # many equal timestamps
    year = rng.integers(0, 12, n_items)
    genre = (rng.random((n_items, 6)) < 0.3).astype(np.int8)
    g = HeteroGraph(u, i, n_users, n_items, device=DEV, item_data={"year": year, "genre": genre},
                    edge_data={"timestamp": ts})
    return g, u, i, ts


def test_latest_item_bit_exact():
    g, u, i, ts = graph_with_time()
    got = latest_items(g, "timestamp").cpu().numpy()
    ip = g.u2i_indptr.cpu().numpy()
    ref = O.latest_item(ip, g.u2i.cpu().numpy(), g.u2i_edata["timestamp"].cpu().numpy())
    assert np.array_equal(got, ref)


def test_latest_item_missing_user_raises():
    g = HeteroGraph(np.array([0, 0]), np.array([1, 2]), 3, 4, device=DEV,
                    edge_data={"timestamp": np.array([1, 2])})
    with pytest.raises(ValueError):
        latest_items(g, "timestamp")


@pytest.mark.parametrize("R,I,K,excl", [(7, 5, 5, False), (64, 100, 10, True),
                                        (33, 3706, 10, True), (5, 3706, 17, True),
                                        (9, 1000, 33, False), (4, 27278, 64, True),
                                        (3, 40, 1, True)])
def test_masked_topk_bit_exact(R, I, K, excl):
    rng = np.random.default_rng(R * 1000 + K)
    scores = rng.integers(-20, 20, (R, I)).astype(np.float32)  # dense ties
    ip = it = g = None
    if excl:
        u = np.repeat(np.arange(R), rng.integers(0, min(I, 50), R))
        it_ = rng.integers(0, I, u.size)
        key = np.unique(u * I + it_)
        g = HeteroGraph(key // I, key % I, R, I, device=DEV)
        ip, it = g.u2i_indptr.cpu().numpy(), g.u2i.cpu().numpy()
    idx, val = masked_topk(torch.from_numpy(scores).to(DEV), K, 0, g, with_scores=True)
    ref = O.masked_topk(scores, K, ip, it)
    assert np.array_equal(idx.cpu().numpy(), ref)
    assert np.array_equal(val.cpu().numpy(),
                          np.take_along_axis(O.masked_topk_scores(scores, ip, it), ref, 1))


def test_recommend_and_hit_rate_exact():
    g, u, i, ts = graph_with_time(seed=2)
    rng = np.random.default_rng(5)
    reprs = torch.from_numpy(rng.integers(-3, 4, (g.n_items, 16)).astype(np.float32)).to(DEV)
    for bs in (32, 100000):
        recs = recommend(g, 10, reprs, None, "user", "timestamp", bs).cpu().numpy()
        ip, u2i = g.u2i_indptr.cpu().numpy(), g.u2i.cpu().numpy()
        latest = O.latest_item(ip, u2i, g.u2i_edata["timestamp"].cpu().numpy())
        r = reprs.cpu().numpy()
        ref = O.masked_topk(r[latest] @ r.T, 10, ip, u2i)
        assert np.array_equal(recs, ref)
    val_idx = rng.choice(u.size, 200, replace=False)
    val, _ = build_val_test_matrix(u, i, val_idx, val_idx[:0], g.n_users, g.n_items)
    hr = hit_rate_eval(torch.from_numpy(ref).to(DEV), val)
    gt = val.tocsr()
    gt.sort_indices()
    assert hr == O.hit_rate(ref, gt.indptr, gt.indices)[0]


def test_item_reprs_are_per_batch_reprs():
    """get_item_reprs = model.get_repr of each batch of seeds, all at one sampler step (the
    batch-global Frobenius norm makes the result batch-size dependent, as in the reference)."""
    g, *_ = graph_with_time(seed=4)
    torch.manual_seed(0)
    model = PinSageModel(g, g.itype, 2, 8, 32, 16)
    smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
    step0 = smp.step
    a = get_item_reprs(model, smp, g, g.itype, 32)
    assert a.shape == (g.n_items, 16) and smp.step == step0 + 1
    with torch.no_grad():
        for b0 in (0, 64, 128):
            smp.step = step0
            seeds = torch.arange(b0, min(g.n_items, b0 + 32), dtype=torch.int32, device=DEV)
            ref = model.get_repr(smp.generate_blocks(seeds))
            assert torch.equal(a[b0:b0 + seeds.numel()], ref)


def test_train_cli_with_hit_rate(capsys):
    from recommender_amd.pinsage.train import main

    main(["--steps", "3", "--eval_every", "2"])
    out = capsys.readouterr().out
    assert "hit_rate" in out
