"""GPU tests of the row-sharded slab: world 1 equals the unsharded DLRM step bit for bit, and
world 2 (two processes sharing the one GPU, exchange over gloo staged through the host) matches
the sharded-step oracle bit for bit."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("D", [32, 128])
def test_world1_sharded_dlrm_equals_unsharded(D):
    """D = 128 with the factored path forced on takes the fused interaction + top chain with the
    rank-one backward, over the sharded exchange's unique rows."""
    from recommender_amd.ctr.layers import MLP
    from recommender_amd.ctr.model import DLRM
    from recommender_amd.ctr.train import TrainStep
    from recommender_amd.sharded import Comm, ShardedSlabEmbedding
    from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

    old_min = MLP.factored_min_batch
    MLP.factored_min_batch = 0 if D == 128 else old_min
    try:
        _sharded_vs_unsharded(D, criteo_cardinalities, criteo_batch, DLRM, TrainStep, Comm,
                              ShardedSlabEmbedding)
    finally:
        MLP.factored_min_batch = old_min


def _sharded_vs_unsharded(D, criteo_cardinalities, criteo_batch, DLRM, TrainStep, Comm,
                          ShardedSlabEmbedding):
    cards = criteo_cardinalities(200_000, 26)
    g = torch.Generator(device=DEV)
    g.manual_seed(1)
    m1 = DLRM([64, D], [64, 1], D, sum(cards), 26, 13, device=DEV, slot_cardinalities=cards, generator=g)
    emb = ShardedSlabEmbedding(cards, D, Comm(), device=DEV, full_weight=m1.embedding_layer.weight)
    m2 = DLRM([64, D], [64, 1], D, sum(cards), 26, 13, device=DEV, embedding_layer=emb)
    sd = {k: v for k, v in m1.state_dict().items() if not k.startswith("embedding_layer")}
    m2.load_state_dict(sd, strict=False)
    s1, s2 = TrainStep(m1, "sgd", lr=0.05), TrainStep(m2, "sgd", lr=0.05)
    r = np.random.default_rng(0)
    for _ in range(2):
        cat, dn, lb = criteo_batch(r, 1024, cards)
        b = tuple(torch.from_numpy(x).to(DEV) for x in (cat, dn, lb))
        l1, l2 = s1(b), s2(b)
        assert float(l1) == float(l2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(emb.full_weight().cpu().numpy(), m1.embedding_layer.weight.cpu().numpy())


def _worker(rank, world, port, q, opt="sgd", even=False):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import embedding as OE
        from oracle import sharded as OS
        from recommender_amd.optim import SparseAdam, SparseSGD
        from recommender_amd.sharded import Comm, ShardedSlabEmbedding

        # even=True: every slot has an even cardinality and offset and step 2's ids are all
        # even, so its global rows are even and rank 1 (owner of the odd rows) receives none
        card = [6, 2, 700, 3000, 40] if even else [5, 1, 700, 3000, 40]
        D, B = 16, 900
        V = sum(card)
        so = np.concatenate([[0], np.cumsum(card)]).astype(np.int64)
        table = np.random.default_rng(9).standard_normal((V, D)).astype(np.float32)
        emb = ShardedSlabEmbedding(card, D, Comm(), device=DEV, full_weight=torch.from_numpy(table))
        if opt == "sgd":
            sopt = SparseSGD([emb.shard], lr=0.05)
        else:
            sopt = SparseAdam([emb.shard], lr=1e-3, mode=opt)
        emb.set_optimizer(sopt)
        m = np.zeros((V, D), np.float32)
        v = np.zeros((V, D), np.float32)
        t_ref = table
        for step in range(2 if opt != "sgd" else 1):
            per_ids, per_g = [], []
            for rr in range(world):
                rg = np.random.default_rng(100 + rr + 10 * step)
                ids = np.stack([np.minimum(rg.zipf(1.1, B) - 1, c - 1) for c in card], 1).astype(np.int64)
                if even and step == 1:
                    ids = ids - ids % 2
                per_ids.append(ids)
                per_g.append(rg.standard_normal((ids.size, D)).astype(np.float32))
            ids_t = torch.from_numpy(per_ids[rank]).to(DEV)
            out = emb(ids_t)
            np.testing.assert_array_equal(out.detach().cpu().numpy(),
                                          OE.embedding_lookup(t_ref, per_ids[rank], so))
            out.backward(torch.from_numpy(per_g[rank]).to(DEV).view(out.shape))
            emb.join()
            sopt.iterations += 1
            if opt == "sgd":
                t_ref = OS.sharded_sgd_step(t_ref, per_ids, per_g, 0.05, world, so)
            else:
                t_ref, m, v = OS.sharded_adam_step(t_ref, m, v, per_ids, per_g, world, step + 1,
                                                   opt, 1e-3, so)
            prev = full if step else table
            full = emb.full_weight().cpu().numpy()
            np.testing.assert_array_equal(full, t_ref)
        if even and opt == "keras":
            # step 2 hands rank 1 no row, yet its rows with step-1 momentum still move
            moved = (full[1::2] != prev[1::2]).any(1)
            assert (m[1::2] != 0).any(1).sum() > 0 and moved.sum() == (m[1::2] != 0).any(1).sum()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("opt,even", [("sgd", False), ("lazy", False), ("keras", False),
                                      ("keras", True)])
def test_world2_sharded_embedding_matches_oracle(opt, even):
    """Two ranks on the one GPU (gloo staged exchange): lookups, the owner-side SGD / lazy Adam /
    Keras Adam apply (grads x 1/W) bit-exact vs oracle/sharded.py; `even`: rank 1 owns no row of
    the batch and its shard still takes Keras Adam's dense update."""
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() % 500) + 17 * ["sgd", "lazy", "keras"].index(opt) + (3 if even else 0)
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, opt, even)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(60)
    assert all(v == "ok" for v in res.values()), res
