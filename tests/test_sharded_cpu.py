"""CPU tests of the multi-rank path: the Comm transport and the dense-gradient all-reduce of
TrainStep over a world-size-2 gloo group, and the sharded-step oracle against the unsharded one."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import embedding as OE
from oracle import sharded as OS


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from recommender_amd.sharded import Comm

        c = Comm()
        assert c.staged and c.world == world and c.rank == rank
        # variable-split all-to-all: rank r sends (d+1) values r*10+d to rank d
        send_counts = [d + 1 for d in range(world)]
        inp = torch.cat([torch.full((d + 1,), float(rank * 10 + d)) for d in range(world)])
        recv_counts = [rank + 1] * world
        out = torch.empty(sum(recv_counts))
        c.all_to_all(out, inp, recv_counts, send_counts)
        exp = torch.cat([torch.full((rank + 1,), float(s * 10 + rank)) for s in range(world)])
        assert torch.equal(out, exp)
        t = torch.full((5,), float(rank + 1))
        c.all_reduce_(t)
        assert torch.equal(t, torch.full((5,), float(sum(range(1, world + 1)))))
        # TrainStep's bucketed dense all-reduce (average over ranks)
        from recommender_amd.ctr.train import TrainStep

        class Fake:
            pass

        ts = TrainStep.__new__(TrainStep)
        ts.comm = c
        p1 = torch.nn.Parameter(torch.zeros(3, 2))
        p2 = torch.nn.Parameter(torch.zeros(4))
        p1.grad = torch.full((3, 2), float(rank))
        p2.grad = torch.full((4,), float(2 * rank))
        ts.dense = [p1, p2]
        ts._allreduce_dense()
        m = (world - 1) / 2
        assert torch.allclose(p1.grad, torch.full((3, 2), m)) and torch.allclose(p2.grad, torch.full((4,), 2 * m))
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_comm_and_dense_allreduce(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(30)
    assert all(v == "ok" for v in res.values()), res


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_sharded_oracle_matches_unsharded(world, rng):
    """Sharded SGD = unsharded SGD on the concatenated global batch up to fp32 rounding of
    the different reduction tree (and bit-exact at world 1)."""
    V, D = 3000, 8
    table = rng.standard_normal((V, D)).astype(np.float32)
    ids = [np.minimum(rng.zipf(1.2, 700) - 1, V - 1) for _ in range(world)]
    grads = [rng.standard_normal((700, D)).astype(np.float32) for _ in range(world)]
    got = OS.sharded_sgd_step(table, ids, grads, 0.1, world)
    all_ids = np.concatenate(ids)
    all_g = np.concatenate(grads) / np.float32(world)
    sr, sp, _ = OE.sort_ids(all_ids, V)
    ur, ug = OE.segment_sum_tiled(sr, sp, all_g.astype(np.float32), V)
    ref = OE.apply_sgd(table, ur, ug, np.float32(0.1))
    if world == 1:
        np.testing.assert_array_equal(got, ref)
    else:
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("mode", ["lazy", "keras"])
@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_adam_oracle_matches_unsharded(mode, world, rng):
    """Sharded lazy / Keras Adam = the unsharded apply on the concatenated batch (grads / W) up to
    fp32 rounding of the reduction tree; bit-exact at world 1."""
    V, D = 2000, 8
    table = rng.standard_normal((V, D)).astype(np.float32)
    m = (rng.standard_normal((V, D)) * 0.01).astype(np.float32)
    v = (rng.random((V, D)) * 0.01).astype(np.float32)
    ids = [np.minimum(rng.zipf(1.2, 500) - 1, V - 1) for _ in range(world)]
    grads = [rng.standard_normal((500, D)).astype(np.float32) for _ in range(world)]
    got = OS.sharded_adam_step(table, m, v, ids, grads, world, 3, mode)
    all_g = np.concatenate(grads) * np.float32(1.0 / world) if world > 1 else np.concatenate(grads)
    sr, sp, _ = OE.sort_ids(np.concatenate(ids), V)
    ur, ug = OE.segment_sum_tiled(sr, sp, all_g.astype(np.float32), V)
    c = OE.keras_adam_coefficients(3)
    fn = OE.apply_keras_adam if mode == "keras" else OE.apply_lazy_adam
    ref = fn(table, m, v, ur, ug, c)
    for a, b in zip(got, ref):
        if world == 1:
            np.testing.assert_array_equal(a, b)
        else:
            np.testing.assert_allclose(a, b, rtol=2e-5, atol=1e-6)


def test_sharded_keras_adam_moves_rows_of_an_untouched_shard(rng):
    """World 2 with every id on an even row: owner 1 receives no row, yet Keras Adam's dense half
    still decays its m / v and moves its rows (recommender_amd/sharded.py backward_exchange)."""
    V, D = 400, 4
    table = rng.standard_normal((V, D)).astype(np.float32)
    m = (rng.standard_normal((V, D)) * 0.01).astype(np.float32)
    v = (rng.random((V, D)) * 0.01).astype(np.float32)
    ids = [2 * rng.integers(0, V // 2, 50) for _ in range(2)]
    grads = [rng.standard_normal((50, D)).astype(np.float32) for _ in range(2)]
    t, m2, v2 = OS.sharded_adam_step(table, m, v, ids, grads, 2, 1, "keras")
    odd = np.arange(1, V, 2)
    assert np.all(t[odd] != table[odd]) and np.all(m2[odd] == m[odd] * np.float32(0.9))
    tl, _, _ = OS.sharded_adam_step(table, m, v, ids, grads, 2, 1, "lazy")
    np.testing.assert_array_equal(tl[odd], table[odd])
