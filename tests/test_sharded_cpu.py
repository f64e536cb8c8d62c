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
