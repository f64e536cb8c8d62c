"""The RCCL path on a one-GPU box: a world-1 `nccl` process group with Comm(force_collectives=True),
so every all-to-all / all-reduce of the row-sharded step and of PinSage's captured step goes
through ProcessGroupNCCL (RCCL) instead of the world-1 copy short-circuit — its streams, work
handles and the cross-stream order of the exchange run as they will at world 8.

(a) The production fused DLRM step on a ShardedSlabEmbedding (reference ctr/train.py:71-97,
    ctr/model.py:45-57) over RCCL, with the exchange prefetched a step ahead (rows ahead + the
    late round run at world 1 when collectives are forced), equals the one-GPU step bit for bit:
    loss, slab and every MLP parameter, six steps — the fifth after a load_state_dict between its
    prefetch and its exchange (rows ahead invalidated: it re-sends its whole block).
(b) PinSage's sync-free step (pinsage/train/train.py:40-48) with its flat-gradient all-reduce
    captured into a HIP graph on the RCCL group and replayed equals the same graph without the
    collective, bit for bit. At world 1 RCCL records no node for the all-reduce
    (tools/probe_rccl_capture.py): this checks the capture path around it, not a captured
    reduction."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _dlrm_part():
    from recommender_amd.ctr.layers import MLP
    from recommender_amd.ctr.model import DLRM
    from recommender_amd.ctr.train import TrainStep
    from recommender_amd.sharded import Comm, ShardedSlabEmbedding
    from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

    MLP.factored_min_batch = 0
    S, D, B = 26, 128, 2048
    cards = criteo_cardinalities(200_000, S)
    V = sum(cards)
    g = torch.Generator(device=DEV)
    g.manual_seed(1)
    m1 = DLRM([128, 64, D], [128, 64, 1], D, V, S, 13, device=DEV, slot_cardinalities=cards,
              generator=g)
    comm = Comm(force_collectives=True)
    assert comm.world == 1 and comm.collective and not comm.staged
    emb = ShardedSlabEmbedding(cards, D, comm, device=DEV, full_weight=m1.embedding_layer.weight)
    m2 = DLRM([128, 64, D], [128, 64, 1], D, V, S, 13, device=DEV, embedding_layer=emb)
    sd = {k: v for k, v in m1.state_dict().items() if not k.startswith("embedding_layer")}
    m2.load_state_dict(sd, strict=False)
    s1, s2 = TrainStep(m1, "sgd", lr=0.05), TrainStep(m2, "sgd", lr=0.05, comm=comm)
    with pytest.raises(RuntimeError, match="cannot be captured"):
        s2.capture_sequence([])
    r = np.random.default_rng(0)
    batches = [tuple(torch.from_numpy(x).to(DEV) for x in criteo_batch(r, B, cards))
               for _ in range(6)]
    for k, b in enumerate(batches):
        assert s2.fused_step_ready(b)
        if k == 4:
            # a write to the shard after this step's early rows were gathered (during step 3)
            # and before its exchange: they are stale, so it re-sends its whole block ('full')
            emb.join()
            torch.cuda.synchronize()
            new_w = m1.embedding_layer.weight * 0.5 + 0.01
            m1.embedding_layer.weight.copy_(new_w)
            sd2 = emb.state_dict()
            sd2["shard.weight"] = new_w.clone()
            emb.load_state_dict(sd2)
        if k + 1 < len(batches):
            s2.prefetch(batches[k + 1])
        l1, l2 = float(s1(b)), float(s2(b))
        assert l1 == l2, (k, l1, l2)
    emb.join()
    torch.cuda.synchronize()
    assert emb.rows_ahead_modes == {"fresh": 1, "late": 4, "full": 1}, emb.rows_ahead_modes
    assert torch.equal(emb.full_weight(), m1.embedding_layer.weight), "slab"
    for a, b_ in zip(list(m1.bottom_mlp.parameters()) + list(m1.top_mlp.parameters()),
                     list(m2.bottom_mlp.parameters()) + list(m2.top_mlp.parameters())):
        assert torch.equal(a, b_), "MLP parameter"


def _pinsage_part():
    from recommender_amd.pinsage import PinSageModel, PinSageSampler
    from recommender_amd.pinsage.train import PinSageStep
    from recommender_amd.sharded import Comm
    from tests.test_pinsage_gpu import _pinsage_params, small_graph

    B = 96
    g, _ = small_graph(7, n_users=200, n_items=300, n_edges=3000, dead_items=25)
    res = []
    for comm in (Comm(force_collectives=True), None):
        model = PinSageModel(g, g.itype, 2, 8, 32, 16,
                             generator=torch.Generator(device=DEV).manual_seed(1))
        smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
        step = PinSageStep(model, lr=1e-2, comm=comm)
        losses, replay = [], None
        for it in range(4):
            batch = smp.sample_static(*smp.sample_pairs_static(B, 4, it))
            if it == 0:
                losses.append(float(step.static_step(*batch)))
                continue
            if replay is None:
                replay = step.capture(batch)
            losses.append(float(replay()))
        torch.cuda.synchronize()
        res.append((losses, _pinsage_params(model)))
    (la, pa), (lb, pb) = res
    assert la == lb, (la, lb)
    for x, y in zip(pa, pb):
        np.testing.assert_array_equal(x, y)


def _worker(rank, world, port, q):
    import sys
    from datetime import timedelta

    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0),
                            timeout=timedelta(seconds=120))
    try:
        assert dist.get_backend() == "nccl"
        _dlrm_part()
        _pinsage_part()
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_rccl_world1_sharded_step_and_captured_allreduce():
    from tests.conftest import run_ranks

    res = run_ranks(_worker, 1, (29950 + os.getpid() % 400,))
    assert res == {0: "ok"}, res
