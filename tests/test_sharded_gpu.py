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


def _fused_dlrm_worldn_worker(rank, world, port, spill, prefetch, q):
    """The production fused DLRM step over a row-sharded slab, `world` ranks on the one GPU
    (gloo): every check is against the oracle on the GLOBAL batch (all ranks' examples). Four
    steps; `spill`: the third batch has uniform ids (many more unique rows than the capacity the
    first exchanged, Zipf, batch calibrated), so its exchange takes the spill round. `prefetch`:
    each step's exchange is queued during the step before (TrainStep.prefetch), so its rows are
    gathered a step early and only the rows the step before updates (its capacity block and
    spill rows) are sent again after that step's apply: every step but the first takes that late
    round."""
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import sharded as OS
        from oracle.check_dlrm import _check_chain, _check_sgd, _grads, _layers, dense_half_tolerances
        from oracle.ctr import DLRMState, dlrm_sgd_step
        from recommender_amd.ctr.layers import MLP
        from recommender_amd.ctr.model import DLRM
        from recommender_amd.ctr.train import TrainStep
        from recommender_amd.sharded import Comm, ShardedSlabEmbedding
        from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

        from recommender_amd import _lib as L
        from recommender_amd.functional import TRAIN_SUMS_ATOP, _train_ws
        from recommender_amd.nn import _composed_forward_hip, cached_vec_chain_compose

        MLP.factored_min_batch = 0
        # 1 024 examples per rank at every world size (global 1 024·W)
        S, D, B, lr = 26, 128, 1024, 0.05
        cards = criteo_cardinalities(200_000, S)
        V = sum(cards)
        so = np.concatenate([[0], np.cumsum(cards)]).astype(np.int64)
        table = np.random.default_rng(9).uniform(-0.05, 0.05, (V, D)).astype(np.float32)
        comm = Comm()
        emb = ShardedSlabEmbedding(cards, D, comm, device=DEV, full_weight=torch.from_numpy(table))
        g = torch.Generator(device=DEV)
        g.manual_seed(3)  # the same MLP init on every rank
        model = DLRM([128, 64, D], [128, 64, 1], D, V, S, 13, device=DEV, generator=g,
                     embedding_layer=emb)
        step = TrainStep(model, "sgd", lr=lr, comm=comm)
        steps = [[criteo_batch(np.random.default_rng(40 + 10 * k + r), B, cards) for r in range(world)]
                 for k in range(4)]
        if spill:
            for r in range(world):
                c2 = steps[2][r][0]
                for j, c in enumerate(cards):
                    c2[:, j] = np.random.default_rng(70 + r + 100 * j).integers(0, c, B)
        top0, bot0 = _layers(model.top_mlp), _layers(model.bottom_mlp)
        cap = {}
        bx = emb.backward_exchange

        def spy(grad_rows, global_grads=False, row_scale=None):
            g_ = grad_rows.detach().clone()
            if row_scale is not None:  # unit rows + G[b]: the rows the dedup forms (fmul_rn)
                g_ = row_scale.repeat_interleave(S)[:, None] * g_
            cap["g"] = g_
            assert global_grads
            return bx(grad_rows, global_grads=global_grads, row_scale=row_scale)

        emb.backward_exchange = spy
        M = TRAIN_SUMS_ATOP + 2 + 13 * D + D
        ar = comm.all_reduce_

        def ar_spy(t, op=None):  # the batch sums before and after their all-reduce
            if op is None and t.numel() == M:
                cap["pre"] = t.detach().clone()
                ar(t, op)
                cap["post"] = t.detach().clone()
                return None
            return ar(t, op)

        comm.all_reduce_ = ar_spy
        want = table
        dev_batches = [tuple(torch.from_numpy(x).to(DEV) for x in per[rank]) for per in steps]
        for k, per in enumerate(steps):
            batch = dev_batches[k]
            assert step.fused_step_ready((batch[0], None, None))
            if k == 0:
                # the one-GPU train kernel on this rank's examples over the whole slab, with the
                # global loss scale 1/(B·W): what the sharded step must reproduce bit for bit
                # before its all-reduce (the exchange only re-indexes the same rows)
                with torch.no_grad():
                    bl, tl = list(model.bottom_mlp.mlp), list(model.top_mlp.mlp)
                    xin = batch[1].reshape(-1, 13).float().contiguous()
                    h, _ = _composed_forward_hip(xin, bl, None)
                    q_, c_ = cached_vec_chain_compose(tl, model.compact_rows, model.compact_rows.numel())
                wfull = torch.from_numpy(table).to(DEV)
                offs_t = torch.from_numpy(so).to(DEV)
                ids0 = batch[0].contiguous()
                y0 = torch.empty(B, device=DEV)
                u0 = torch.empty(B * S, D, device=DEV)
                g0 = torch.empty(B, device=DEV)
                sums0 = torch.empty(M, device=DEV)
                ws0 = _train_ws(B, torch.device(DEV)).clone()
                err0 = torch.zeros(1, dtype=torch.int32, device=DEV)
                lab0 = batch[2].reshape(-1).float().contiguous()
                L.call("rs_dlrm_train_step_fwd_unit", L.ptr(wfull), V, D, L.ptr(ids0),
                       L.id_dtype_code(ids0), S, L.ptr(offs_t), L.ptr(h), L.ptr(xin), 13,
                       L.ptr(lab0), B, L.ptr(q_), L.ptr(c_),
                       1e-7, 1.0 / (B * world), L.ptr(y0), L.ptr(u0), L.ptr(g0), L.ptr(sums0),
                       L.ptr(ws0), ws0.numel(), L.ptr(err0), L.stream_ptr(torch.device(DEV)))
                torch.cuda.synchronize()
                del wfull
            if prefetch and k + 1 < len(steps):
                step.prefetch(dev_batches[k + 1])
            loss = float(step(batch))
            emb.join()
            torch.cuda.synchronize()
            # all ranks' gradient rows, for the sharded-apply oracle
            gr = [torch.empty_like(cap["g"].cpu()) for _ in range(world)]
            dist.all_gather(gr, cap["g"].cpu())
            want = OS.sharded_sgd_step(want, [p[0] for p in per], [x.numpy() for x in gr], lr,
                                       world, so, global_grads=True)
            full = emb.full_weight().cpu().numpy()
            np.testing.assert_array_equal(full, want)
            if k == 0:
                assert (full != table).any(1).sum() > 1000
                # (1) the sharded rank's kernel == the one-GPU kernel on its examples, bit for bit
                assert int(err0.item()) == 0
                assert torch.equal(step.last_pred, y0), "predictions differ from the one-GPU kernel"
                assert torch.equal(cap["pre"], sums0), "batch sums differ from the one-GPU kernel"
                assert torch.equal(cap["g"], g0.repeat_interleave(S)[:, None] * u0), "gradient rows"
                # (2) the all-reduce: the fp32 sum of every rank's partial row within (W-1)·u
                parts = [torch.empty_like(cap["pre"]).cpu() for _ in range(world)]
                dist.all_gather(parts, cap["pre"].cpu())
                P = torch.stack(parts).double()
                ar_err = (cap["post"].cpu().double() - P.sum(0)).abs()
                assert (ar_err <= (world - 1) * 2.0 ** -24 * P.abs().sum(0) + 1e-45).all(), "all-reduce"
                # the dense half and the loss against the oracle step on the global batch
                st = DLRMState(table.copy(), so, [(k_.copy(), b_.copy()) for k_, b_ in bot0],
                               [(k_.copy(), b_.copy()) for k_, b_ in top0])
                det = {}
                gcat = np.concatenate([p[0] for p in per])
                gdn = np.concatenate([p[1] for p in per])
                glb = np.concatenate([p[2] for p in per])
                ref_loss = dlrm_sgd_step(st, gcat, gdn, glb, lr, det)
                assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss), (loss, ref_loss)
                top_tol, bot_tol = dense_half_tolerances(det, B * world, world=world)
                if rank == 0:  # the round-5 bound (top inputs at their value) for the record
                    d5 = {k_: v_ for k_, v_ in det.items() if k_ != "top_in_bound"}
                    t5, _ = dense_half_tolerances(d5, B * world)
                    r5 = max(float((np.abs(g_.astype(np.float64) - r_) / (t_ + 1e-38)).max())
                             for (gk, gb), (rk, rb), (tk, tb) in
                             zip(_grads(model.top_mlp), det["top_grads"], t5)
                             for g_, r_, t_ in ((gk, rk, tk), (gb, rb, tb)))
                wt = _check_chain("top MLP", _grads(model.top_mlp), det["top_grads"], top_tol)
                wb = _check_chain("bottom MLP", _grads(model.bottom_mlp), det["bottom_grads"], bot_tol)
                if rank == 0:
                    print(f"[world {world}] top err/tol {wt:.3g} (round-5 bound {r5:.3g}), "
                          f"bottom {wb:.3g}", flush=True)
                _check_sgd("top MLP", top0, _layers(model.top_mlp), _grads(model.top_mlp), lr)
                _check_sgd("bottom MLP", bot0, _layers(model.bottom_mlp), _grads(model.bottom_mlp),
                           lr)
                # this rank's gradient rows against the oracle's rows of its examples
                dx = det["dx"].reshape(world, B * S, D)[rank]
                dxb = det["dx_bound"].reshape(world, B * S, D)[rank]
                err = np.abs(cap["g"].cpu().numpy().astype(np.float64) - dx)
                assert (err <= 1e-5 * dxb + 1e-38).all(), "gradient rows"
                assert emb.spill_rounds == 0
        if spill:
            assert emb.spill_rounds == 1, emb.spill_rounds
        modes = emb.rows_ahead_modes
        want_modes = ({"fresh": 1, "late": 3, "full": 0} if prefetch else
                      {"fresh": 4, "late": 0, "full": 0})
        assert modes == want_modes, modes
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,spill,prefetch", [(2, False, False), (2, True, True),
                                                  (2, False, True), (3, True, False),
                                                  (3, False, True), (4, False, False),
                                                  (4, True, True), (8, False, True),
                                                  (8, True, False)])
def test_worldn_fused_dlrm_step_matches_oracle(world, spill, prefetch):
    """TrainStep's fused DLRM step on a row-sharded slab at world 2 / 3 / 4 / 8 (gloo, all ranks
    on the one GPU; 1 024 examples per rank; W = 8 is the production width): the train kernel
    reads the exchanged unique rows with dL/dl_b = 1/(B·W); the batch sums are all-reduced (the
    dense half of the global step); the owners apply the gradient rows. First step: each rank's
    predictions, gradient rows and pre-all-reduce batch sums equal the one-GPU train kernel's on
    that rank's examples bit for bit, and the all-reduced sums are within (W-1)·u of the exact
    sum of the ranks' partials — so the sharded dense half has no error source of its own. Four steps, slab bit-exact vs oracle/sharded.py fed with every rank's kernel rows after
    each; loss, the twelve MLP gradients (per-element bounds) and the SGD apply vs the oracle step
    on the global batch. `spill`: the third step's batch overflows the calibrated capacity and
    is exchanged with the spill round — still bit-exact, on every rank. `prefetch`: rows a step
    ahead (each step's capacity block gathered during the step before, the rows that step
    updated re-sent after its apply), the same bits."""
    from tests.conftest import run_ranks

    port = 29300 + (os.getpid() % 400) + 13 * world + (5 if spill else 0) + (7 if prefetch else 0)
    res = run_ranks(_fused_dlrm_worldn_worker, world, (port, spill, prefetch))
    assert all(v == "ok" for v in res.values()), res


def _prefetch_world2_worker(rank, world, port, q):
    """The row-sharded fused DLRM step with the exchange's first half queued a step ahead
    (TrainStep.prefetch -> ShardedSlabEmbedding.prefetch) equals the same steps without it, bit for
    bit (slab and MLP), over 3 steps; a prefetched batch whose ids change in place is exchanged
    again."""
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from recommender_amd.ctr.layers import MLP
        from recommender_amd.ctr.model import DLRM
        from recommender_amd.ctr.train import TrainStep
        from recommender_amd.sharded import Comm, ShardedSlabEmbedding
        from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

        MLP.factored_min_batch = 0
        S, D, B = 26, 128, 512
        cards = criteo_cardinalities(100_000, S)
        V = sum(cards)
        table = torch.from_numpy(np.random.default_rng(9).uniform(-0.05, 0.05, (V, D)).astype(np.float32))
        rng = np.random.default_rng(50 + rank)
        batches = [tuple(torch.from_numpy(x).to(DEV) for x in criteo_batch(rng, B, cards)) for _ in range(3)]
        repl = torch.from_numpy(criteo_batch(rng, B, cards)[0]).to(DEV)
        comm = Comm()
        res = []
        for pre in (False, True):
            emb = ShardedSlabEmbedding(cards, D, comm, device=DEV, full_weight=table)
            g = torch.Generator(device=DEV)
            g.manual_seed(3)
            model = DLRM([128, 64, D], [128, 64, 1], D, V, S, 13, device=DEV, generator=g,
                         embedding_layer=emb)
            step = TrainStep(model, "sgd", lr=0.05, comm=comm)
            bs = [tuple(t.clone() for t in b) for b in batches]
            for i, b in enumerate(bs):
                if pre and i + 1 < len(bs):
                    step.prefetch(bs[i + 1])
                if i == 2:  # prefetched during step 1, then changed in place
                    b[0].copy_(repl)
                    if pre:
                        # the prefetched exchange no longer matches: loud, on every rank (the
                        # collectives stay paired), then the step exchanges afresh
                        try:
                            step(b)
                        except RuntimeError as e:
                            assert "prefetched" in str(e)
                        else:
                            raise AssertionError("a changed prefetched batch must raise")
                step(b)
            emb.join()
            torch.cuda.synchronize()
            assert not emb._prefetched
            res.append((emb.full_weight().cpu(), [p.detach().cpu() for p in model.parameters()]))
        (wa, pa), (wb, pb) = res
        assert torch.equal(wa, wb)
        for x, y in zip(pa, pb):
            assert torch.equal(x, y)
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_world2_prefetched_exchange_bit_identical():
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29800 + (os.getpid() % 500)
    ps = [ctx.Process(target=_prefetch_world2_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(60)
    assert all(v == "ok" for v in res.values()), res


def test_exchange_capacity_spill_round():
    """A batch with more unique rows for one owner than the exchange capacity takes the spill
    round (the excess rows in a second pair of equal-split all-to-alls) instead of failing: the
    lookup equals the slab's rows, and three SGD steps on a capacity-64 slab equal the same steps
    on a calibrated one, bit for bit."""
    from recommender_amd.optim import SparseSGD
    from recommender_amd.sharded import Comm, ShardedSlabEmbedding
    from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

    cards = criteo_cardinalities(100_000, 26)
    rng = np.random.default_rng(3)
    batches = [torch.from_numpy(criteo_batch(rng, 256, cards)[0]).to(DEV) for _ in range(3)]
    w0 = torch.from_numpy(np.random.default_rng(5).uniform(-0.05, 0.05, (sum(cards), 16))
                          .astype(np.float32))
    res = []
    for capacity in (64, None):
        emb = ShardedSlabEmbedding(cards, 16, Comm(), device=DEV, full_weight=w0, capacity=capacity)
        emb.set_optimizer(SparseSGD([emb.shard], lr=0.1))
        for ids in batches:
            out = emb(ids)
            torch.cuda.synchronize()
            full = emb.full_weight()
            rows = ids.long() + emb.slot_offsets[:-1][None, :]
            assert torch.equal(out.detach().reshape(-1, 16), full[rows.reshape(-1)])
            (out * 0.5).sum().backward()
            emb.join()
        torch.cuda.synchronize()
        res.append((emb.full_weight().cpu(), emb.spill_rounds))
    (wa, spills), (wb, none) = res
    assert spills == 3 and none == 0
    assert torch.equal(wa, wb)
