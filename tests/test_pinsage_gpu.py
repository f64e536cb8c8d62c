"""GPU parity for PinSage.

Sampling / index work (Philox, metapath walks, item pairs, PinSAGE neighbours with leak-edge
removal, first-appearance unique, to_block + transpose, the whole sample_from_item_pairs) is
compared BIT-EXACT against oracle/pinsage.py on the same seeds. The float path (weighted
mean-pool, global Frobenius norm, the full PinSageModel forward + gradients) is compared with
a plain torch fp32 autograd restatement of pinsage/train/layers.py / model.py at rtol 2e-5.
Graphs carry dead ends on both sides (items without users, users without items)."""
import numpy as np
import pytest
import torch

from oracle import pinsage as O
from recommender_amd import _lib as L
from recommender_amd.pinsage import PinSageModel, PinSageSampler
from recommender_amd.pinsage.graph import HeteroGraph
from recommender_amd.pinsage.layers import frobenius_normalize, weighted_mean_agg
from recommender_amd.pinsage.model import oob_flag as model_oob_flag
from recommender_amd.pinsage.sampler import item_pairs
from recommender_amd.pinsage.train import PinSageStep
from tests.conftest import assert_close_rel, assert_close_f64

pytestmark = pytest.mark.gpu
DEV = "cuda"
RTOL = 2e-5


def small_graph(seed=0, n_users=60, n_items=90, n_edges=500, dead_items=7, dead_users=5):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, n_users - dead_users, n_edges)
    i = rng.integers(0, n_items - dead_items, n_edges)
    # power-law-ish: half of the edges on the 10 most popular items
    hot = rng.random(n_edges) < 0.5
    i[hot] = rng.integers(0, 10, int(hot.sum()))
    key = np.unique(u * n_items + i)
    u, i = key // n_items, key % n_items
    year = rng.integers(0, 12, n_items)
    genre = (rng.random((n_items, 6)) < 0.3).astype(np.int8)
    g = HeteroGraph(u, i, n_users, n_items, device=DEV, item_data={"year": year, "genre": genre})
    og = O.BipartiteGraph.from_edges(u, i, n_users, n_items)
    return g, og


def test_graph_csr_matches_oracle():
    g, og = small_graph()
    np.testing.assert_array_equal(g.i2u_indptr.cpu().numpy(), og.i2u_indptr)
    np.testing.assert_array_equal(g.i2u.cpu().numpy(), og.i2u)
    np.testing.assert_array_equal(g.u2i_indptr.cpu().numpy(), og.u2i_indptr)
    np.testing.assert_array_equal(g.u2i.cpu().numpy(), og.u2i)


def test_philox_known_answers_and_random(rng):
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, exp in kat:
        c = torch.tensor(np.array(ctr, np.uint32).view(np.int32), device=DEV)
        out = torch.empty(4, dtype=torch.int32, device=DEV)
        L.call("rs_philox4x32_10", L.ptr(c), 1, key[0], key[1], L.ptr(out), L.stream_ptr(DEV))
        assert tuple(out.cpu().numpy().view(np.uint32).tolist()) == exp
    ctr = rng.integers(0, 2**32, (1000, 4), dtype=np.uint64).astype(np.uint32)
    c = torch.tensor(ctr.view(np.int32), device=DEV)
    out = torch.empty(4000, dtype=torch.int32, device=DEV)
    L.call("rs_philox4x32_10", L.ptr(c), 1000, 0x12345678, 0x9abcdef0, L.ptr(out),
           L.stream_ptr(DEV))
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32).reshape(1000, 4),
                                  O.philox4x32_10(ctr, 0x12345678, 0x9abcdef0))


@pytest.mark.parametrize("num_walks,T,p,layer", [(4, 2, 0.0, 0), (5, 1, 0.0, 1), (3, 3, 0.3, 2)])
def test_metapath_walk_bit_exact(num_walks, T, p, layer):
    g, og = small_graph(1)
    seeds = np.arange(g.n_items, dtype=np.int32)
    s = torch.tensor(seeds, device=DEV)
    tr = torch.empty(seeds.size * num_walks, 2 * T + 1, dtype=torch.int32, device=DEV)
    seed = 0x1234_5678_9ABC
    L.call("rs_metapath_walk", *(L.ptr(t) for t in g.csr_args()), L.ptr(s), seeds.size,
           num_walks, T, p, seed, 7, layer, L.ptr(tr), L.stream_ptr(DEV))
    ref = O.metapath_walk(og, seeds, num_walks, T, p, seed, 7, layer)
    np.testing.assert_array_equal(tr.cpu().numpy(), ref)
    assert (ref[:, 1:] == -1).any()  # dead ends exercised
    if p > 0:
        # early stops exercised: a live node followed by -1 on a node that has neighbours
        assert ((ref[:, 1:-1] >= 0) & (ref[:, 2:] == -1)).any()


@pytest.mark.parametrize("batch,base,step", [(32, 0, 0), (1000, 4096, 3), (1, 7, 11)])
def test_item_pairs_bit_exact(batch, base, step):
    g, og = small_graph(2)
    h, p, n = item_pairs(g, batch, 4, step, base)
    rh, rp, rn = O.item_pairs(og, base, batch, 4, step)
    for a, b in ((h, rh), (p, rp), (n, rn)):
        np.testing.assert_array_equal(a.cpu().numpy(), b)
    if batch >= 1000:
        assert rh.size < batch  # some heads dead-ended and were masked


@pytest.mark.parametrize("num_walks,T,k,p", [(4, 2, 3, 0.0), (64, 2, 10, 0.0), (7, 3, 4, 0.2),
                                             (1, 1, 1, 0.0)])
def test_neighbors_bit_exact(num_walks, T, k, p):
    g, og = small_graph(3)
    smp = PinSageSampler(g, g.itype, g.utype, 2, T, num_walks, p, k, seed=99)
    seeds = np.arange(g.n_items, dtype=np.int32)
    nbr, cnt = smp.neighbors(torch.tensor(seeds, device=DEV), layer=1, step=5)
    rn, rc = O.pinsage_neighbors(og, seeds, num_walks, T, p, k, 99, 5, 1)
    np.testing.assert_array_equal(nbr.cpu().numpy(), rn)
    np.testing.assert_array_equal(cnt.cpu().numpy(), rc)


def test_neighbors_exclusion_bit_exact(rng):
    g, og = small_graph(4)
    smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 8, 0.0, 5, seed=3)
    seeds = np.arange(g.n_items, dtype=np.int32)
    # exclude about half of the edges the unfiltered sampler would emit
    rn, _ = O.pinsage_neighbors(og, seeds, 8, 2, 0.0, 5, 3, 0, 0)
    s_idx, r_idx = np.nonzero(rn >= 0)
    pick = rng.random(s_idx.size) < 0.5
    src = rn[s_idx[pick], r_idx[pick]].astype(np.int32)
    dst = seeds[s_idx[pick]]
    heads = torch.tensor(src, device=DEV)
    tails = torch.tensor(dst, device=DEV)
    excl = smp._exclusion(heads, tails, tails)
    nbr, cnt = smp.neighbors(torch.tensor(seeds, device=DEV), layer=0, excl=excl, step=0)
    ex = set(zip(src.tolist(), dst.tolist()))
    en, ec = O.pinsage_neighbors(og, seeds, 8, 2, 0.0, 5, 3, 0, 0, exclude=ex)
    np.testing.assert_array_equal(nbr.cpu().numpy(), en)
    np.testing.assert_array_equal(cnt.cpu().numpy(), ec)
    assert (en == -1).sum() > (rn == -1).sum()


def test_unique_first_bit_exact(rng):
    g, _ = small_graph()
    smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3)
    for n in (1, 17, 5000):
        ids = rng.integers(-1, 90, n).astype(np.int32)
        uniq, local, nu = smp.unique_first(torch.tensor(ids, device=DEV), 90)
        ru, rl = O.unique_first(ids)
        assert int(nu.item()) == ru.size
        np.testing.assert_array_equal(uniq[: ru.size].cpu().numpy(), ru)
        np.testing.assert_array_equal(local.cpu().numpy(), rl)
    # out-of-range id: flagged, treated as absent
    smp.err_flag.zero_()
    uniq, local, nu = smp.unique_first(torch.tensor([3, 200, 3], dtype=torch.int32, device=DEV), 90)
    assert int(nu.item()) == 1 and local.cpu().tolist() == [0, -1, 0]
    assert int(smp.err_flag.item()) != 0


def check_block(b, rb):
    E = int(b.n_edges.item())
    assert b.n_dst == rb.n_dst and b.n_src == rb.n_src and E == rb.edge_src.size
    np.testing.assert_array_equal(b.src_nodes.cpu().numpy(), rb.src_nodes)
    np.testing.assert_array_equal(b.indptr.cpu().numpy(), rb.indptr)
    np.testing.assert_array_equal(b.edge_src[:E].cpu().numpy(), rb.edge_src)
    np.testing.assert_array_equal(b.edge_dst[:E].cpu().numpy(), rb.edge_dst)
    np.testing.assert_array_equal(b.edge_w[:E].cpu().numpy(), rb.edge_w)
    np.testing.assert_array_equal(b.t_indptr.cpu().numpy(), rb.t_indptr)
    np.testing.assert_array_equal(b.t_edge[:E].cpu().numpy(), rb.t_edge)


def test_to_block_bit_exact(rng):
    g, _ = small_graph()
    smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3)
    dst = rng.choice(90, 40, replace=False).astype(np.int32)
    nbr = rng.integers(-1, 90, (40, 3)).astype(np.int32)
    cnt = np.where(nbr >= 0, rng.integers(1, 9, (40, 3)), 0).astype(np.int32)
    b = smp.to_block(torch.tensor(dst, device=DEV), torch.tensor(nbr, device=DEV),
                     torch.tensor(cnt, device=DEV))
    check_block(b, O.to_block(dst, nbr, cnt))


@pytest.mark.parametrize("batch", [32, 700])
def test_sample_from_item_pairs_bit_exact(batch):
    g, og = small_graph(5)
    smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
    h, p, n = item_pairs(g, batch, 4, 0)
    pos_g, neg_g, blocks = smp.sample_from_item_pairs(h, p, n)
    seeds, pe, ne, rblocks = O.sample_from_item_pairs(og, h.cpu().numpy(), p.cpu().numpy(),
                                                      n.cpu().numpy(), 2, 4, 2, 0.0, 3, 4, 0)
    np.testing.assert_array_equal(pos_g.nodes.cpu().numpy(), seeds)
    np.testing.assert_array_equal(pos_g.src.cpu().numpy(), pe[0])
    np.testing.assert_array_equal(pos_g.dst.cpu().numpy(), pe[1])
    np.testing.assert_array_equal(neg_g.dst.cpu().numpy(), ne[1])
    assert len(blocks) == 2
    for b, rb in zip(blocks, rblocks):
        check_block(b, rb)
    assert smp.step == 1


# ---------------------------------------------------------------- float path vs torch fp32
def torch_agg(u, b):
    E = int(b.n_edges.item())
    src = b.edge_src[:E].long()
    dst = b.edge_dst[:E].long()
    w = b.edge_w[:E].to(u.dtype)
    vs = torch.zeros(b.n_dst, u.shape[1], device=u.device, dtype=u.dtype).index_add(
        0, dst, u[src] * w[:, None])
    ws = torch.zeros(b.n_dst, device=u.device, dtype=u.dtype).index_add(0, dst, w)
    return vs / torch.clamp(ws, min=1)[:, None]


def random_block(rng, n_dst=300, n_extra=500, k=3):
    g, _ = small_graph()
    smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, k)
    n_nodes = n_dst + n_extra
    dst = np.arange(n_dst, dtype=np.int32)
    nbr = rng.integers(-1, n_nodes, (n_dst, k)).astype(np.int32)
    nbr[:5] = -1  # dsts without in-edges (ws clipped to 1)
    cnt = np.where(nbr >= 0, rng.integers(1, 9, (n_dst, k)), 0).astype(np.int32)
    smp.g.n_items = n_nodes  # id space for unique_first only
    return smp.to_block(torch.tensor(dst, device=DEV), torch.tensor(nbr, device=DEV),
                        torch.tensor(cnt, device=DEV))


@pytest.mark.parametrize("H", [32, 5, 70])
def test_weighted_mean_agg_fwd_bwd(rng, H):
    b = random_block(rng)
    u = torch.randn(b.n_src, H, device=DEV, requires_grad=True)
    g = torch.randn(b.n_dst, H, device=DEV)
    out = weighted_mean_agg(u, b)
    out.backward(g)
    u2 = u.detach().clone().requires_grad_(True)
    ref = torch_agg(u2, b)
    ref.backward(g)
    assert_close_rel(out.detach().cpu(), ref.detach().cpu(), RTOL, msg="agg fwd")
    # sums of signed terms: judge against the term magnitude (index_add order differs)
    assert_close_rel(u.grad.cpu(), u2.grad.cpu(), RTOL, scale=float(u2.grad.abs().max()) * 1e-2,
                     msg="agg bwd")


@pytest.mark.parametrize("shape", [(1, 1), (300, 16), (5000, 16)])
def test_frobenius_normalize(shape):
    x = torch.randn(*shape, device=DEV).abs().requires_grad_(True)
    g = torch.randn(*shape, device=DEV)
    y = frobenius_normalize(x)
    y.backward(g)
    x2 = x.detach().clone().requires_grad_(True)
    y2 = x2 / torch.norm(x2)
    y2.backward(g)
    assert_close_rel(y.detach().cpu(), y2.detach().cpu(), RTOL, msg="frob fwd")
    # the gradient's natural size is |dy| / ||x||; a 1x1 block's exact gradient is 0 (torch
    # returns rounding noise there), so the floor is taken from that size
    nat = float(g.abs().max()) / float(x2.detach().norm())
    assert_close_rel(x.grad.cpu(), x2.grad.cpu(), RTOL, scale=nat * 1e-2, msg="frob bwd")


def torch_reference_repr(model, blocks, dtype=torch.float32):
    """pinsage/train/layers.py / model.py restated in plain torch (autograd; float64: the
    accuracy reference, float32: a sample of another fp32 evaluation's rounding)."""
    fp = model.feature_projector
    P = {}

    def leaf(name, t):
        P[name] = t.detach().to(dtype).clone().requires_grad_(True)
        return P[name]

    ids = blocks[0].src_nodes.long()
    ye = leaf("year", fp.year_embedding.weight)[fp.year[ids].long()]
    ge = leaf("genre", fp.genre_embedding.weight)[fp.genre[ids].long()].mean(1)
    ie = leaf("id", fp.id_embedding.weight)[fp.item_id[ids].long()]
    h = torch.cat([ye, ge, ie], -1)
    for li, (conv, b) in enumerate(zip(model.sagenet.convolves, blocks)):
        h_dst = h[: b.n_dst]
        u = torch.relu(h @ leaf(f"c{li}k1", conv.fc_1.kernel) + leaf(f"c{li}b1", conv.fc_1.bias))
        nv = torch_agg(u, b)
        new = torch.relu(torch.cat([nv, h_dst], -1) @ leaf(f"c{li}k2", conv.fc_2.kernel)
                         + leaf(f"c{li}b2", conv.fc_2.bias))
        h = new / torch.norm(new)
    s = model.sagenet
    h = torch.relu(h @ leaf("k1", s.fc_1.kernel) + leaf("b1", s.fc_1.bias))
    return h @ leaf("k2", s.fc_2.kernel) + leaf("b2", s.fc_2.bias), P


def test_pinsage_model_forward_backward():
    g, og = small_graph(6, n_users=200, n_items=300, n_edges=3000)
    gen = torch.Generator(device=DEV).manual_seed(0)
    model = PinSageModel(g, g.itype, 2, 8, 32, 16, generator=gen)
    smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
    h, p, n = item_pairs(g, 128, 4, 0)
    pos_g, neg_g, blocks = smp.sample_from_item_pairs(h, p, n)
    from recommender_amd.optim import densify_grad
    from recommender_amd.pinsage.model import margin_loss, item2item_scorer

    def run():
        for prm in model.parameters():
            prm.grad = None
        pos, neg = model(pos_g, neg_g, blocks)
        loss = margin_loss(pos, neg)
        loss.backward()
        grads = {n: prm.grad.clone() for n, prm in model.named_parameters() if prm.grad is not None}
        for t, name in zip(model.tables(), ("year", "genre", "id")):
            ids, rows = t.take_grad()
            grads[f"table {name}"] = densify_grad(t, ids, rows)
        return pos.detach(), neg.detach(), loss, grads

    pos, neg, loss, grads = run()
    # deterministic: the same step again gives the same bits (no float atomics on the path)
    pos2, neg2, loss2, grads2 = run()
    assert torch.equal(pos, pos2) and torch.equal(neg, neg2) and torch.equal(loss, loss2)
    assert grads.keys() == grads2.keys()
    for k in grads:
        assert torch.equal(grads[k], grads2[k]), f"{k} differs between two identical steps"
    # the restatement in float64 (the reference) and in fp32 (its rounding: the noise sample of
    # tests/conftest.py assert_close_f64: 1e-5 relative + 4x the fp32 error + 1e-6 of the largest)
    ref = {}
    for dt in (torch.float64, torch.float32):
        rh, P = torch_reference_repr(model, blocks, dt)
        rpos, rneg = item2item_scorer(pos_g, rh), item2item_scorer(neg_g, rh)
        rloss = torch.clamp(rneg + 1 - rpos, min=0).mean()
        rloss.backward()
        ref[dt] = (rpos.detach(), rneg.detach(), float(rloss), P)
    (p64, n64, l64, P64), (p32, n32, _, P32) = ref[torch.float64], ref[torch.float32]

    def close(got, name, r64, r32):
        # one fp32 sample of the restatement's rounding (the model sums some rows in other,
        # fixed orders: the genre multi-hot mean sequentially, the row gathers' backward by
        # sorted tiles): 4x its error, tests/conftest.py's default
        assert_close_f64(got, r64, r32, name, floor=1e-6, noise=4.0)

    close(pos, "pos score", p64, p32)
    close(neg, "neg score", n64, n32)
    assert abs(loss.item() - l64) <= 1e-5 * abs(l64)
    s = model.sagenet
    pairs = [(s.fc_2.kernel, "k2"), (s.fc_2.bias, "b2"), (s.fc_1.kernel, "k1"), (s.fc_1.bias, "b1")]
    for li, c in enumerate(s.convolves):
        pairs += [(c.fc_1.kernel, f"c{li}k1"), (c.fc_1.bias, f"c{li}b1"),
                  (c.fc_2.kernel, f"c{li}k2"), (c.fc_2.bias, f"c{li}b2")]
    for prm, name in pairs:
        close(prm.grad, name, P64[name].grad, P32[name].grad)
    assert int(model_oob_flag(pos.device)) == 0
    for name in ("year", "genre", "id"):
        close(grads[f"table {name}"], f"table {name}", P64[name].grad, P32[name].grad)


def test_pinsage_train_steps_reduce_loss():
    g, _ = small_graph(7, n_users=200, n_items=300, n_edges=3000)
    gen = torch.Generator(device=DEV).manual_seed(1)
    model = PinSageModel(g, g.itype, 2, 8, 32, 16, generator=gen)
    step = PinSageStep(model, lr=1e-2)
    smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
    h, p, n = item_pairs(g, 256, 4, 0)
    batch = smp.sample_from_item_pairs(h, p, n)
    losses = [float(step(*batch)) for _ in range(30)]
    assert np.isfinite(losses).all()
    assert losses[-1] < losses[0]


def test_sampling_matches_golden_fixture():
    import os

    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "pinsage.npz"))
    g = HeteroGraph(d["users"], d["items"], 40, 70, device=DEV,
                    item_data={"year": np.zeros(70, np.int64), "genre": np.zeros((70, 2), np.int8)})
    h, p, n = item_pairs(g, 48, 4, 2)
    np.testing.assert_array_equal(h.cpu().numpy(), d["heads"])
    np.testing.assert_array_equal(p.cpu().numpy(), d["pos"])
    smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
    smp.step = 2
    pos_g, neg_g, blocks = smp.sample_from_item_pairs(h, p, n)
    np.testing.assert_array_equal(pos_g.nodes.cpu().numpy(), d["seeds"])
    np.testing.assert_array_equal(neg_g.dst.cpu().numpy(), d["neg_dst"])
    for li, b in enumerate(blocks):
        E = int(b.n_edges.item())
        np.testing.assert_array_equal(b.src_nodes.cpu().numpy(), d[f"b{li}_src_nodes"])
        np.testing.assert_array_equal(b.indptr.cpu().numpy(), d[f"b{li}_indptr"])
        np.testing.assert_array_equal(b.edge_src[:E].cpu().numpy(), d[f"b{li}_edge_src"])
        np.testing.assert_array_equal(b.edge_w[:E].cpu().numpy(), d[f"b{li}_edge_w"])
        np.testing.assert_array_equal(b.t_indptr.cpu().numpy(), d[f"b{li}_t_indptr"])
        np.testing.assert_array_equal(b.t_edge[:E].cpu().numpy(), d[f"b{li}_t_edge"])


def _pinsage_params(model):
    return [p.detach().cpu().numpy().copy() for p in model.dense_parameters()] + \
        [t.weight.detach().cpu().numpy().copy() for t in model.tables()]


def _pinsage_world2_worker(rank, world, port, q):
    import os

    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from recommender_amd.optim import dedup_grad
        from recommender_amd.pinsage.model import margin_loss
        from recommender_amd.sharded import Comm

        B = 64
        g, _ = small_graph(7, n_users=200, n_items=300, n_edges=3000)
        model = PinSageModel(g, g.itype, 2, 8, 32, 16, generator=torch.Generator(device=DEV).manual_seed(1))
        step = PinSageStep(model, lr=1e-2, comm=Comm())
        smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
        if rank == 0:  # the expected result: one process, each rank's sub-batch in turn
            ref = PinSageModel(g, g.itype, 2, 8, 32, 16,
                               generator=torch.Generator(device=DEV).manual_seed(1))
            rstep = PinSageStep(ref, lr=1e-2)
            rsmp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
        for it in range(2):
            h, p, n = item_pairs(g, B, 4, it, pair_base=rank * B)
            step(*smp.sample_from_item_pairs(h, p, n))
            if rank == 0:
                buckets = []
                for r in range(world):
                    rstep.opt_dense.zero_grad(set_to_none=True)
                    rsmp.step = it
                    hr, pr, nr = item_pairs(g, B, 4, it, pair_base=r * B)
                    ps, ns = ref(*rsmp.sample_from_item_pairs(hr, pr, nr))
                    margin_loss(ps, ns, delta=1.0).backward()
                    grads = [x.grad if x.grad is not None else torch.zeros_like(x) for x in rstep.dense]
                    tabs = []
                    for t in ref.tables():
                        got = t.take_grad()
                        d = torch.zeros(t.input_dim, t.output_dim, device=DEV)
                        if got is not None:
                            rows, ug = dedup_grad(t, got[0], got[1])
                            d.index_copy_(0, rows, ug)
                        tabs.append(d)
                    buckets.append(grads + tabs)
                avg = [(a + b) * (1.0 / world) for a, b in zip(*buckets)]
                for x, gavg in zip(rstep.dense, avg[: len(rstep.dense)]):
                    x.grad = gavg
                rstep.opt_dense.step()
                prm = rstep.opt_sparse._params()
                for t, gavg in zip(ref.tables(), avg[len(rstep.dense):]):
                    ids = torch.arange(t.input_dim, device=DEV, dtype=torch.int32)
                    rstep.opt_sparse.apply(t, ids, gavg, prm)
                rstep.opt_sparse.iterations += 1
        torch.cuda.synchronize()
        mine = _pinsage_params(model)
        allp = [None] * world
        dist.all_gather_object(allp, mine)
        if rank == 0:
            for a, b in zip(allp[0], allp[1]):
                np.testing.assert_array_equal(a, b)  # the replicas stay identical
            for a, b in zip(mine, _pinsage_params(ref)):
                # the other rank's sub-batch ran in another process: its GEMM / kernel choices
                # may round differently (1.7e-6 relative measured), so 1e-5 here
                np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-7)
            moved = [float((a != b).mean()) for a, b in zip(mine, _pinsage_params(PinSageModel(
                g, g.itype, 2, 8, 32, 16, generator=torch.Generator(device=DEV).manual_seed(1))))]
            assert min(moved) > 0.0, moved
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_world2_pinsage_step_equals_two_sub_batches():
    """pairs sharded over two ranks (rank r draws pairs [rB, (r+1)B) of the
    step, pinsage/train/data_loader.py:6-18 keyed by pair index), graph and tables replicated,
    one all-reduce of the dense + densified table gradients (pinsage/train/train.py:40-48 under
    MirroredStrategy). Two steps on two gloo ranks sharing the GPU equal (1e-5) one process that
    averages the two sub-batches' gradients itself, and the replicas stay bit-identical. (The
    global Frobenius normalisation of Convolve, pinsage/train/layers.py:28-29, is per replica
    batch, as under MirroredStrategy, so a rank pair is NOT one 2B batch.)"""
    import os

    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29900 + (os.getpid() % 500)
    ps = [ctx.Process(target=_pinsage_world2_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(60)
    assert all(v == "ok" for v in res.values()), res


# ---- sync-free capacity-shaped step (PinSageSampler.sample_static, PinSageStep.capture) -----
def _live(t, n):
    return t[: int(n.item()) if torch.is_tensor(n) else n].cpu().numpy()


@pytest.mark.parametrize("batch", [48, 128])
def test_sample_static_equals_dynamic(batch):
    """The capacity-shaped batch's live part is the dynamic batch bit for bit (pairs with a
    dead-end walk dropped, seeds, both blocks' src nodes / CSR / transpose); padding is -1
    ids, empty CSR rows and k empty neighbour slots per padding seed."""
    g, _ = small_graph(3, n_users=120, n_items=200, n_edges=1500, dead_items=20)
    dyn = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
    sta = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
    for step in range(2):
        h, p, n = item_pairs(g, batch, 4, step)
        sh, sp, sn, nv = sta.sample_pairs_static(batch, 4, step)
        nvalid = int(nv.item())
        assert nvalid == h.numel() and nvalid < batch  # dead items drop some pairs
        for a, b in ((sh, h), (sp, p), (sn, n)):
            np.testing.assert_array_equal(_live(a, nvalid), b.cpu().numpy())
            assert (a[nvalid:] == -1).all()
        pg, ng, blocks = dyn.sample_from_item_pairs(h, p, n)
        spg, sng, sblocks = sta.sample_static(sh, sp, sn, nv)
        S = pg.nodes.numel()
        np.testing.assert_array_equal(_live(spg.nodes, S), pg.nodes.cpu().numpy())
        assert (spg.nodes[S:] == -1).all()
        np.testing.assert_array_equal(_live(spg.src, nvalid), pg.src.cpu().numpy())
        np.testing.assert_array_equal(_live(spg.dst, nvalid), pg.dst.cpu().numpy())
        np.testing.assert_array_equal(_live(sng.dst, nvalid), ng.dst.cpu().numpy())
        assert int(spg.valid.sum()) == nvalid
        for b, sb in zip(blocks, sblocks):
            E = int(b.n_edges.item())
            assert int(sb.n_edges.item()) == E
            assert int(sb.n_dst_live.item()) == b.n_dst and int(sb.n_src_live.item()) == b.n_src
            np.testing.assert_array_equal(_live(sb.src_nodes, b.n_src), b.src_nodes.cpu().numpy())
            assert (sb.src_nodes[b.n_src:] == -1).all()
            np.testing.assert_array_equal(_live(sb.indptr, b.n_dst + 1), b.indptr.cpu().numpy())
            assert (sb.indptr[b.n_dst:] == E).all()  # padding dst rows hold no edges
            for f in ("edge_src", "edge_dst", "edge_w", "t_edge"):
                np.testing.assert_array_equal(_live(getattr(sb, f), E),
                                              getattr(b, f)[:E].cpu().numpy(), err_msg=f)
            np.testing.assert_array_equal(_live(sb.t_indptr, b.n_src + 1),
                                          b.t_indptr.cpu().numpy())
            assert (sb.t_indptr[b.n_src:] == E).all()


def test_frobenius_rows_bit_exact_on_live_rows():
    """rs_frobenius_normalize_rows_*: norm and y / dx over the live rows equal the unpadded
    call bit for bit; padding rows come out 0."""
    torch.manual_seed(5)
    x = torch.randn(700, 16, device=DEV)
    dy = torch.randn(700, 16, device=DEV)
    n_live = torch.tensor([513], dtype=torch.int32, device=DEV)
    xs = x.clone().requires_grad_(True)
    y = frobenius_normalize(xs, n_live)
    y.backward(dy)
    xr = x[:513].clone().requires_grad_(True)
    yr = frobenius_normalize(xr)
    yr.backward(dy[:513])
    assert torch.equal(y[:513], yr) and not y[513:].any()
    assert torch.equal(xs.grad[:513], xr.grad) and not xs.grad[513:].any()


def _pinsage_setup(seed_model=1):
    g, _ = small_graph(7, n_users=200, n_items=300, n_edges=3000, dead_items=25)
    gen = torch.Generator(device=DEV).manual_seed(seed_model)
    model = PinSageModel(g, g.itype, 2, 8, 32, 16, generator=gen)
    smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
    return g, model, smp


def _param_ref_names(model):
    """named_parameters name -> torch_reference_repr leaf name."""
    s = model.sagenet
    out = {}
    pairs = [(s.fc_2.kernel, "k2"), (s.fc_2.bias, "b2"), (s.fc_1.kernel, "k1"), (s.fc_1.bias, "b1")]
    for li, c in enumerate(s.convolves):
        pairs += [(c.fc_1.kernel, f"c{li}k1"), (c.fc_1.bias, f"c{li}b1"),
                  (c.fc_2.kernel, f"c{li}k2"), (c.fc_2.bias, f"c{li}b2")]
    ids = {id(p): nm for p, nm in pairs}
    for k, v in model.named_parameters():
        if id(v) in ids:
            out[k] = ids[id(v)]
    return out


def test_static_forward_backward_equals_dynamic():
    """PinSageModel on the capacity-shaped batch: live scores, the masked margin loss and
    every gradient (dense and densified tables) — and the dynamic batch's — within fp32 rounding
    of the float64 restatement per element (padding contributes exactly nothing)."""
    from recommender_amd.optim import densify_grad
    from recommender_amd.pinsage.model import item2item_scorer, margin_loss

    B = 128
    g, model, dyn = _pinsage_setup()
    sta = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
    h, p, n = item_pairs(g, B, 4, 0)
    pg, ng, blocks = dyn.sample_from_item_pairs(h, p, n)
    pos, neg = model(pg, ng, blocks)
    margin_loss(pos, neg).backward()
    ref = {k: v.grad.clone() for k, v in model.named_parameters() if v.grad is not None}
    ref_tab = [densify_grad(t, *t.take_grad()) for t in model.tables()]
    model.zero_grad(set_to_none=True)
    spg, sng, sblocks = sta.sample_static(*sta.sample_pairs_static(B, 4, 0))
    spos, sneg = model(spg, sng, sblocks)
    sloss = margin_loss(spos, sneg, 1.0, spg.valid, spg.n_valid)
    sloss.backward()
    nv = h.numel()
    # both batches against the float64 restatement of the dynamic one (the fp32 restatement's
    # error as the noise sample: tests/conftest.py assert_close_f64)
    r = {}
    for dt in (torch.float64, torch.float32):
        rh, P = torch_reference_repr(model, blocks, dt)
        rp, rn = item2item_scorer(pg, rh), item2item_scorer(ng, rh)
        torch.clamp(rn + 1 - rp, min=0).mean().backward()
        r[dt] = (rp.detach(), rn.detach(), P)
    (p64, n64, P64), (p32, n32, P32) = r[torch.float64], r[torch.float32]
    for got, name in ((spos[:nv], "static pos"), (pos, "dynamic pos")):
        assert_close_f64(got, p64, p32, name, floor=1e-6)
    for got, name in ((sneg[:nv], "static neg"), (neg, "dynamic neg")):
        assert_close_f64(got, n64, n32, name, floor=1e-6)
    rl = margin_loss(pos, neg).item()
    assert abs(sloss.item() - rl) <= RTOL * abs(rl)
    names = _param_ref_names(model)
    for k, v in model.named_parameters():
        if k in ref:
            assert_close_f64(v.grad, P64[names[k]].grad, P32[names[k]].grad, f"static {k}",
                             floor=1e-6)
            assert_close_f64(ref[k], P64[names[k]].grad, P32[names[k]].grad, f"dynamic {k}",
                             floor=1e-6)
    for t, rt, name in zip(model.tables(), ref_tab, ("year", "genre", "id")):
        d = densify_grad(t, *t.take_grad())
        assert_close_f64(d, P64[name].grad, P32[name].grad, f"static table {name}", floor=1e-6)
        assert_close_f64(rt, P64[name].grad, P32[name].grad, f"dynamic table {name}", floor=1e-6)


def test_static_step_graph_replay_bit_exact_and_matches_dynamic():
    """Four training steps four ways: (a) the dynamic PinSageStep (host-synced shapes,
    SparseAdam + KerasAdam), (b) four eager static_steps, (c) one eager static_step, then
    the step captured once into a HIP graph and replayed three times on freshly sampled
    batches, (d) as (c) with the sampling inside the graph (capture_with_sampling: the RNG
    steps advance in device memory, so each replay samples the next step's batch). (c) equals (b) to 1e-5 (the lr_t of each replay comes from device memory; a
    frozen lr_t would be off by the bias-correction ratio, 0.18 vs 0.32 at step 4); (b) equals (a)
    to fp32 rounding order."""
    B = 96
    res = []
    for mode in ("dynamic", "static", "graph", "graph_all"):
        g, model, smp = _pinsage_setup()
        step = PinSageStep(model, lr=1e-2)
        losses = []
        replay = None
        for it in range(4):
            if mode == "dynamic":
                h, p, n = item_pairs(g, B, 4, it)
                losses.append(float(step(*smp.sample_from_item_pairs(h, p, n))))
                continue
            if mode == "graph_all" and it > 0:
                if replay is None:  # sampling inside the graph too, RNG steps on the device
                    replay = step.capture_with_sampling(smp, B, 4, it)
                losses.append(float(replay()))
                continue
            batch = smp.sample_static(*smp.sample_pairs_static(B, 4, it))
            if mode == "static" or it == 0:
                losses.append(float(step.static_step(*batch)))
                continue
            if replay is None:
                replay = step.capture(batch)
            losses.append(float(replay()))
        torch.cuda.synchronize()
        res.append((losses, _pinsage_params(model)))
    (l_dyn, p_dyn), (l_sta, p_sta), (l_gr, p_gr), (l_all, p_all) = res
    np.testing.assert_allclose(l_all, l_sta, rtol=1e-6)
    for a, b in zip(p_sta, p_all):
        np.testing.assert_allclose(b, a, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(l_gr, l_sta, rtol=1e-6)
    for a, b in zip(p_sta, p_gr):
        # measured: ulp-level (1.5e-6 relative) differences in one weight — the library GEMM
        # may pick another algorithm under stream capture than eagerly
        np.testing.assert_allclose(b, a, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(l_sta, l_dyn, rtol=1e-5)
    for a, b in zip(p_sta, p_dyn):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-6)
    moved = [float((a != b).mean()) for a, b in zip(p_gr, _pinsage_params(_pinsage_setup()[1]))]
    assert min(moved) > 0.0, moved


def test_graph_keras_adam_equals_keras_adam():
    """GraphKerasAdam (flat buffer, one rs_keras_adam_flat launch, lr_t from device memory)
    makes KerasAdam's update bit for bit over several steps, including parameters whose size
    is not a multiple of 4 and a window roll-over of the device lr_t history."""
    from recommender_amd.optim import GraphKerasAdam, KerasAdam

    torch.manual_seed(3)
    shapes = [(7, 5), (16,), (3,), (300, 8)]
    a = [torch.randn(s, device=DEV) for s in shapes]
    b = [t.clone() for t in a]
    ka = KerasAdam(a, lr=1e-2)
    ga = GraphKerasAdam(b, lr=1e-2, window=2)
    for it in range(5):
        gs = [torch.randn(s, device=DEV) for s in shapes]
        for t, g in zip(a, gs):
            t.grad = g
        ka.step()
        ga.prepare()
        ga.apply(gs)
        ga.iterations += 1
        for x, y in zip(a, b):
            assert torch.equal(x, y), it


def _pinsage_world2_static_worker(rank, world, port, q):
    import os

    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from recommender_amd.optim import dedup_grad
        from recommender_amd.pinsage.model import margin_loss
        from recommender_amd.sharded import Comm

        B = 64
        g, _ = small_graph(7, n_users=200, n_items=300, n_edges=3000)

        def fresh():
            return PinSageModel(g, g.itype, 2, 8, 32, 16,
                                generator=torch.Generator(device=DEV).manual_seed(1))

        # (a) eager sharded step with a dense parameter that has no gradient on rank 1 only, and
        # one that has none on any rank: same bucket layout on both ranks, the
        # first moves by the mean (rank 0's gradient / 2), the second is skipped as Keras does
        model = fresh()
        step = PinSageStep(model, lr=1e-2, comm=Comm())
        smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
        dense = model.dense_parameters()
        x, y = dense[0], dense[1]
        x0, y0 = x.detach().clone(), y.detach().clone()
        reduce = step._allreduce_and_apply_tables

        def drop_grads():  # the dense layers write .grad themselves: drop them before the bucket
            if rank == 1:
                x.grad = None
            y.grad = None
            reduce()

        step._allreduce_and_apply_tables = drop_grads
        h, p, n = item_pairs(g, B, 4, 0, pair_base=rank * B)
        step(*smp.sample_from_item_pairs(h, p, n))
        torch.cuda.synchronize()
        assert y.grad is None and x.grad is not None
        assert torch.equal(y, y0), "a parameter without a gradient on every rank must not move"
        assert not torch.equal(x, x0)
        mine = _pinsage_params(model)
        allp = [None] * world
        dist.all_gather_object(allp, mine)
        for a, b in zip(allp[0], allp[1]):
            np.testing.assert_array_equal(a, b)

        # (b) the sync-free static step sharded (flat-buffer all-reduce inside static_step) vs
        # one process averaging the two sub-batches' gradients (the dynamic step's arithmetic)
        model = fresh()
        step = PinSageStep(model, lr=1e-2, comm=Comm())
        smp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
        if rank == 0:
            ref = fresh()
            rstep = PinSageStep(ref, lr=1e-2)
            rsmp = PinSageSampler(g, g.itype, g.utype, 2, 2, 4, 0.0, 3, seed=4)
        for it in range(2):
            smp.step = it
            step.static_step(*smp.sample_static(*smp.sample_pairs_static(B, 4, it, rank * B)))
            if rank == 0:
                buckets = []
                for r in range(world):
                    rstep.opt_dense.zero_grad(set_to_none=True)
                    rsmp.step = it
                    hr, pr, nr = item_pairs(g, B, 4, it, pair_base=r * B)
                    ps, ns = ref(*rsmp.sample_from_item_pairs(hr, pr, nr))
                    margin_loss(ps, ns, delta=1.0).backward()
                    grads = [t.grad for t in rstep.dense]
                    tabs = []
                    for t in ref.tables():
                        got = t.take_grad()
                        d = torch.zeros(t.input_dim, t.output_dim, device=DEV)
                        rows, ug = dedup_grad(t, got[0], got[1])
                        d.index_copy_(0, rows, ug)
                        tabs.append(d)
                    buckets.append(grads + tabs)
                avg = [(a + b) * (1.0 / world) for a, b in zip(*buckets)]
                for t, gavg in zip(rstep.dense, avg[: len(rstep.dense)]):
                    t.grad = gavg
                rstep.opt_dense.step()
                prm = rstep.opt_sparse._params()
                for t, gavg in zip(ref.tables(), avg[len(rstep.dense):]):
                    ids = torch.arange(t.input_dim, device=DEV, dtype=torch.int32)
                    rstep.opt_sparse.apply(t, ids, gavg, prm)
                rstep.opt_sparse.iterations += 1
        torch.cuda.synchronize()
        mine = _pinsage_params(model)
        allp = [None] * world
        dist.all_gather_object(allp, mine)
        if rank == 0:
            for a, b in zip(allp[0], allp[1]):
                np.testing.assert_array_equal(a, b)  # the replicas stay identical
            for a, b in zip(mine, _pinsage_params(ref)):
                # static vs dynamic batches: fp32 rounding order (as the world-1 comparison)
                np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-6)
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_world2_pinsage_static_step_and_missing_gradients():
    """cfg5's sync-free (graph-capturable) step sharded over two gloo ranks: pairs split by
    global pair index, the flat gradient buffer all-reduced inside static_step, two steps equal
    one process averaging the two sub-batches (1e-4: static vs dynamic rounding), replicas
    bit-identical; and the eager sharded step with a parameter lacking a gradient on one rank
    (moves by the mean) or on every rank (skipped, as Keras skips it)."""
    import os

    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31300 + (os.getpid() % 500)
    ps = [ctx.Process(target=_pinsage_world2_static_worker, args=(r, world, port, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(60)
    assert all(v == "ok" for v in res.values()), res


@pytest.mark.parametrize("padded", [False, True])
def test_pair_margin_loss_fused_matches_scorer_and_margin(padded):
    """pair_margin_loss (rs_pair_margin_fwd / _bwd: both pair graphs' dot scores, the hinge, the
    live-pair mean and its gradient in one kernel each way) against item2item_scorer +
    margin_loss by autograd: loss and dL/dh within fp32 rounding; shared nodes across pairs (the
    backward scatter collides), padding pairs (-1 ids, valid 0) scoring node 0 with no weight,
    a hinge exactly at 0."""
    from recommender_amd.pinsage.graph import PairGraph
    from recommender_amd.pinsage.model import item2item_scorer, margin_loss, pair_margin_loss

    g = torch.Generator(device=DEV).manual_seed(7)
    N, D, P = 300, 16, 1000
    h = torch.randn(N, D, device=DEV, generator=g) * 0.3
    src = torch.randint(0, N, (P,), device=DEV, generator=g, dtype=torch.int32)
    pdst = torch.randint(0, 40, (P,), device=DEV, generator=g, dtype=torch.int32)  # collisions
    ndst = torch.randint(0, N, (P,), device=DEV, generator=g, dtype=torch.int32)
    ndst[5], pdst[5], src[5] = 3, 3, 4  # neg == pos row: hinge exactly delta, not at 0
    valid, n_valid = None, None
    if padded:
        valid = torch.ones(P, dtype=torch.bool, device=DEV)
        valid[P - 37:] = False
        src[P - 37:], pdst[P - 37:], ndst[P - 37:] = -1, -1, -1
        n_valid = torch.tensor([P - 37], dtype=torch.int32, device=DEV)
    pos_g = PairGraph(src, pdst, torch.arange(N, device=DEV), valid, n_valid)
    neg_g = PairGraph(src, ndst, torch.arange(N, device=DEV), valid, n_valid)
    h1 = h.clone().requires_grad_()
    loss = pair_margin_loss(pos_g, neg_g, h1, 1.0)
    loss.backward()
    h2 = h.clone().requires_grad_()
    ref = margin_loss(item2item_scorer(pos_g, h2), item2item_scorer(neg_g, h2), 1.0, valid, n_valid)
    ref.backward()
    assert abs(float(loss) - float(ref)) <= 1e-6 * abs(float(ref)) + 1e-7
    # a row's gradient sums its pairs' terms in sorted-tile order (the reference's index_add in
    # atomic arrival order): near-cancelling elements judged against the largest
    assert_close_rel(h1.grad.cpu(), h2.grad.cpu(), rtol=1e-5, scale=float(h2.grad.abs().max()) * 1e-1)
    # deterministic: the same call again gives the same bits
    h3 = h.clone().requires_grad_()
    loss3 = pair_margin_loss(pos_g, neg_g, h3, 1.0)
    loss3.backward()
    assert torch.equal(loss3, loss) and torch.equal(h3.grad, h1.grad)
    assert int(model_oob_flag(h.device)) == 0


def test_pair_margin_out_of_range_node_flags_and_reads_zero():
    """A pair endpoint past h's rows (the index_select it replaces raised) reads a zero row,
    receives no gradient and sets RS_ERRBIT_OOB; the other pairs are unaffected."""
    from recommender_amd.pinsage.graph import PairGraph
    from recommender_amd.pinsage.model import pair_margin_loss

    g = torch.Generator(device=DEV).manual_seed(9)
    N, D, P = 50, 8, 64
    h = torch.randn(N, D, device=DEV, generator=g)
    src = torch.randint(0, N, (P,), device=DEV, generator=g, dtype=torch.int32)
    pdst = torch.randint(0, N, (P,), device=DEV, generator=g, dtype=torch.int32)
    ndst = torch.randint(0, N, (P,), device=DEV, generator=g, dtype=torch.int32)
    flag = model_oob_flag(h.device)
    flag.zero_()
    ndst[3] = N + 5
    pos_g = PairGraph(src, pdst, torch.arange(N, device=DEV))
    neg_g = PairGraph(src, ndst, torch.arange(N, device=DEV))
    h1 = h.clone().requires_grad_()
    loss = pair_margin_loss(pos_g, neg_g, h1, 1.0)
    loss.backward()
    assert int(flag) & L.RS_ERRBIT_OOB
    # restated: the bad endpoint's score reads a zero row (score 0)
    pos = (h[src.long()] * h[pdst.long()]).sum(1)
    nd = ndst.long().clamp_max(N - 1)
    neg = (h[src.long()] * h[nd]).sum(1)
    neg[3] = 0.0
    ref = torch.clamp(neg + 1.0 - pos, min=0).mean()
    assert abs(float(loss) - float(ref)) <= 1e-5 * abs(float(ref))
    assert torch.isfinite(h1.grad).all()
    # the train loop's sync points turn the flag into an error (and clear it)
    from recommender_amd.pinsage.model import check_oob

    with pytest.raises(L.RecsysError, match="outside the representation rows"):
        check_oob(h.device)
    assert int(flag) == 0
    check_oob(h.device)  # clear: no error


def test_multihot_mean_lookup_matches_gather_mean():
    """multihot_mean_lookup (the genre feature: rs_multihot_mean_fwd / _bwd) against the gathered
    ids → table lookup → mean(dim=1) path: outputs, and the table's densified gradient, within
    fp32 rounding; ids spread over the whole table, repeated items, G = 20."""
    from recommender_amd.embedding import Embedding
    from recommender_amd.optim import densify_grad
    from recommender_amd.pinsage.layers import multihot_mean_lookup

    g = torch.Generator(device=DEV).manual_seed(3)
    n_items, G, V, D, N = 500, 20, 20, 8, 3000
    mh = torch.randint(0, V, (n_items, G), device=DEV, generator=g, dtype=torch.int32)
    mh[::3] = (mh[::3] < 2).to(torch.int32)  # genre-like {0, 1} rows
    items = torch.randint(0, n_items, (N,), device=DEV, generator=g)
    w = torch.randn(V, D, device=DEV, generator=g)
    up = torch.randn(N, D, device=DEV, generator=g)
    res = []
    for fused in (True, False):
        t = Embedding(V, D, device=DEV, weight=w.cpu())
        if fused:
            out = multihot_mean_lookup(t, mh, items)
        else:
            out = t(mh.index_select(0, items)).mean(dim=1)
        (out * up).sum().backward()
        ids, rows = t.take_grad()
        res.append((out.detach(), densify_grad(t, ids, rows)))
    (o1, d1), (o2, d2) = res
    # 20-term sums in another order: near-cancelling elements judged against the largest
    assert_close_rel(o1.cpu(), o2.cpu(), rtol=1e-5, scale=float(o2.abs().max()) * 1e-1)
    assert_close_rel(d1.cpu(), d2.cpu(), rtol=1e-5, scale=float(d2.abs().max()) * 1e-1)
