"""GPU parity: embedding gather, radix sort / dedup and the sparse optimizer applies vs the
CPU oracle (bit-exact: gather is a copy, sort is integer work, the segmented sums follow the
oracle's fixed order and -ffp-contract=off keeps the update roundings identical)."""
import numpy as np
import pytest
import torch

from oracle import embedding as O
from recommender_amd import _lib as L
from recommender_amd.embedding import Embedding, SlabEmbedding
from recommender_amd.optim import SortedIds, SparseAdam, SparseSGD, dedup_grad, keras_adam_coefficients

pytestmark = pytest.mark.gpu
DEV = "cuda"


def zipf_ids(rng, n, card, a=1.05):
    x = rng.zipf(a, size=n) - 1
    return np.minimum(x, card - 1)


@pytest.mark.parametrize("dim", [16, 18, 64, 128, 160, 7])
@pytest.mark.parametrize("id_dtype", [np.int64, np.int32])
def test_gather_shared_table(dim, id_dtype, rng):
    V, B, S = 5000, 257, 26
    w = rng.standard_normal((V, dim)).astype(np.float32)
    ids = rng.integers(0, V, (B, S)).astype(id_dtype)
    t = Embedding(V, dim, device=DEV, weight=torch.from_numpy(w))
    out = t(torch.from_numpy(ids).to(DEV))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.detach().cpu().numpy(), O.embedding_lookup(w, ids))
    assert not t.oob_detected()


@pytest.mark.parametrize("dim,ld", [(18, 36), (18, 20), (6, 10), (18, 18), (16, 40), (7, 9)])
def test_gather_strided_vs_oracle(dim, ld, rng):
    """rs_embedding_fwd_strided into a column block of a wider row (out_ld > dim, the flat pair
    form for even D that is not a multiple of 4): the block equals the oracle's lookup, OOB ids
    read zero rows and flag, and every other column keeps its sentinel."""
    V, n = 5000, 40_961
    w = rng.standard_normal((V, dim)).astype(np.float32)
    ids = rng.integers(0, V, n).astype(np.int64)
    ids[::97] = V + 5
    out = torch.full((n, ld), 7.0, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    tw = torch.from_numpy(w).to(DEV)
    ti = torch.from_numpy(ids).to(DEV)
    L.call("rs_embedding_fwd_strided", L.ptr(tw), V, dim, L.ptr(ti), 1, n, None, 1, L.ptr(out),
           ld, L.ptr(err), L.stream_ptr(DEV))
    got = out.cpu().numpy()
    np.testing.assert_array_equal(got[:, :dim], O.embedding_lookup(w, ids, raise_oob=False))
    assert (got[:, dim:] == 7.0).all()
    assert int(err.item()) != 0


@pytest.mark.parametrize("da,db", [(18, 18), (16, 7), (64, 128)])
def test_concat_lookup_matches_cat_of_lookups(da, db, rng):
    """functional.embedding_lookup_concat (two strided gathers into one [.., da + db] output,
    dien/model.py:14-19's tf.concat) == torch.cat of the two lookups, forward bit for bit; its
    backward hands each table its column block (with the grad mask), so the densified table
    gradients equal the two-lookup path's bit for bit; an out-of-range id flags its own table."""
    from recommender_amd.functional import embedding_lookup_concat
    from recommender_amd.optim import densify_grad, _Workspace

    Va, Vb, B, Lh = 3000, 40, 33, 17
    wa = torch.from_numpy(rng.standard_normal((Va, da)).astype(np.float32))
    wb = torch.from_numpy(rng.standard_normal((Vb, db)).astype(np.float32))
    ia = torch.from_numpy(rng.integers(0, Va, (B, Lh)).astype(np.int32)).to(DEV)
    ib = torch.from_numpy(rng.integers(0, Vb, (B, Lh)).astype(np.int32)).to(DEV)
    ib[5, 3] = Vb + 2  # out of range for table b only
    mask = ia != 0
    mask[::3, 10:] = False
    up = torch.from_numpy(rng.standard_normal((B, Lh, da + db)).astype(np.float32)).to(DEV)
    grads = []
    for fused in (True, False):
        ta = Embedding(Va, da, device=DEV, weight=wa)
        tb = Embedding(Vb, db, device=DEV, weight=wb)
        if fused:
            out = embedding_lookup_concat(ta, ia, tb, ib, mask)
        else:
            out = torch.cat([ta(ia, mask), tb(ib, mask)], -1)
        (out * up).sum().backward()
        torch.cuda.synchronize()
        assert not ta.oob_detected() and tb.oob_detected()
        ws = _Workspace()
        g = []
        for t in (ta, tb):
            ids, rows, valid = t.take_grad(with_valid=True)
            g.append(densify_grad(t, ids, rows, ws, valid=valid).cpu())
        grads.append((out.detach().cpu(), g))
    (o1, g1), (o2, g2) = grads
    assert torch.equal(o1, o2)
    assert torch.equal(g1[0], g2[0]) and torch.equal(g1[1], g2[1])


@pytest.mark.parametrize("dim", [18, 16, 64, 128, 7])
@pytest.mark.parametrize("n_lookups", [2, 3, 4])
def test_densify_segments_equal_concatenation(dim, n_lookups, rng):
    """densify_grad over a table's lookups handed as separate (strided) row views
    (take_grad(segments=True): rs_embedding_grad_dense_segs) equals the densified concatenation
    bit for bit — with and without valid flags, with column-block views (row stride > dim), a
    one-row lookup, and an out-of-range id (dropped on both sides)."""
    from recommender_amd.optim import _Workspace, densify_grad

    V = 3001 if dim != 7 else 500
    sizes = [1, 4096 * 3 + 5, 700, 9000][:n_lookups]
    for with_valid in (False, True):
        ws = _Workspace()
        ids = [torch.from_numpy(rng.integers(0, V, n).astype(np.int32)).to(DEV) for n in sizes]
        ids[-1][3] = V + 1
        wide = [torch.from_numpy(rng.standard_normal((n, 2 * dim + 2)).astype(np.float32)).to(DEV)
                for n in sizes]
        views = [w[:, :dim] if i % 2 == 0 else w[:, dim + 2:] for i, w in enumerate(wide)]
        valid = None
        if with_valid:
            valid = [torch.from_numpy((rng.random(n) < 0.7).astype(np.uint8)).to(DEV)
                     for n in sizes]
        res = []
        for segmented in (True, False):
            t = Embedding(V, dim, device=DEV)
            for k in range(n_lookups):
                t.accumulate_grad(ids[k], views[k], None if valid is None else valid[k])
            got = t.take_grad(with_valid=True, segments=segmented)
            assert isinstance(got[1], list) == segmented
            res.append(densify_grad(t, got[0], got[1], ws, valid=got[2]).cpu())
        assert torch.equal(res[0], res[1])
        assert res[0].abs().sum() > 0


def test_gather_slab_and_oob(rng):
    card = [7, 1, 300, 50]
    dim = 64
    t = SlabEmbedding(card, dim, device=DEV)
    w = t.weight.cpu().numpy()
    so = np.concatenate([[0], np.cumsum(card)])
    ids = np.stack([rng.integers(0, c, 1000) for c in card], 1).astype(np.int64)
    ids[3, 1] = 1      # out of range for a 1-row slot
    ids[10, 2] = -5    # negative
    out = t(torch.from_numpy(ids).to(DEV)).detach().cpu().numpy()
    ref = O.embedding_lookup(w, ids, so, raise_oob=False)
    np.testing.assert_array_equal(out, ref)
    assert (out[3, 1] == 0).all() and (out[10, 2] == 0).all()
    assert t.oob_detected()
    with pytest.raises(IndexError):
        O.embedding_lookup(w, ids, so, raise_oob=True)


@pytest.mark.parametrize("n,V", [(1, 10), (1000, 7), (4096 * 3 + 17, 1000), (200_000, 40_000_000), (65536, 3)])
def test_sort_ids(n, V, rng):
    ids = zipf_ids(rng, n, V).astype(np.int64)
    ids[::97] = V + 3  # OOB
    s = SortedIds(torch.from_numpy(ids).to(DEV), V)
    rows_ref, pos_ref, nu_ref = O.sort_ids(ids, V)
    np.testing.assert_array_equal(s.rows.cpu().numpy().view(np.uint32), rows_ref)
    np.testing.assert_array_equal(s.pos.cpu().numpy(), pos_ref)
    assert int(s.n_unique.item()) == nu_ref


@pytest.mark.parametrize("n", [2, 16383, 16384])
@pytest.mark.parametrize("V", [1, 3000, 65535, 262141])
@pytest.mark.parametrize("masked", [False, True])
def test_sort_ids_small_one_workgroup(n, V, masked, rng):
    """A one-slot sort of at most 16 384 ids over fewer than 2^18 - 2 rows runs as one workgroup
    (small_sort_kernel: 8-bit digit passes between two LDS buffers): bit-exact against the
    oracle's stable sort — the 16 384 limit, one-row and 18-bit key spaces, OOB ids, masked
    positions, a one-slot slab's offsets, the unique count."""
    ids = zipf_ids(rng, n, V).astype(np.int64)
    ids[1::7] = rng.integers(0, V, ids[1::7].shape)
    ids[::97] = V + 3  # OOB
    ids[5::101] = -1
    so = np.array([0, V], np.int64) if masked else None  # a one-slot slab on one side
    dev_so = None if so is None else torch.from_numpy(so).to(DEV)
    if masked:
        keep = rng.random(n) < 0.6
        s = SortedIds(torch.from_numpy(ids.astype(np.int32)).to(DEV), V, dev_so,
                      valid=torch.from_numpy(keep.astype(np.uint8)).to(DEV))
        rows_ref, pos_ref, nu_ref = O.sort_ids(np.where(keep, ids, -1), V, so)
    else:
        s = SortedIds(torch.from_numpy(ids).to(DEV), V, dev_so)
        rows_ref, pos_ref, nu_ref = O.sort_ids(ids, V, so)
    np.testing.assert_array_equal(s.rows.cpu().numpy().view(np.uint32), rows_ref)
    np.testing.assert_array_equal(s.pos.cpu().numpy(), pos_ref)
    assert int(s.n_unique.item()) == nu_ref


@pytest.mark.parametrize("runs,run_len,V", [(1, 1000, 500), (2, 4096, 30_000), (3, 777, 50),
                                             (8, 35_000, 5_000_000)])
def test_sort_ids_runs_merge_equals_masked_sort(runs, run_len, V, rng):
    """rs_sort_ids_runs (the row-sharded owner's merge of its W received blocks): each run
    ascending unique rows then -1 padding, rows shared between runs, an all-padding run and an
    out-of-range row at a run's end — bit-exact against the oracle's stable sort with the padding
    masked, and the OOB row flagged."""
    ids = np.full((runs, run_len), -1, np.int64)
    for r in range(runs):
        k = 0 if (runs > 2 and r == 1) else min(int(rng.integers(run_len // 3, run_len + 1)), V)
        ids[r, :k] = np.sort(rng.choice(V, size=k, replace=False))
    if runs > 1 and (ids[0] >= 0).sum() < run_len:
        k0 = int((ids[0] >= 0).sum())
        ids[0, k0] = V + 2  # a row past the table: a sentinel, flagged
    flat = ids.reshape(-1).astype(np.int32)
    keep = (flat >= 0) & (flat < V)
    rows_ref, pos_ref, _ = O.sort_ids(np.where(keep, flat, -1).astype(np.int64), V)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    s = SortedIds.from_runs(torch.from_numpy(flat).to(DEV), runs, V, err)
    np.testing.assert_array_equal(s.rows.cpu().numpy().view(np.uint32), rows_ref)
    np.testing.assert_array_equal(s.pos.cpu().numpy(), pos_ref)
    assert (int(err.item()) != 0) == bool((flat >= V).any())


@pytest.mark.parametrize("n", [16384, 40_000])
def test_index_add_rows_fixed_order(n, rng):
    """rs_index_add_rows (PinSage's deterministic scatter-add: sort + tiled segmented sum) through
    the C-ABI: out[r] = Σ rows[i] over ids[i] = r within fp32 summation error of the float64 sum,
    run-to-run identical, masked positions left out, an out-of-range id skipped and flagged —
    at the one-workgroup sort's limit and past it."""
    V, D = 5000, 24
    ids = zipf_ids(rng, n, V).astype(np.int32)
    ids[7] = V + 1  # OOB
    keep = rng.random(n) < 0.9
    rows = rng.standard_normal((n, D)).astype(np.float32)
    ok = keep & (ids >= 0) & (ids < V)
    ref = np.zeros((V, D))
    np.add.at(ref, ids[ok].astype(np.int64), rows[ok].astype(np.float64))
    gi = torch.from_numpy(ids).to(DEV)
    gv = torch.from_numpy(keep.astype(np.uint8)).to(DEV)
    gr = torch.from_numpy(rows).to(DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    ws = torch.empty(L.lib().rs_index_add_rows_workspace_size(n, D), dtype=torch.uint8, device=DEV)
    outs = []
    for _ in range(2):
        out = torch.empty(V, D, device=DEV)
        L.call("rs_index_add_rows", L.ptr(gi), L.id_dtype_code(gi), n, L.ptr(gv), L.ptr(gr), D, V,
               L.ptr(out), L.ptr(err), L.ptr(ws), ws.numel(), L.stream_ptr(DEV))
        outs.append(out)
    assert torch.equal(outs[0], outs[1])
    got = outs[0].cpu().numpy()
    cnt = np.maximum(np.bincount(ids[ok].astype(np.int64), minlength=V), 1)[:, None]
    assert (np.abs(got - ref) <= 1e-5 * (np.abs(ref) + np.sqrt(cnt) * 4.0)).all()
    if keep[7]:  # a masked-out position is not an error
        assert int(err.item()) != 0


@pytest.mark.parametrize("n", [(1 << 17) - 1, 1 << 17, (1 << 20) - 1, 1 << 20])
@pytest.mark.parametrize("masked", [False, True])
def test_sort_ids_tile_size_switch_points(n, masked, rng):
    """The sort's keys per lane (tile size) switch at n = 2^17 (512 -> 1024-key tiles) and 2^20
    (1024 -> 4096): both sides of each switch, plain and masked (left-out positions take the
    sentinel key), rows / positions / unique count bit-exact vs the oracle's stable sort."""
    V = 40_000_000
    ids = zipf_ids(rng, n, V).astype(np.int64)
    ids[::101] = V + 5  # OOB
    dev_ids = torch.from_numpy(ids).to(DEV)
    if masked:
        keep = rng.random(n) < 0.4
        s = SortedIds(dev_ids, V, valid=torch.from_numpy(keep.astype(np.uint8)).to(DEV))
        rows_ref, pos_ref, nu_ref = O.sort_ids(np.where(keep, ids, -1), V)
    else:
        s = SortedIds(dev_ids, V)
        rows_ref, pos_ref, nu_ref = O.sort_ids(ids, V)
    np.testing.assert_array_equal(s.rows.cpu().numpy().view(np.uint32), rows_ref)
    np.testing.assert_array_equal(s.pos.cpu().numpy(), pos_ref)
    assert int(s.n_unique.item()) == nu_ref


@pytest.mark.parametrize("per_slot", [10_000_000, 40_000_000])
def test_sort_ids_large_slab_four_passes(per_slot, rng):
    """SURVEY cfg2's 26 x 10M-row slab (260M rows: 28 key bits, four 7-bit passes) and a 1.04B-row
    key space (30 bits, four 8-bit passes): the slab itself is not needed, only its slot offsets.
    Zipf ids per slot plus out-of-range ones, bit-exact vs the oracle's stable sort."""
    from recommender_amd.synthetic import criteo_batch

    S, B = 26, 8192
    cards = [per_slot] * S
    cat, _, _ = criteo_batch(rng, B, cards)
    cat[::113, 5] = per_slot + 7  # OOB in slot 5
    so = np.concatenate([[0], np.cumsum(cards)]).astype(np.int64)
    V = int(so[-1])
    s = SortedIds(torch.from_numpy(cat).to(DEV), V, torch.from_numpy(so).to(DEV))
    rows_ref, pos_ref, nu_ref = O.sort_ids(cat, V, so)
    np.testing.assert_array_equal(s.rows.cpu().numpy().view(np.uint32), rows_ref)
    np.testing.assert_array_equal(s.pos.cpu().numpy(), pos_ref)
    assert int(s.n_unique.item()) == nu_ref


@pytest.mark.parametrize("B", [1, 4095, 4096, 4097, 65536, 131072])
@pytest.mark.parametrize("layout", ["slab26", "shared"])
@pytest.mark.parametrize("masked", [False, True])
def test_sort_ids_slot_segmented(B, layout, masked, rng):
    """The slot-segmented sort (rs_sort_ids_slots: per-slot two-pass 12-bit LSD, 4 launches)
    against the oracle's stable sort, bit-exact: tile edges (4096-example tiles, up to the
    32-tile limit), one-row / 12-bit / 13-bit / 2^24-row / Criteo-scale slots (one and two
    passes), int32 and int64 ids, out-of-range ids in several slots and masked positions (the
    sentinels grouped by slot after all valid rows), the unique count."""
    if layout == "slab26":
        cards = [1, 4096, 4097, 1 << 24, 12_010_734, 3, 100_000] + [1000 + 37 * i for i in range(19)]
        S = len(cards)
        so = np.concatenate([[0], np.cumsum(cards)]).astype(np.int64)
        V = int(so[-1])
        ids = np.stack([zipf_ids(rng, B, c) for c in cards], 1).astype(np.int64)
        for j, c in enumerate(cards):  # every third id uniform: all digits of wide slots
            ids[1::3, j] = rng.integers(0, c, ids[1::3, j].shape)
        ids[::53, 4] = cards[4] + 11  # OOB in two slots
        ids[::71, 9] = -2
        dev_so = torch.from_numpy(so).to(DEV)
        msr = max(cards)
    else:
        S, V = 1, 5_000_000
        so, dev_so, msr = None, None, None
        ids = zipf_ids(rng, B, V).astype(np.int64)
        ids[::61] = V + 1
    dt = np.int32 if masked else np.int64  # both id widths
    ids_t = torch.from_numpy(ids.astype(dt)).to(DEV)
    flat = ids.reshape(-1)
    if masked:
        keep = rng.random(flat.size) < 0.7
        s = SortedIds(ids_t, V, dev_so, valid=torch.from_numpy(keep.astype(np.uint8)).to(DEV),
                      max_slot_rows=msr)
        rows_ref, pos_ref, nu_ref = O.sort_ids(np.where(keep, flat, -1).reshape(ids.shape), V, so)
    else:
        s = SortedIds(ids_t, V, dev_so, max_slot_rows=msr)
        rows_ref, pos_ref, nu_ref = O.sort_ids(ids, V, so)
    np.testing.assert_array_equal(s.rows.cpu().numpy().view(np.uint32), rows_ref)
    np.testing.assert_array_equal(s.pos.cpu().numpy(), pos_ref)
    assert int(s.n_unique.item()) == nu_ref


@pytest.mark.parametrize("B", [2049, 6000, 65536, 131072])
@pytest.mark.parametrize("pattern", ["one_id", "two_buckets", "sparse_buckets", "window_edges"])
def test_sort_ids_slot_segmented_clustered_ids(B, pattern, rng):
    """The slot-segmented sort on clustered wide-slot ids: one id for the whole slot, two hot
    12-bit high-digit buckets, a few occupied buckets among 4096, and runs of 1500-2600 keys per
    bucket — bit-exact vs the oracle's stable sort, with OOB ids and masked positions mixed in."""
    cards = [1 << 24, 5000, 9_000_001, 4097]
    S = len(cards)
    so = np.concatenate([[0], np.cumsum(cards)]).astype(np.int64)
    V = int(so[-1])
    ids = np.empty((B, S), np.int64)
    for j, c in enumerate(cards):
        sh = max(int(c - 1).bit_length() - 12, 0)  # low bits below the bucket digit
        if pattern == "one_id":
            ids[:, j] = c // 3
        elif pattern == "two_buckets":
            ids[:, j] = np.where(rng.random(B) < 0.5, 7, (c - 1) >> sh << sh)
            ids[::5, j] = rng.integers(0, c, ids[::5, j].shape)
        elif pattern == "sparse_buckets":
            buckets = rng.choice((c - 1 >> sh) + 1, 5, replace=False)
            ids[:, j] = (rng.choice(buckets, B) << sh) + rng.integers(0, 1 << sh, B)
            ids[:, j] = np.minimum(ids[:, j], c - 1)
        else:  # runs of 1500..2600 keys per bucket over consecutive buckets
            sizes = rng.integers(1500, 2600, B // 1500 + 2)
            bucket = np.repeat(np.arange(sizes.size), sizes)[:B] % ((c - 1 >> sh) + 1)
            ids[:, j] = np.minimum((bucket << sh) + rng.integers(0, 1 << sh, B), c - 1)
    ids[::97, 2] = cards[2] + 3  # OOB
    keep = rng.random(ids.size) < 0.9
    s = SortedIds(torch.from_numpy(ids).to(DEV), V, torch.from_numpy(so).to(DEV),
                  valid=torch.from_numpy(keep.astype(np.uint8)).to(DEV), max_slot_rows=max(cards))
    rows_ref, pos_ref, nu_ref = O.sort_ids(np.where(keep, ids.reshape(-1), -1).reshape(ids.shape), V, so)
    np.testing.assert_array_equal(s.rows.cpu().numpy().view(np.uint32), rows_ref)
    np.testing.assert_array_equal(s.pos.cpu().numpy(), pos_ref)
    assert int(s.n_unique.item()) == nu_ref


def test_sort_ids_lsd_slot_sentinels(rng):
    """A slab with a slot past 2^24 rows takes the LSD sort: its sentinels (OOB ids in several
    slots, masked positions) come out grouped by slot like the slot-segmented sort's."""
    cards = [40_000_000, 17, 300_000, 5]
    S, B = len(cards), 20_000
    so = np.concatenate([[0], np.cumsum(cards)]).astype(np.int64)
    V = int(so[-1])
    ids = np.stack([zipf_ids(rng, B, c) for c in cards], 1).astype(np.int64)
    ids[::29, 1] = 99
    ids[::31, 3] = -1
    keep = rng.random(ids.size) < 0.8
    s = SortedIds(torch.from_numpy(ids).to(DEV), V, torch.from_numpy(so).to(DEV),
                  valid=torch.from_numpy(keep.astype(np.uint8)).to(DEV), max_slot_rows=max(cards))
    rows_ref, pos_ref, nu_ref = O.sort_ids(np.where(keep, ids.reshape(-1), -1).reshape(ids.shape), V, so)
    np.testing.assert_array_equal(s.rows.cpu().numpy().view(np.uint32), rows_ref)
    np.testing.assert_array_equal(s.pos.cpu().numpy(), pos_ref)
    assert int(s.n_unique.item()) == nu_ref


def test_sort_ids_empty():
    s = SortedIds(torch.zeros(0, dtype=torch.int64, device=DEV), 10)
    assert s.n == 0 and int(s.n_unique.item()) == 0


@pytest.mark.parametrize("dim", [128, 64, 18, 16, 160, 3])
@pytest.mark.parametrize("dist", ["zipf", "one_hot_row", "uniform"])
def test_dedup_grad_order(dim, dist, rng):
    V, n = 20_000, 33 * 32 + 5
    if dist == "zipf":
        ids = zipf_ids(rng, n, V)
    elif dist == "one_hot_row":
        ids = np.full(n, 17)
        ids[::5] = 3
    else:
        ids = rng.integers(0, V, n)
    ids = ids.astype(np.int64)
    g = rng.standard_normal((n, dim)).astype(np.float32)
    t = Embedding(V, dim, device=DEV)
    ur, ug = dedup_grad(t, torch.from_numpy(ids).to(DEV), torch.from_numpy(g).to(DEV))
    sr, sp, nu = O.sort_ids(ids, V)
    rr, rg = O.segment_sum_tiled(sr, sp, g, V)
    np.testing.assert_array_equal(ur.cpu().numpy(), rr.astype(np.int64))
    np.testing.assert_array_equal(ug.cpu().numpy(), rg)


@pytest.mark.parametrize("lens", [
    [31, 32, 33, 1, 1024, 1023, 1025, 2, 2048 + 7, 5, 32 * 32 * 3, 64],
    [992, 32, 1, 31, 1024 * 2 - 1, 1, 1056, 7],
    [1] * 100 + [3000] + [1] * 33,
])
def test_segment_runs_across_tile_groups(lens, rng):
    """D = 128 walk (seg_group32_kernel: tiles of 32 in aligned groups of 32, level-1 fold in
    LDS, level-2 fold across groups): runs ending on / just past tile and group edges, runs
    spanning several groups, a group whose first tile continues a run, singletons between.
    Dedup rows and SGD update bit-exact against the oracle's tiled order."""
    V, dim = 50_000, 128
    rows = rng.choice(V, len(lens), replace=False)
    ids = np.concatenate([np.full(n, r) for n, r in zip(lens, sorted(rows))]).astype(np.int64)
    ids = ids[rng.permutation(ids.size)]
    g = rng.standard_normal((ids.size, dim)).astype(np.float32)
    t = Embedding(V, dim, device=DEV)
    ur, ug = dedup_grad(t, torch.from_numpy(ids).to(DEV), torch.from_numpy(g).to(DEV))
    sr, sp, _ = O.sort_ids(ids, V)
    rr, rg = O.segment_sum_tiled(sr, sp, g, V)
    np.testing.assert_array_equal(ur.cpu().numpy(), rr.astype(np.int64))
    np.testing.assert_array_equal(ug.cpu().numpy(), rg)
    w0 = rng.standard_normal((V, dim)).astype(np.float32)
    t = Embedding(V, dim, device=DEV, weight=torch.from_numpy(w0))
    opt = SparseSGD(t, lr=0.05)
    t.accumulate_grad(torch.from_numpy(ids).to(DEV), torch.from_numpy(g).to(DEV))
    opt.step()
    np.testing.assert_array_equal(t.weight.cpu().numpy(), O.apply_sgd(w0, rr, rg, np.float32(0.05)))


@pytest.mark.parametrize("dim", [128, 18])
def test_sgd_apply_bitexact(dim, rng):
    V, B, S = 30_000, 512, 26
    w0 = rng.standard_normal((V, dim)).astype(np.float32)
    ids = zipf_ids(rng, B * S, V).reshape(B, S).astype(np.int64)
    g = rng.standard_normal((B * S, dim)).astype(np.float32)
    t = Embedding(V, dim, device=DEV, weight=torch.from_numpy(w0))
    opt = SparseSGD(t, lr=0.05)
    t.accumulate_grad(torch.from_numpy(ids).to(DEV), torch.from_numpy(g).to(DEV))
    opt.step()
    sr, sp, _ = O.sort_ids(ids, V)
    ur, ug = O.segment_sum_tiled(sr, sp, g, V)
    ref = O.apply_sgd(w0, ur, ug, np.float32(0.05))
    np.testing.assert_array_equal(t.weight.cpu().numpy(), ref)


@pytest.mark.parametrize("mode", ["lazy", "keras"])
def test_adam_apply_bitexact(mode, rng):
    V, dim, n = 5000, 64, 4000
    w0 = rng.standard_normal((V, dim)).astype(np.float32)
    t = Embedding(V, dim, device=DEV, weight=torch.from_numpy(w0))
    opt = SparseAdam(t, lr=1e-3, mode=mode)
    w, m, v = w0.copy(), np.zeros_like(w0), np.zeros_like(w0)
    for step in range(1, 4):
        ids = zipf_ids(rng, n, V).astype(np.int64)
        g = rng.standard_normal((n, dim)).astype(np.float32)
        t.accumulate_grad(torch.from_numpy(ids).to(DEV), torch.from_numpy(g).to(DEV))
        opt.step()
        sr, sp, _ = O.sort_ids(ids, V)
        ur, ug = O.segment_sum_tiled(sr, sp, g, V)
        c = O.keras_adam_coefficients(step)
        if mode == "lazy":
            w, m, v = O.apply_lazy_adam(w, m, v, ur, ug, c)
        else:
            w, m, v = O.apply_keras_adam(w, m, v, ur, ug, c)
    mg, vg, _ = opt.state[id(t)]
    np.testing.assert_array_equal(mg.cpu().numpy(), m)
    np.testing.assert_array_equal(vg.cpu().numpy(), v)
    np.testing.assert_array_equal(t.weight.cpu().numpy(), w)


def test_keras_adam_coefficients_match_oracle():
    for step in (1, 2, 10, 1000):
        c = keras_adam_coefficients(step)
        r = O.keras_adam_coefficients(step)
        assert np.float32(c.lr) == r["lr"]


@pytest.mark.parametrize("optimizer", ["sgd", "lazy_adam", "keras_adam"])
def test_fused_side_stream_apply_matches_unfused(optimizer, rng):
    """The side-stream fused optimizer (sort before the dense forward, apply inside the
    backward; optionally joined only at the next step's first table read) must give the same
    table bit for bit as the step()-time apply."""
    from recommender_amd.ctr.train import TrainStep, build_model
    from recommender_amd.synthetic import criteo_batch, criteo_cardinalities

    cards = criteo_cardinalities(300_000, 26)
    models, steps = [], []
    for fused, defer in ((False, False), (True, False), (True, True)):
        g = torch.Generator(device=DEV)
        g.manual_seed(7)
        m = build_model("DLRM", 32, sum(cards), 26, 13, DEV, slot_cardinalities=cards,
                        bottom=[64, 32], top=[64, 1], generator=g)
        models.append(m)
        steps.append(TrainStep(m, optimizer, lr=0.05 if optimizer == "sgd" else 1e-3, fused=fused,
                               defer_sparse_join=defer))
    r = np.random.default_rng(3)
    for _ in range(3):
        cat, dn, lb = criteo_batch(r, 2048, cards)
        b = (torch.from_numpy(cat).to(DEV), torch.from_numpy(dn).to(DEV), torch.from_numpy(lb).to(DEV))
        for st in steps:
            st(b)
    torch.cuda.synchronize()
    ref = models[0].embedding_layer.weight.cpu().numpy()
    for m in models[1:]:  # fused, and fused with the join deferred to the next table read
        np.testing.assert_array_equal(ref, m.embedding_layer.weight.cpu().numpy())


def test_golden_fixture_on_gpu():
    """The HIP path reproduces the committed golden vectors bit for bit."""
    import os

    f = np.load(os.path.join(os.path.dirname(__file__), "golden", "embedding.npz"))
    so, ids, table, grad = f["slot_offsets"], f["ids"], f["table"], f["grad"]
    card = np.diff(so)
    t = SlabEmbedding(card, table.shape[1], device=DEV, weight=torch.from_numpy(table))
    out = t(torch.from_numpy(ids).to(DEV)).detach().cpu().numpy()
    np.testing.assert_array_equal(out, f["emb"])
    s = SortedIds.for_table(t, torch.from_numpy(ids).to(DEV))
    np.testing.assert_array_equal(s.rows.cpu().numpy().view(np.uint32), f["sorted_rows"])
    np.testing.assert_array_equal(s.pos.cpu().numpy(), f["sorted_pos"])
    ur, ug = dedup_grad(t, torch.from_numpy(ids).to(DEV), torch.from_numpy(grad).to(DEV))
    np.testing.assert_array_equal(ur.cpu().numpy(), f["uniq_rows"].astype(np.int64))
    np.testing.assert_array_equal(ug.cpu().numpy(), f["uniq_grad"])
    for kind, key in (("sgd", "sgd"), ("lazy", "lazy_w"), ("keras", "keras_w")):
        t.weight.copy_(torch.from_numpy(table))
        opt = SparseSGD(t, lr=0.05) if kind == "sgd" else SparseAdam(t, lr=1e-3, mode=kind)
        t.accumulate_grad(torch.from_numpy(ids).to(DEV), torch.from_numpy(grad).to(DEV))
        opt.step()
        np.testing.assert_array_equal(t.weight.cpu().numpy(), f[key], err_msg=kind)


@pytest.mark.parametrize("kind", ["dedup", "sgd", "lazy_adam", "keras_adam"])
def test_one_call_sparse_entry_points_match_two_call(kind, rng):
    """rs_embedding_bwd_dedup / rs_apply_sgd / rs_apply_lazy_adam / rs_apply_keras_dense_adam
    (SURVEY §8(b) names) are bit-identical to rs_sort_ids + dedup / apply (+ dense sweep)."""
    card = [50, 3, 4000, 700]
    so_np = np.concatenate([[0], np.cumsum(card)]).astype(np.int64)
    V, D, B = int(so_np[-1]), 48, 3000
    ids = np.stack([rng.integers(0, c, B) for c in card], 1).astype(np.int64)
    g = rng.standard_normal((B * 4, D)).astype(np.float32)
    so = torch.from_numpy(so_np).to(DEV)
    idt, gt = torch.from_numpy(ids).to(DEV), torch.from_numpy(g).to(DEV)
    st = L.stream_ptr(torch.device(DEV))
    n = ids.size
    ws = torch.empty(L.lib().rs_sparse_workspace_size(n, D), dtype=torch.uint8, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    prm = L.AdamParams(1e-2, 0.9, 0.999, 0.1, 0.001, 1e-7)
    if kind == "dedup":
        ur = torch.empty(n, dtype=torch.int32, device=DEV)
        ug = torch.empty(n, D, device=DEV)
        nu = torch.zeros(1, dtype=torch.int32, device=DEV)
        L.call("rs_embedding_bwd_dedup", L.ptr(idt), 1, n, L.ptr(so), 4, V, L.ptr(gt), D, L.ptr(ur),
               L.ptr(ug), L.ptr(nu), L.ptr(err), L.ptr(ws), ws.numel(), st)
        u = int(nu.item())
        s = SortedIds(idt, V, so)
        w2 = torch.empty(L.lib().rs_dedup_workspace_size(n, D), dtype=torch.uint8, device=DEV)
        ur2 = torch.empty(n, dtype=torch.int32, device=DEV)
        ug2 = torch.empty(n, D, device=DEV)
        L.call("rs_embedding_dedup_grad", L.ptr(s.rows), L.ptr(s.pos), n, L.ptr(gt), D, V,
               L.ptr(ur2), L.ptr(ug2), L.ptr(w2), w2.numel(), st)
        assert u == int(s.n_unique.item())
        assert torch.equal(ur[:u], ur2[:u]) and torch.equal(ug[:u], ug2[:u])
        return
    tabs = [torch.from_numpy(rng.standard_normal((V, D)).astype(np.float32)).to(DEV)]
    tabs.append(tabs[0].clone())
    ms = [torch.full((V, D), 0.01, device=DEV) for _ in range(2)]
    vs = [torch.full((V, D), 0.02, device=DEV) for _ in range(2)]
    bms = [torch.zeros((V + 31) // 32, dtype=torch.int32, device=DEV) for _ in range(2)]
    if kind == "sgd":
        L.call("rs_apply_sgd", L.ptr(tabs[0]), V, D, L.ptr(idt), 1, n, L.ptr(so), 4, L.ptr(gt),
               0.01, L.ptr(err), L.ptr(ws), ws.numel(), st)
        opt, m, v, bm = L.RS_OPT_SGD, None, None, None
        prm = L.AdamParams(0.01, 0, 0, 0, 0, 0)
    elif kind == "lazy_adam":
        L.call("rs_apply_lazy_adam", L.ptr(tabs[0]), L.ptr(ms[0]), L.ptr(vs[0]), V, D, L.ptr(idt),
               1, n, L.ptr(so), 4, L.ptr(gt), prm, L.ptr(err), L.ptr(ws), ws.numel(), st)
        opt, m, v, bm = L.RS_OPT_LAZY_ADAM, ms[1], vs[1], None
    else:
        L.call("rs_apply_keras_dense_adam", L.ptr(tabs[0]), L.ptr(ms[0]), L.ptr(vs[0]), V, D,
               L.ptr(idt), 1, n, L.ptr(so), 4, L.ptr(gt), prm, L.ptr(bms[0]), L.ptr(err), L.ptr(ws),
               ws.numel(), st)
        opt, m, v, bm = L.RS_OPT_KERAS_ADAM, ms[1], vs[1], bms[1]
    s = SortedIds(idt, V, so)
    w2 = torch.empty(L.lib().rs_apply_workspace_size(n, D), dtype=torch.uint8, device=DEV)
    L.call("rs_embedding_apply", opt, L.ptr(tabs[1]), L.ptr(m), L.ptr(v), V, D, L.ptr(s.rows),
           L.ptr(s.pos), n, L.ptr(gt), prm, L.ptr(bm), L.ptr(w2), w2.numel(), st)
    if kind == "keras_adam":
        L.call("rs_keras_adam_dense_sweep", L.ptr(tabs[1]), L.ptr(m), L.ptr(v), V, D, prm,
               L.ptr(bm), st)
    assert torch.equal(tabs[0], tabs[1])
    if m is not None:
        assert torch.equal(ms[0], ms[1]) and torch.equal(vs[0], vs[1])


@pytest.mark.parametrize("dim", [128, 18, 7])
def test_keras_decay_zero_state_skip_bit_exact(dim, rng):
    """The Keras dense decay of rows without a gradient skips (m, v) chunks that are +0 / ±0 —
    the identity for any number of steps — without touching their weights. Against the oracle's
    Keras sparse apply with no gradient rows (oracle/embedding.py apply_keras_adam: the dense
    decay of every row), bit for bit (signed zeros compared as bits): rows of zero state, rows
    with m = -0 and w = -0 (not skipped: w becomes +0), m = +0 with v = -0, one nonzero element
    in a zero row, and ordinary rows — one dense sweep, and a deferred replay of 5 steps
    (rs_keras_adam_materialize) against 5 decays."""
    from recommender_amd.optim import keras_adam_coefficients as kc

    V = 64
    w = rng.standard_normal((V, dim)).astype(np.float32)
    m = (rng.standard_normal((V, dim)) * 1e-3).astype(np.float32)
    v = (rng.random((V, dim)) * 1e-4).astype(np.float32)
    m[:32] = 0.0
    v[:32] = 0.0
    m[4:8] = -0.0
    w[4:8, ::2] = -0.0
    w[8:12, 1::2] = -0.0  # +0 state: stays -0
    v[12:16] = -0.0
    m[16, dim // 2] = 1e-3  # one live element in a zero row
    v[16, dim // 2] = 1e-6
    bits = lambda a: a.view(np.uint32)  # noqa: E731
    none = np.zeros(0, np.int64)
    for steps in (1, 5):
        tw, tm, tv = (torch.from_numpy(a.copy()).to(DEV) for a in (w, m, v))
        ow, om, ov = w.copy(), m.copy(), v.copy()
        lr_hist = np.zeros(steps + 1, np.float32)
        for st in range(1, steps + 1):
            c = O.keras_adam_coefficients(st)
            lr_hist[st] = c["lr"]
            ow, om, ov = O.apply_keras_adam(ow, om, ov, none, np.zeros((0, dim), np.float32), c)
        if steps == 1:
            bm = torch.zeros((V + 31) // 32, dtype=torch.int32, device=DEV)
            L.call("rs_keras_adam_dense_sweep", L.ptr(tw), L.ptr(tm), L.ptr(tv), V, dim, kc(1),
                   L.ptr(bm), L.stream_ptr(DEV))
        else:
            last = torch.zeros(V, dtype=torch.int32, device=DEV)
            lr_t = torch.from_numpy(lr_hist).to(DEV)
            L.call("rs_keras_adam_materialize", L.ptr(tw), L.ptr(tm), L.ptr(tv), L.ptr(last), V,
                   dim, L.ptr(lr_t), steps, kc(steps), L.stream_ptr(DEV))
        torch.cuda.synchronize()
        for got, ref in ((tw, ow), (tm, om), (tv, ov)):
            np.testing.assert_array_equal(bits(got.cpu().numpy()), bits(ref.astype(np.float32)))
        assert (bits(ow[4:8, ::2]) == 0).all()  # -0 w under a -0 m: +0, as the formula gives


@pytest.mark.parametrize("V,dim,n", [(2, 8, 540_000), (100, 8, 30_000), (2048, 8, 5000),
                                     (64, 256, 3000), (20, 16, 1), (7, 4, 0)])
@pytest.mark.parametrize("id_dtype", [np.int32, np.int64])
def test_grad_dense_small_vs_float64(V, dim, n, id_dtype, rng):
    """rs_embedding_grad_dense_small (PinSage year / genre tables densified for a sync-free
    Keras Adam step): equals the float64 segmented sum within fp32 summation error (its order
    is fixed — per-block LDS lanes, then blocks — not position order), deterministic across
    calls, OOB ids skipped and flagged."""
    from recommender_amd.optim import densify_grad

    t = Embedding(V, dim, device=DEV)
    ids = rng.integers(0, V, n).astype(id_dtype)
    if V == 2:  # the genre table: two live rows take every entry
        ids = (rng.random(n) < 0.3).astype(id_dtype)
    rows = rng.standard_normal((n, dim)).astype(np.float32)
    ref = np.zeros((V, dim))
    np.add.at(ref, ids.astype(np.int64), rows.astype(np.float64))
    gi, gr = torch.from_numpy(ids).to(DEV), torch.from_numpy(rows).to(DEV)
    got = densify_grad(t, gi, gr)
    again = densify_grad(t, gi, gr)
    assert torch.equal(got, again)
    cnt = np.maximum(np.bincount(ids.astype(np.int64), minlength=V), 1)[:, None]
    bound = 1e-5 * (np.abs(ref) + np.sqrt(cnt) * 4.0)  # fp32 sum error ~ sqrt(count)·|row|·eps
    assert (np.abs(got.cpu().numpy() - ref) <= bound).all()
    assert not t.oob_detected()
    if n:
        bad = gi.clone()
        bad[n // 2] = V  # out of range: skipped, flagged
        d = densify_grad(t, bad, gr)
        assert t.oob_detected()
        ref2 = ref.copy()
        ref2[ids[n // 2]] -= rows[n // 2]
        assert (np.abs(d.cpu().numpy() - ref2) <= bound + 1e-5 * np.abs(rows[n // 2]).max()).all()


@pytest.mark.parametrize("dim", [18, 128])
@pytest.mark.parametrize("frac", [0.12, 0.0, 1.0])
def test_masked_sort_dense_grad(dim, frac, rng):
    """densify_grad with a position mask (DIEN's padded history steps): the masked sort gives the
    left-out positions the sentinel key without flagging them, and rs_embedding_grad_dense writes
    each kept row's segment sum in place, bit-exact against the oracle's tiled order on the kept
    positions (left-out ids as out-of-range), every other row 0; the unmasked densify equals the
    same oracle over all positions."""
    from recommender_amd.optim import densify_grad

    V, n = 63_001, 40 * 32 + 7
    ids = zipf_ids(rng, n, V).astype(np.int64)
    ids[rng.random(n) < 0.3] = 0  # a padding row shared by many positions
    keep = rng.random(n) < frac
    g = rng.standard_normal((n, dim)).astype(np.float32)
    t = Embedding(V, dim, device=DEV)
    dense = densify_grad(t, torch.from_numpy(ids).to(DEV), torch.from_numpy(g).to(DEV),
                         valid=torch.from_numpy(keep.astype(np.uint8)).to(DEV))
    assert int(t.err_flag.item()) == 0  # left-out positions are not out-of-range ids
    sr, sp, _ = O.sort_ids(np.where(keep, ids, -1), V)
    ref = np.zeros((V, dim), np.float32)
    rr, rg = O.segment_sum_tiled(sr, sp, g, V)
    ref[rr.astype(np.int64)] = rg
    np.testing.assert_array_equal(dense.cpu().numpy(), ref)
    full = densify_grad(t, torch.from_numpy(ids).to(DEV), torch.from_numpy(g).to(DEV))
    sr, sp, _ = O.sort_ids(ids, V)
    ref = np.zeros((V, dim), np.float32)
    rr, rg = O.segment_sum_tiled(sr, sp, g, V)
    ref[rr.astype(np.int64)] = rg
    np.testing.assert_array_equal(full.cpu().numpy(), ref)
