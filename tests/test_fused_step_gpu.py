"""The one-kernel production DLRM step (functional.dlrm_fused_train_forward /
rs_dlrm_train_step_fwd_unit: forward, mean BCE, G, table gradient rows and the MLP chains' batch
reductions in one pass) against the autograd path over the same kernels (TrainStep
fused_step=False), and against the CPU oracle on a small slab (oracle/check_dlrm.py; the
north-star size is tests/test_northstar_gpu.py)."""
import numpy as np
import pytest
import torch

from oracle.check_dlrm import checked_dlrm_sgd_step
from recommender_amd.ctr.layers import MLP
from recommender_amd.ctr.train import TrainStep, build_model
from recommender_amd.synthetic import criteo_batch, criteo_cardinalities
from tests.conftest import assert_close_rel

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture
def factored_any_batch():
    old = MLP.factored_min_batch
    MLP.factored_min_batch = 0
    yield
    MLP.factored_min_batch = old


def _model(cards, seed, bottom, top):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return build_model("DLRM", bottom[-1], sum(cards), 26, 13, torch.device(DEV),
                       slot_cardinalities=cards, bottom=bottom, top=top, generator=g)


@pytest.mark.parametrize("reduction", ["mean", "sum"])
@pytest.mark.parametrize("bottom,top", [([64, 128], [64, 32, 1]), ([512, 256, 128], [512, 256, 1]),
                                        ([512, 256, 64], [512, 256, 1])])
def test_fused_step_matches_autograd_path(factored_any_batch, reduction, bottom, top):
    cards = criteo_cardinalities(300_000, 26)
    rng = np.random.default_rng(11)
    batches = []
    for _ in range(3):
        cat, dn, lb = criteo_batch(rng, 2048, cards)
        batches.append(tuple(torch.from_numpy(x).to(DEV) for x in (cat, dn, lb)))
    runs = []
    for fused in (True, False):
        m = _model(cards, 3, bottom, top)
        st = TrainStep(m, "sgd", lr=0.05, loss_reduction=reduction, defer_sparse_join=True,
                       fused_step=fused)
        assert st.fused_step_ready(batches[0]) == fused
        losses, preds = [], []
        for b in batches:
            losses.append(float(st(b)))
            preds.append(st.last_pred.reshape(-1).clone())
        m.embedding_layer.wait_update()
        torch.cuda.synchronize()
        runs.append((m, losses, preds))
    (mf, lf, pf), (ma, la, pa) = runs
    for a, b in zip(lf, la):
        assert abs(a - b) <= 1e-5 * abs(b), (lf, la)
    for a, b in zip(pf, pa):
        assert_close_rel(a.cpu().numpy(), b.cpu().numpy(), 1e-5, 1e-3, "predictions")
    pa_ = dict(ma.named_parameters())
    for n, p in mf.named_parameters():
        if n.endswith("grad_handle"):
            continue
        # three SGD steps from one init: compare the parameter CHANGE. Both are fp32 batch sums
        # with cancellation (2048 examples, other orders): 1e-4 relative with a floor of 5% of
        # the tensor's largest change; the float64-oracle bound checks are
        # test_fused_step_vs_oracle_small_slab and tests/test_northstar_gpu.py
        ref = pa_[n].detach()
        init = dict(_model(cards, 3, bottom, top).named_parameters())[n].detach()
        d_f, d_a = (p.detach() - init).cpu().numpy(), (ref - init).cpu().numpy()
        assert_close_rel(d_f, d_a, 1e-4, np.abs(d_a).max() * 5e-2 + 1e-30, n)
    w0 = _model(cards, 3, bottom, top).embedding_layer.weight
    d_f = (mf.embedding_layer.weight - w0)
    d_a = (ma.embedding_layer.weight - w0)
    touched = (d_a != 0).any(1)
    assert int(touched.sum()) > 1000
    assert_close_rel(d_f[touched].cpu().numpy(), d_a[touched].cpu().numpy(), 1e-4,
                     float(d_a.abs().max()) * 5e-2, "table change")


def test_fused_step_vs_oracle_small_slab(factored_any_batch):
    """oracle/check_dlrm.py on the fused step: loss / logits 1e-5, grad rows 1e-5 of their bound,
    touched rows bit-exact against the oracle apply of the kernel's rows (two steps)."""
    cards = criteo_cardinalities(200_000, 26)
    m = _model(cards, 4, [128, 64, 128], [128, 64, 1])
    st = TrainStep(m, "sgd", lr=0.05, fused=True, defer_sparse_join=True)
    rng = np.random.default_rng(4)
    for _ in range(2):
        cat, dn, lb = criteo_batch(rng, 1024, cards)
        assert st.fused_step_ready(tuple(torch.from_numpy(x).to(DEV) for x in (cat, dn, lb)))
        r = checked_dlrm_sgd_step(m, st, cat, dn, lb, 0.05)
        print(r)


@pytest.mark.parametrize("fused_step", [True, False])
def test_prefetched_sort_bit_identical(factored_any_batch, fused_step):
    """TrainStep.prefetch (the next batch's sort queued one step ahead on its own stream) gives
    bit-identical parameters and table to plain steps; a batch whose ids change in place after
    the prefetch is sorted again (the stale sort is dropped)."""
    cards = criteo_cardinalities(300_000, 26)
    rng = np.random.default_rng(12)
    batches = []
    for _ in range(4):
        cat, dn, lb = criteo_batch(rng, 2048, cards)
        batches.append(tuple(torch.from_numpy(x).to(DEV) for x in (cat, dn, lb)))
    repl = torch.from_numpy(criteo_batch(rng, 2048, cards)[0]).to(DEV)
    runs = []
    for pre in (False, True):
        m = _model(cards, 5, [512, 256, 128], [512, 256, 1])
        st = TrainStep(m, "sgd", lr=0.05, defer_sparse_join=True, fused_step=fused_step)
        bs = [tuple(t.clone() for t in b) for b in batches]
        for i, b in enumerate(bs):
            if pre and i + 1 < len(bs):
                st.prefetch(bs[i + 1])
            if i == 2:  # batch 2 was prefetched during step 1: change its ids in place now
                b[0].copy_(repl)
            st(b)
        m.embedding_layer.wait_update()
        torch.cuda.synchronize()
        assert not m.embedding_layer._prefetched
        runs.append(m)
    a, b = runs
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        assert torch.equal(p, q), n
    assert torch.equal(a.embedding_layer.weight, b.embedding_layer.weight)


@pytest.mark.parametrize("fused_step", [True, False])
def test_keras_adam_deferred_decay_bit_exact(factored_any_batch, fused_step):
    """SparseAdam(mode='keras', defer_decay=True): per-row replay of the dense decay when a row
    is next read, then materialize() — table, m and v BIT-identical to the per-step dense sweep
    (rs_keras_adam_dense_sweep) over 5 steps of batches touching different rows (lags 1..4), on
    the fused one-kernel step and on the autograd path; reading without presort raises."""
    cards = criteo_cardinalities(50_000, 26)
    rng = np.random.default_rng(21)
    batches = []
    for _ in range(5):
        cat, dn, lb = criteo_batch(rng, 1024, cards)
        batches.append(tuple(torch.from_numpy(x).to(DEV) for x in (cat, dn, lb)))
    runs = []
    for defer in (False, True):
        m = _model(cards, 6, [128, 64, 128], [128, 64, 1])
        st = TrainStep(m, "keras_adam", lr=1e-2, defer_sparse_join=True, fused_step=fused_step,
                       defer_decay=defer)
        assert st.fused_step_ready(batches[0]) == fused_step
        for b in batches:
            st(b)
        emb = m.embedding_layer
        if defer:
            with pytest.raises(RuntimeError):
                emb.wait_update()
            st.opt_sparse.materialize()
            assert int(st.opt_sparse.last[id(emb)].min()) == 5
        emb.wait_update()
        torch.cuda.synchronize()
        mm, vv, _ = st.opt_sparse._slots(emb)
        runs.append((emb.weight.clone(), mm.clone(), vv.clone(),
                     [p.detach().clone() for p in m.parameters()]))
    (w0, m0, v0, p0), (w1, m1, v1, p1) = runs
    assert torch.equal(w0, w1) and torch.equal(m0, m1) and torch.equal(v0, v1)
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)
    # not vacuous: thousands of rows were touched, most of them in only some of the steps, so
    # their skipped steps were replayed (by the next touch's catch-up or by materialize)
    assert int((m0 != 0).any(1).sum()) > 2000


@pytest.mark.parametrize("bottom,top", [([512, 256, 128], [512, 256, 1]), ([128, 64, 128], [128, 64, 1])])
def test_dense_tail_bit_identical(factored_any_batch, bottom, top):
    """rs_dlrm_dense_tail (the MLP gradients, the SGD update and the next step's compositions in
    six grouped launches) against chain_param_grads + torch.optim.SGD + the forward's own
    compositions: parameters, gradients, predictions and table bit-identical over 3 steps."""
    cards = criteo_cardinalities(300_000, 26)
    rng = np.random.default_rng(21)
    batches = []
    for _ in range(3):
        cat, dn, lb = criteo_batch(rng, 2048, cards)
        batches.append(tuple(torch.from_numpy(x).to(DEV) for x in (cat, dn, lb)))
    runs = []
    for tail in (True, False):
        m = _model(cards, 6, bottom, top)
        st = TrainStep(m, "sgd", lr=0.05, defer_sparse_join=True)
        st.dense_tail = tail
        preds, grads = [], None
        for b in batches:
            st(b)
            preds.append(st.last_pred.clone())
            grads = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
        m.embedding_layer.wait_update()
        torch.cuda.synchronize()
        runs.append((m, preds, grads))
    (mt, pt, gt), (mr, pr, gr) = runs
    for a, b in zip(pt, pr):
        assert torch.equal(a, b)
    assert gt.keys() == gr.keys() and len(gt) == 12
    for n in gt:
        assert torch.equal(gt[n], gr[n]), n
    for (n, p), q in zip(mt.named_parameters(), mr.parameters()):
        assert torch.equal(p, q), n
    assert torch.equal(mt.embedding_layer.weight, mr.embedding_layer.weight)


def test_keras_deferred_decay_presort_without_step(factored_any_batch):
    """A presort whose step never runs (a forward-only call under grad) must not make its rows
    skip that step's Keras decay: steps 1, 2, a forward-only call on a batch with other rows,
    step 3, then materialize() — table / m / v bit-identical to the per-step dense sweep."""
    cards = criteo_cardinalities(50_000, 26)
    rng = np.random.default_rng(23)
    batches = [tuple(torch.from_numpy(x).to(DEV) for x in criteo_batch(rng, 1024, cards))
               for _ in range(4)]
    runs = []
    for defer in (False, True):
        m = _model(cards, 6, [128, 64, 128], [128, 64, 1])
        st = TrainStep(m, "keras_adam", lr=1e-2, defer_sparse_join=True, defer_decay=defer)
        st(batches[0])
        st(batches[1])
        if defer:  # the forward alone: presort + catch-up of batch 3's rows, no apply
            cat = batches[3][0]
            m.embedding_layer.presort(cat.reshape(-1, 26).contiguous())
        st(batches[2])
        emb = m.embedding_layer
        if defer:
            st.opt_sparse.materialize()
        emb.wait_update_raw()
        torch.cuda.synchronize()
        mm, vv, _ = st.opt_sparse._slots(emb)
        runs.append((emb.weight.clone(), mm.clone(), vv.clone()))
    (w0, m0, v0), (w1, m1, v1) = runs
    assert torch.equal(m0, m1) and torch.equal(v0, v1)
    assert torch.equal(w0, w1)
