"""GPU parity of the EGES pair pipeline (rs_eges_walks, rs_skipgram_pairs,
rs_log_uniform_sample, rs_csr_weight_prefix) against oracle/eges.py — bit-exact ids."""
import numpy as np
import pytest
import torch

from oracle import eges as O
from recommender_amd.eges.sampler import EGESPairSampler
from tests.eges_graph import make_graph

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def graph():
    return make_graph(np.random.default_rng(11))


def sampler(graph, **kw):
    indptr, indices, w = graph
    return EGESPairSampler(indptr, indices, w, 300, device=DEV, **kw)


def test_weight_prefix_bit_exact(graph):
    s = sampler(graph)
    ref = O.weight_prefix(graph[0], graph[2])
    assert np.array_equal(s.cumw.cpu().numpy(), ref)


@pytest.mark.parametrize("n_walks,length,base,step", [(257, 10, 0, 0), (64, 3, 1000, 7),
                                                     (1, 0, 5, 2)])
def test_walks_bit_exact(graph, n_walks, length, base, step):
    s = sampler(graph, walk_length=length)
    tr = s.walks(n_walks, step, walk_base=base).cpu().numpy()
    ref = O.weighted_walks(graph[0], graph[1], O.weight_prefix(graph[0], graph[2]), 300, base,
                           n_walks, length, s.seed, step)
    assert np.array_equal(tr, ref)
    assert (tr == -1).any() or length < 3  # the isolated items produce dead ends


@pytest.mark.parametrize("window", [1, 5])
def test_skipgrams_bit_exact(graph, window):
    s = sampler(graph, window=window)
    tr = s.walks(300, 3)
    tgt, ctx = s.skipgrams(tr)
    rt, rc = O.skipgram_pairs(tr.cpu().numpy(), window)
    assert np.array_equal(tgt.cpu().numpy(), rt) and np.array_equal(ctx.cpu().numpy(), rc)


def test_skipgrams_empty(graph):
    s = sampler(graph)
    tgt, ctx = s.skipgrams(torch.full((4, 11), -1, dtype=torch.int32, device=DEV))
    assert tgt.numel() == 0 and ctx.numel() == 0


@pytest.mark.parametrize("n,ns,base", [(500, 5, 0), (33, 20, 12345)])
def test_negatives_bit_exact(graph, n, ns, base):
    s = sampler(graph, num_ns=ns)
    out = s.negatives(n, 9, pair_base=base).cpu().numpy()
    ref = O.log_uniform_sample(O.log_uniform_cdf(300), base, n, ns, s.seed, 9)
    assert np.array_equal(out, ref)
    assert int(s.err.item()) == 0


def test_stream_batches(graph):
    rng = np.random.default_rng(0)
    cat, brand = rng.integers(0, 9, 300), rng.integers(0, 13, 300)
    s = sampler(graph, item2cat=cat, item2brand=brand, walks_per_refill=64)
    t, c, b, ctx, lab = s.next_batch(1000)
    assert t.shape == (1000, 1) and ctx.shape == (1000, 6) and lab.shape == (1000, 6)
    # the stream = refills concatenated: rebuild refill 0.. from the oracle
    cumw = O.weight_prefix(graph[0], graph[2])
    cdf = O.log_uniform_cdf(300)
    tg, cx = [], []
    for r in range(s.refills):
        tr = O.weighted_walks(graph[0], graph[1], cumw, 300, 0, 64, 10, s.seed, r)
        a, bb = O.skipgram_pairs(tr, 5)
        neg = O.log_uniform_sample(cdf, 0, a.size, 5, s.seed, r)
        tg.append(a)
        cx.append(np.concatenate([bb[:, None], neg], 1))
    tg, cx = np.concatenate(tg)[:1000], np.concatenate(cx)[:1000]
    assert np.array_equal(t[:, 0].cpu().numpy(), tg) and np.array_equal(ctx.cpu().numpy(), cx)
    assert np.array_equal(c[:, 0].cpu().numpy(), cat[tg]) and np.array_equal(b[:, 0].cpu().numpy(), brand[tg])
    assert float(lab[:, 0].min()) == 1.0 and float(lab[:, 1:].abs().max()) == 0.0


@pytest.mark.parametrize("model_type", ["BGE", "EGES"])
def test_train_cli_on_device_pairs(model_type, capsys):
    from recommender_amd.eges.train import main

    main(["--model_type", model_type, "--steps", "3", "--n_items", "2000",
          "--train_batch_size", "256"])
    assert "examples/s" in capsys.readouterr().out
