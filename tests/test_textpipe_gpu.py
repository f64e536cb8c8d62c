"""GPU parity for the Ali-CCP and Amazon (DIEN) text pipelines against
oracle/textpipe.py on synthetic text: joined rows, vocabulary sizes and ids, encoded ids and
labels bit-exact (ids in first-appearance order on both sides); DIEN negatives checked for range,
the item → cat mapping, determinism under a seed and rough uniformity (the draw stream itself is
Philox, not NumPy's: parity unpinned for the draws, see oracle/textpipe.py)."""
import numpy as np
import pytest
import torch

from oracle import textpipe as O
from recommender_amd.data import AliCCPVocab, DienVocab, aliccp_join, subsample_impressions
from tests.textpipe_text import make_aliccp, make_amazon

pytestmark = pytest.mark.gpu


def _oracle_ids(rows, vocab):
    ids, lab = O.aliccp_encode(rows, vocab)
    return ids, lab


@pytest.mark.parametrize("n_skel,n_common", [(600, 40), (3000, 150), (1, 1)])
def test_aliccp_pipeline_matches_oracle(rng, n_skel, n_common):
    sk, cm = make_aliccp(rng, n_skel, n_common)
    sk_t, cm_t = make_aliccp(rng, 400, n_common)
    rows = O.aliccp_join(sk, cm)
    vocab = O.aliccp_vocab(rows)
    g_rows = aliccp_join(sk.encode(), cm.encode())
    assert g_rows.n == len(rows)
    v = AliCCPVocab.build(g_rows)
    assert v.sizes == [len(m) for m in vocab]
    feats, lab = v.encode(g_rows)
    ids, rl = _oracle_ids(rows, vocab)
    got = torch.cat([feats[c] for c in O.ALICCP_COLUMNS], 1).cpu().numpy()
    np.testing.assert_array_equal(got, ids)
    np.testing.assert_array_equal(lab.cpu().numpy(), rl)
    # the test split is encoded with the train vocabulary (process_test)
    rows_t = O.aliccp_join(sk_t, cm)
    ft, lt = v.encode(aliccp_join(sk_t.encode(), cm.encode()))
    it, rlt = _oracle_ids(rows_t, vocab)
    np.testing.assert_array_equal(torch.cat([ft[c] for c in O.ALICCP_COLUMNS], 1).cpu().numpy(), it)
    np.testing.assert_array_equal(lt.cpu().numpy(), rlt)
    if n_skel >= 600:
        assert sum(v.sizes) > 20 and (ids == 0).any()


def test_aliccp_unknown_common_id_raises(rng):
    sk, cm = make_aliccp(rng, 50, 5)
    with pytest.raises(KeyError):
        aliccp_join((sk + "z,1,0,nope,0,\n").encode(), cm.encode())


def test_subsample_matches_reference_loop(rng):
    lab = np.stack([rng.random(1000) < 0.2, rng.random(1000) < 0.1], 1).astype(np.int32)
    keep, nc = [], 0
    for i, (c, _) in enumerate(lab):  # esmm/tfrecord_io.py:53-59
        if c == 0:
            nc += 1
        if c == 0 and nc % 5 != 0:
            continue
        keep.append(i)
    got = subsample_impressions(torch.from_numpy(lab).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got, keep)


@pytest.mark.parametrize("maxlen,trailing", [(100, True), (7, False)])
def test_dien_pipeline_matches_oracle(rng, maxlen, trailing):
    train = make_amazon(rng, 600, trailing_newline=trailing)
    test = make_amazon(rng, 200, unseen_items=15)
    items, cats, i2c = O.dien_vocab(train)
    v = DienVocab.build(train.encode())
    assert v.n_item_ids == len(items) and v.n_cat_ids == len(cats)
    np.testing.assert_array_equal(v.cat_of_item.cpu().numpy(), O.dien_cat_of_item(items, cats, i2c))
    for text in (train, test):
        feats, lab = v.encode(text.encode(), maxlen=maxlen)
        rf, rl = O.dien_encode(text, items, cats, maxlen)
        for k in rf:
            np.testing.assert_array_equal(feats[k].cpu().numpy(), rf[k], err_msg=k)
        np.testing.assert_array_equal(lab.cpu().numpy(), rl)
    assert (rf["target_item"] == items["unk"]).any() or (rf["pos_his_item"] == items["unk"]).any()


def test_dien_negatives(rng):
    train = make_amazon(rng, 800)
    items, cats, i2c = O.dien_vocab(train)
    coi = O.dien_cat_of_item(items, cats, i2c)
    v = DienVocab.build(train.encode())
    f1, _ = v.encode(train.encode(), 100, sample_negative=True, seed=4)
    f2, _ = v.encode(train.encode(), 100, sample_negative=True, seed=4)
    f3, _ = v.encode(train.encode(), 100, sample_negative=True, seed=5)
    ni, nc = f1["neg_his_item"].cpu().numpy(), f1["neg_his_cat"].cpu().numpy()
    assert ni.min() >= 1 and ni.max() <= len(items) - 1  # randint(1, len(item_vocab))
    np.testing.assert_array_equal(nc, coi[ni])
    assert torch.equal(f1["neg_his_item"], f2["neg_his_item"])
    assert not torch.equal(f1["neg_his_item"], f3["neg_his_item"])
    counts = np.bincount(ni.ravel(), minlength=len(items))[1:]
    expect = ni.size / (len(items) - 1)
    assert np.abs(counts - expect).max() < 6 * np.sqrt(expect)


def test_dien_unknown_cat_raises(rng):
    train = make_amazon(rng, 100)
    v = DienVocab.build(train.encode())
    with pytest.raises(KeyError):
        v.encode(("1\tu\tI1\tNEWCAT\tI2\tC0\n").encode())
