"""GPU parity for the Criteo ingestion kernels vs oracle/criteo.py on
synthetic TSV text: vocabulary ids and the encoded categorical ids bit-exact, dense log(x + 1)
within 1 ulp, labels exact; edge cases: empty and negative ints, empty tokens (imputation),
'\\r\\n' lines, no trailing newline, C26 tokens equal to C1 tokens (distinct keys)."""
import numpy as np
import pytest
import torch

from oracle import criteo as O
from recommender_amd.data import CriteoVocab
from tests.criteo_text import make_tsv

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n_lines,trailing", [(400, False), (1500, True), (1, True)])
def test_ingestion_matches_oracle(rng, n_lines, trailing):
    train = make_tsv(rng, n_lines, trailing_newline=trailing)
    test = make_tsv(rng, 300, trailing_newline=not trailing)
    vocab = O.build_vocab(train)
    v = CriteoVocab.build(train.encode())
    assert v.size == len(vocab)
    for text in (train, test):
        cat, dense, label = v.encode(text.encode())
        rc, rd, rl = O.encode(text, vocab)
        np.testing.assert_array_equal(cat.cpu().numpy(), rc)
        np.testing.assert_array_equal(label.cpu().numpy(), rl)
        np.testing.assert_allclose(dense.cpu().numpy(), rd, rtol=2e-7, atol=0)
    if n_lines >= 400:
        assert len(vocab) > 5 and (rc == 0).any()


def test_malformed_line_raises(rng):
    bad = make_tsv(rng, 10) + "\n1\t2\t3\n"
    with pytest.raises(ValueError):
        CriteoVocab.build(bad.encode())
