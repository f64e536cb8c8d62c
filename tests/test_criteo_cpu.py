"""CPU checks of the Criteo ingestion oracle (ctr/tfrecord_io.py restatement)."""
import numpy as np

from oracle import criteo as O
from tests.criteo_text import make_tsv


def test_oracle_semantics_by_hand():
    line = "\t".join(["1", "", "-3", "7"] + ["1"] * 10 + ["aa"] * 25 + [""]) + "\n"
    text = line * 11 + "\t".join(["0"] + ["0"] * 13 + ["bb"] + ["aa"] * 24 + ["aa"]) + "\n"
    vocab = O.build_vocab(text)
    # 'aa' seen 11*25 + 24 times, '<null:25>' 11 times, 'aa\n' once, 'bb' once
    assert vocab == {"aa": 0, "<null:25>": 1}
    cat, dense, label = O.encode(text, vocab)
    assert cat[0, 0] == 0 and cat[0, 25] == 1 and cat[-1, 0] == 0 and cat[-1, 25] == 0
    np.testing.assert_allclose(dense[0, :3], np.log(np.float32([1, 1, 8])))
    assert label[0] == 1 and label[-1] == 0


def test_generator_shapes(rng):
    text = make_tsv(rng, 50)
    cat, dense, label = O.encode(text, O.build_vocab(text))
    assert cat.shape == (50, 26) and dense.shape == (50, 13) and label.shape == (50,)
