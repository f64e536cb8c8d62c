"""CPU checks of the Ali-CCP / Amazon text-pipeline oracle (esmm/process_public_dataset.py,
dien/util.py, dien/data_loader.py restatements) on hand-written lines."""
import numpy as np

from oracle import textpipe as O
from tests.textpipe_text import make_aliccp, make_amazon

S2, S3, S1 = "\x02", "\x03", "\x01"


def _f(k, v):
    return f"{k}{S2}{v}{S3}1.0"


def test_aliccp_join_and_vocab_by_hand():
    common = "u1,2," + S1.join([_f("101", "7"), _f("121", "5")]) + "\n"
    lines = []
    for k in range(13):  # '101' overridden by the common value 7; '205' seen 13 times
        lines.append(f"s{k},0,0,u1,2," + S1.join([_f("101", "9"), _f("205", "x"), _f("205", "y")]))
    lines.append("sX,0,1,u1,1," + _f("205", "z"))  # dropped (click 0, purchase 1)
    lines.append("sY,1,1,u1,1," + _f("216", "q") + S1 + "853")  # trailing key, no value
    rows = O.aliccp_join("\n".join(lines) + "\n", common)
    assert len(rows) == 14 and rows[-1][:2] == (1, 1)
    c = O.ALICCP_COLUMNS
    assert rows[0][2][c.index("101")] == "7" and rows[0][2][c.index("205")] == "y"
    assert rows[-1][2][c.index("853")] is None and rows[-1][2][c.index("216")] == "q"
    vocab = O.aliccp_vocab(rows)
    # '7' in 101 and '5' in 121: 14 rows ≥ 12; 'y' in 205: 13 rows; 'q': once
    assert vocab[c.index("101")] == {"7": 1} and vocab[c.index("205")] == {"y": 1}
    assert vocab[c.index("216")] == {}
    ids, lab = O.aliccp_encode(rows, vocab)
    assert ids.shape == (14, 18) and (ids[:, c.index("101")] == 1).all()
    assert (ids[:, c.index("124")] == 0).all()  # absent → '0' → OOV 0
    assert lab[-1].tolist() == [1, 1]


def test_aliccp_threshold_is_twelve():
    common = "u,1," + _f("301", "a") + "\n"
    rows = O.aliccp_join("".join(f"s,0,0,u,0,{_f('508', 'v')}\n" for _ in range(11)), common)
    assert O.aliccp_vocab(rows)[O.ALICCP_COLUMNS.index("508")] == {}  # seen 11: count 10
    rows = O.aliccp_join("".join(f"s,0,0,u,0,{_f('508', 'v')}\n" for _ in range(12)), common)
    assert O.aliccp_vocab(rows)[O.ALICCP_COLUMNS.index("508")] == {"v": 1}


def test_dien_vocab_and_padding_by_hand():
    text = ("1\tu\tA\tc1\tB" + S2 + "C" + S2 + "A\tc2" + S2 + "c1" + S2 + "c3\n"
            "0\tu\tD\tc2\tB\tc9\n")
    items, cats, i2c = O.dien_vocab(text)
    assert items == {"A": 1, "B": 2, "C": 3, "D": 4, "mask": 0, "unk": 5}
    assert cats == {"c1": 1, "c2": 2, "c3": 3, "c9": 4, "mask": 0, "unk": 5}
    assert i2c["B"] == "c9" and i2c["A"] == "c3" and i2c["C"] == "c1"  # the last pair wins
    feats, lab = O.dien_encode(text + "1\tu\tZ\tc2\tZ" + S2 + "B\tc2" + S2 + "c9\n", items, cats, 2)
    np.testing.assert_array_equal(feats["pos_his_item"], [[3, 1], [2, 0], [5, 2]])  # pre-trunc
    np.testing.assert_array_equal(feats["pos_his_cat"], [[1, 3], [4, 0], [2, 4]])
    assert feats["target_item"][2, 0] == 5 and lab[:, 0].tolist() == [1, 0, 1]
    coi = O.dien_cat_of_item(items, cats, i2c)
    assert coi.tolist() == [0, 3, 4, 1, 2, 5]


def test_generators(rng):
    sk, cm = make_aliccp(rng, 100, 10)
    rows = O.aliccp_join(sk, cm)
    assert 80 < len(rows) <= 100
    text = make_amazon(rng, 50)
    items, cats, _ = O.dien_vocab(text)
    feats, _ = O.dien_encode(text, items, cats, 100)
    assert feats["pos_his_item"].shape == (50, 100)
