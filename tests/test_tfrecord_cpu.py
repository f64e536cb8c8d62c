"""CPU tests of the Criteo TFRecord path (ctr/tfrecord_io.py:39-96): the oracle's CRC32C known
answer, the product writer's bytes equal the oracle's, and the host framing index (the C-ABI
host entry, no GPU needed) on good and corrupt files."""
import numpy as np
import pytest

from oracle import tfrecord as OT


def _arrays(rng, n):
    ints = np.log1p(rng.geometric(0.01, (n, 13))).astype(np.float32)
    cats = rng.integers(0, 1_000_000, (n, 26)).astype(np.int64)
    cats[0, 0] = (1 << 40) + 3  # wide ids survive
    labels = (rng.random(n) < 0.25).astype(np.int64)
    return ints, cats, labels


def test_crc32c_known_answer():
    assert OT.crc32c(b"123456789") == 0xE3069283  # RFC 3720 B.4 / iSCSI check value
    assert OT.crc32c(b"") == 0


def test_writer_matches_oracle_and_round_trips(rng):
    from recommender_amd.data.tfrecord import encode_records, index_records

    ints, cats, labels = _arrays(rng, 40)
    mine = encode_records(ints, cats, labels)
    assert mine == OT.write_records(ints, cats, labels)
    a, b, c = OT.read_records(mine)
    np.testing.assert_array_equal(a, ints)
    np.testing.assert_array_equal(b, cats)
    np.testing.assert_array_equal(c, labels)
    offs, lens = index_records(np.frombuffer(mine, np.uint8))
    assert offs.size == 40 and offs[0] == 0
    np.testing.assert_array_equal(offs[1:], offs[:-1] + 16 + lens[:-1])


def test_index_rejects_corrupt_framing(rng):
    from recommender_amd import _lib as L
    from recommender_amd.data.tfrecord import index_records

    ints, cats, labels = _arrays(rng, 3)
    good = bytearray(OT.write_records(ints, cats, labels))
    bad = good.copy()
    bad[8] ^= 0x01  # the first length CRC
    with pytest.raises(L.RecsysError):
        index_records(np.frombuffer(bytes(bad), np.uint8))
    index_records(np.frombuffer(bytes(bad), np.uint8), verify_crc=False)  # unchecked: framing ok
    with pytest.raises(L.RecsysError):
        index_records(np.frombuffer(bytes(good[:-3]), np.uint8))  # truncated


@pytest.mark.parametrize("extra", [0, 1, 2, 3, 4])
def test_index_rejects_file_cut_after_a_record_header(rng, extra):
    """A file cut just after a record's 12-byte header (+0..4 bytes): the length and its CRC are
    intact, so only the bounds check stands between the index and an out-of-range record."""
    from recommender_amd import _lib as L
    from recommender_amd.data.tfrecord import index_records

    ints, cats, labels = _arrays(rng, 2)
    good = bytes(OT.write_records(ints, cats, labels))
    offs, lens = index_records(np.frombuffer(good, np.uint8))
    cut = good[: int(offs[1]) + 12 + extra]
    for verify in (True, False):
        with pytest.raises(L.RecsysError):
            index_records(np.frombuffer(cut, np.uint8), verify_crc=verify)


@pytest.mark.parametrize("n", [0, 1, 5, 257])
def test_encode_records_fixed_equals_per_record(n):
    """The column-wise batch encoder (one template record tiled, data bytes and payload CRCs
    filled per column) writes the per-record encoder's bytes exactly, labels 0..127 and a
    fallback for other label widths."""
    from recommender_amd.data.tfrecord import encode_records, encode_records_fixed

    r = np.random.default_rng(n)
    ints = r.standard_normal((n, 13)).astype(np.float32)
    cats = r.integers(0, 1 << 40, (n, 26))
    for labs in (r.integers(0, 2, n), np.full(n, 127), np.full(n, 300)):
        assert encode_records_fixed(ints, cats, labs) == encode_records(ints, cats, labs)
