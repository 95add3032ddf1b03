"""The NumPy restatement of the device sampler (tests/philox_np.py): Philox4x32-10
against the published Random123 known-answer vectors, and the draw's statistics."""
import numpy as np

from philox_np import draw, philox4x32_10, sample_key

# Random123 kat_vectors, "philox4x32 10": counter (4 words), key (2 words) -> output
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


def test_philox_known_answers():
    for ctr, key, want in KAT:
        got = philox4x32_10(np.array(ctr, dtype=np.uint32), key)
        assert tuple(int(x) for x in got) == want, (ctr, [hex(int(x)) for x in got])
    # vectorised over a batch of counters = row by row
    ctrs = np.array([k[0] for k in KAT[:1]] * 3, dtype=np.uint32)
    assert np.array_equal(philox4x32_10(ctrs, KAT[0][1])[2], np.array(KAT[0][2], dtype=np.uint32))


def test_sample_key_depends_on_seed_and_alpha():
    ks = {sample_key(s, a) for s in (0, 1, 9) for a in (3.0, 30.0)}
    assert len(ks) == 6 and all(0 <= k < 2 ** 64 for k in ks)


def test_draw_statistics():
    idx, nz = draw(sample_key(7, 10.0), 3, 4096, 1000, 5)
    assert idx.min() >= 0 and idx.max() < 1000
    assert 0.0 <= nz["t"].min() and nz["t"].max() < 1.0
    allz = np.concatenate([nz[k].ravel() for k in ("z_next", "x0", "z_d", "z_metric")])
    assert abs(allz.mean()) < 0.03 and abs(allz.std() - 1.0) < 0.03
    idx2, _ = draw(sample_key(7, 10.0), 4, 4096, 1000, 5)
    assert not np.array_equal(idx, idx2)
