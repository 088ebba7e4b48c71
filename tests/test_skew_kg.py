"""bench.make_zipf_kg (SURVEY 8(d)'s skew variant): the KG the skewed GPU
tests and `bench.py --skew zipf` use -- reproducible, unique triples, ids in
range, and actually skewed."""
import numpy as np


def test_zipf_kg_unique_in_range_skewed_and_reproducible():
    from bench import make_zipf_kg
    k = make_zipf_kg(2000, 11, 12000, seed=3)
    assert k.shape == (12000, 3) and k.dtype == np.int32
    assert k[:, :2].min() >= 0 and k[:, :2].max() < 2000
    assert k[:, 2].min() >= 0 and k[:, 2].max() < 11
    assert len({tuple(t) for t in k.tolist()}) == 12000
    counts = np.bincount(np.concatenate([k[:, 0], k[:, 1]]), minlength=2000)
    assert counts.max() > 50 * counts.mean() / 5          # hot rows
    assert (counts == 0).sum() > 100                      # and a cold tail
    assert np.array_equal(k, make_zipf_kg(2000, 11, 12000, seed=3))
    assert not np.array_equal(k, make_zipf_kg(2000, 11, 12000, seed=4))
