"""Host-side accumulator policy of the TransE device loops (CPU): the bound
that decides exact packed int16x4 entity sums vs fp32 sums, and the number
of relation accumulator copies the two-launch runner needs.  Counts follow
the kernels' occurrence counting (skge/transe.py:73-136 via
csrc/skge_pipeline.hip): s and o of a positive <= 3 each, an accepted
corruption 1."""
import types

import numpy as np
import torch

from skge_amd.device import PACKED_MAX, packed_count_bound, relation_replicas


def _kg(trip):
    return types.SimpleNamespace(trip=torch.as_tensor(np.asarray(trip, dtype=np.int32)))


def test_bound_uniform_wn18_shape_fits_even_at_two_batches():
    rs = np.random.RandomState(0)
    trip = np.stack([rs.randint(40943, size=141442), rs.randint(40943, size=141442),
                     rs.randint(18, size=141442)], axis=1)
    kg = _kg(trip)
    occ = np.bincount(trip[:, 0], minlength=40943) + np.bincount(trip[:, 1], minlength=40943)
    for batch in (1414, 70721):
        b = packed_count_bound(kg, 40943, batch)
        assert b >= 3 * occ.max()
        assert b <= PACKED_MAX
    # WN18-shaped relations at nb=2: 4 * ~7.9k positives per relation fits one copy
    assert relation_replicas(kg, 18, 1414) == 1


def test_bound_hub_entity_forces_fp32():
    # entity 0 is the subject of 12000 triples: 3 * 12000 > 32767 at nb=1
    n = 20000
    o = np.arange(1, 12001)
    trip = np.stack([np.zeros_like(o), o, o % 7], axis=1)
    kg = _kg(trip)
    assert packed_count_bound(kg, n, len(trip)) > PACKED_MAX
    # small batches bound the hub's per-batch count instead
    assert packed_count_bound(kg, n, 1000) <= PACKED_MAX


def test_corruption_term_tiny_graph():
    # 10 entities, one batch of 40000: ~8000 occurrences per row (24000
    # counted) and corruptions concentrate (lambda = 8000 per row)
    rs = np.random.RandomState(1)
    trip = np.stack([rs.randint(10, size=40000), rs.randint(10, size=40000),
                     rs.randint(3, size=40000)], axis=1)
    kg = _kg(trip)
    assert packed_count_bound(kg, 10, 40000) > PACKED_MAX   # -> fp32 sums
    # a batch of 4000 is a uniform sample of the 40000 triples: ~400 of a row's
    # ~4000 subject (and object) occurrences land in it, bounded by the
    # binomial tail, not by the whole-KG count (round 4)
    b = packed_count_bound(kg, 10, 4000)
    assert 3 * 2 * 400 + 800 < b <= PACKED_MAX


def test_bound_skewed_kg_batch_sample():
    """Zipf-skewed WN18-sized KG (bench.make_zipf_kg): the hottest row is in
    ~16% of the triples.  Its per-batch share, not its whole-KG count, bounds
    the packed fields, so batches up to ~14k positives keep packed sums; at
    nb = 2 the hot row's ~11k per-batch occurrences (x3) do not fit."""
    from bench import make_zipf_kg
    trip = make_zipf_kg(40943, 18, 141442, seed=3)
    kg = _kg(trip)
    occ = (np.bincount(trip[:, 0], minlength=40943) + np.bincount(trip[:, 1], minlength=40943))
    for batch in (1414, 7072, 14144):
        b = packed_count_bound(kg, 40943, batch)
        assert b <= PACKED_MAX, batch
        assert b >= 3 * occ.max() * batch / len(trip)   # above the hot row's mean share
    assert packed_count_bound(kg, 40943, 70721) > PACKED_MAX


def test_relation_replicas_dominant_relation():
    rs = np.random.RandomState(2)
    T = 141442
    p = np.where(rs.rand(T) < 0.5, 0, rs.randint(1, 18, size=T))   # relation 0: half the triples
    trip = np.stack([rs.randint(40943, size=T), rs.randint(40943, size=T), p], axis=1)
    kg = _kg(trip)
    assert relation_replicas(kg, 18, 1414) == 1          # 4 * 1414 fits
    r = relation_replicas(kg, 18, 70721)                   # ~35k positives of relation 0
    mu = 70721 / r * 0.5                                   # relation 0's expected share of a copy
    assert r == 8 and 4 * (mu + 12 * np.sqrt(mu) + 40) <= PACKED_MAX
    assert relation_replicas(kg, 18, 70721, max_reps=4) == 0


def test_relation_replicas_config5_shape():
    # |R| = 10k uniform, 10k triples each (T = 100M scaled by 1/100 here, the
    # same per-relation share): ~13 positives of a relation per 131072-batch
    rs = np.random.RandomState(3)
    T = 1000000
    trip = np.stack([rs.randint(500000, size=T), rs.randint(500000, size=T),
                     rs.randint(10000, size=T)], axis=1)
    assert relation_replicas(_kg(trip), 10000, 131072) == 1
    assert relation_replicas(_kg(trip), 10000, 131072, ranks=8) == 1   # the sharded union batch


def test_padded_width_whole_lines(monkeypatch):
    """d % 4 != 0 tables run on zero-padded copies: whole 128-B lines (32
    floats) when that costs <= 30% more row bytes, else the next quad."""
    from skge_amd.device import padded_width
    monkeypatch.delenv("SKGE_PIPE_PAD_TO", raising=False)
    assert padded_width(50) == 64       # BASELINE configs[0]: 256-B rows
    assert padded_width(30) == 32
    assert padded_width(13) == 16       # 32 would be 2.5x the row
    assert padded_width(97) == 100      # 128 would be +32%
    assert padded_width(99) == 128      # +29%
    monkeypatch.setenv("SKGE_PIPE_PAD_TO", "4")
    assert padded_width(50) == 52       # the round-3 width (A/B switch)
