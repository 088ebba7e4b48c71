"""Accumulator policy and fit() routing of the device loops (GPU).

* hot relations at large batches: the pipelined runner's int32x2 relation
  sums and the two-launch runner's relation copies stay exact where int16
  fields would wrap; both equal fp32 sums of the same integer contributions;
* a hub entity whose per-batch count would wrap a 16-bit field: auto mode
  picks fp32 sums; forcing packed sums trips the run-time check, which
  device_optim reads before any post_epoch callback;
* PairwiseStochasticTrainer(device_loop=True) with labelled negatives or a
  sampler the device cannot mirror trains on the per-batch path (identical
  parameters to device_loop=False);
* the reference's post-fit outputs: neighbours accumulate over fits, the
  labelled-negatives branch writes no files (skge/base.py:1348-1386).
"""
import numpy as np
import pytest
import torch

from test_gpu_device_loop import make_kg

pytestmark = pytest.mark.gpu


def _dominant_kg(n_ent, n_rel, T, frac, seed=0):
    """Unique triples where relation 0 holds about `frac` of them."""
    rs = np.random.RandomState(seed)
    seen, out = set(), []
    while len(out) < T:
        s, o = int(rs.randint(n_ent)), int(rs.randint(n_ent))
        p = 0 if rs.rand() < frac else int(rs.randint(1, n_rel))
        if (s, o, p) not in seen:
            seen.add((s, o, p))
            out.append((s, o, p))
    return np.array(out, dtype=np.int32)


def _train(trip, n_ent, n_rel, d, nb, epochs=1, seed=7, margin=2.0, **kw):
    import skge_amd as S
    from skge_amd.device import DeviceKG, EpochRunner
    np.random.seed(seed)
    m = S.TransE((n_ent, n_ent, n_rel), d)
    m.add_hyperparam("margin", margin)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
    kg = DeviceKG(trip, m.device)
    r = EpochRunner(m, upd, kg, nbatches=nb, seed=3, **kw)
    r.run(epochs)
    r.synchronize()
    out = (m.E.data.cpu().numpy().copy(), m.R.data.cpu().numpy().copy(),
           int(r.nviol_total.item()), r)
    return out


@pytest.mark.parametrize("pipelined", [True, False])
def test_dominant_relation_large_batch_exact(pipelined):
    """Relation 0 holds ~60% of 30000 triples; one batch of 15000 positives
    puts ~9000 of them on one relation row (count ~36000 > 32767)."""
    trip = _dominant_kg(4000, 9, 30000, 0.6)
    E1, R1, v1, r1 = _train(trip, 4000, 9, 64, 2, pipelined=pipelined)
    assert r1.packed and r1.pipelined == pipelined
    if pipelined:
        assert r1.rel_w32
    else:
        assert r1.accR.replicas >= 2
    E2, R2, v2, r2 = _train(trip, 4000, 9, 64, 2, pipelined=False, force_f32=True)
    assert not r2.packed
    assert v1 > 0 and abs(v1 - v2) <= 2
    np.testing.assert_allclose(R1, R2, atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(E1, E2, atol=1e-5, rtol=1e-5)


def test_dominant_relation_pipelined_equals_two_launch_bitwise():
    trip = _dominant_kg(3000, 7, 24000, 0.7, seed=4)
    a = _train(trip, 3000, 7, 200, 2, epochs=2, pipelined=True)
    b = _train(trip, 3000, 7, 200, 2, epochs=2, pipelined=False)
    assert a[3].packed and b[3].packed and b[3].accR.replicas >= 2
    assert a[2] == b[2] > 0
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def _hub_kg():
    o = np.arange(1, 12001)
    return np.stack([np.zeros_like(o), o, o % 5], axis=1).astype(np.int32)


def test_hub_entity_auto_picks_fp32():
    trip = _hub_kg()
    E, R, v, r = _train(trip, 13000, 5, 32, 1, margin=1e9)
    assert not r.packed
    assert r.count_bound > 32767
    assert v == 2 * len(trip)   # every pair violates a 1e9 margin


def test_forced_packed_overflow_stops_fit_before_callbacks(monkeypatch):
    import skge_amd as S
    from skge_amd import _lib as L
    from skge_amd import device as D
    trip = _hub_kg()
    np.random.seed(1)
    m = S.TransE((13000, 13000, 5), 32)
    seen = []
    orig = D.make_runner

    def forced(model, updaters, kg, nbatches, **kw):
        kw.pop("runner", None)
        return D.EpochRunner(model, updaters, kg, nbatches, packed=True,
                             seed=kw["seed"], ntries=kw["ntries"], nviol_total=kw["nviol_total"])

    monkeypatch.setattr(D, "make_runner", forced)
    xs = [tuple(x) for x in trip.tolist()]
    tr = S.PairwiseStochasticTrainer(m, nbatches=1, max_epochs=3, margin=1e9, device_loop=True,
                                     file_grad=None, file_embed=None,
                                     samplef=S.RandomModeSampler(1, [0, 1], xs, (13000, 13000, 5)).sample,
                                     post_epoch=[lambda t: seen.append(t.epoch) or True])
    with pytest.raises(L.SkgeError, match="32767"):
        tr.fit(xs, [1] * len(trip))
    assert seen == []
    monkeypatch.setattr(D, "make_runner", orig)
    L.lib().skge_device_error(L.stream_ptr(), 1)   # leave the global error word clean


def _fit_pair(xs, ys, device_loop, sampler=None, nb=4, epochs=2):
    import skge_amd as S
    np.random.seed(42)
    m = S.TransE((60, 60, 4), 16)
    kw = {}
    if sampler is not None:
        kw["samplef"] = sampler(m).sample
    np.random.seed(5)   # the host shuffles / samplers draw the same stream either way
    tr = S.PairwiseStochasticTrainer(m, nbatches=nb, max_epochs=epochs, margin=1.0,
                                     device_loop=device_loop, file_grad=None, file_embed=None,
                                     **kw)
    tr.fit(xs, ys)
    return np.asarray(m.E).copy(), np.asarray(m.R).copy()


def test_device_loop_labelled_negatives_use_per_batch_path():
    trip, tset = make_kg(60, 4, 400, seed=3)
    pos = [tuple(x) for x in trip[:200].tolist()]
    rs = np.random.RandomState(9)
    neg = [(int(rs.randint(60)), o, p) for (s, o, p) in pos]
    xs, ys = pos + neg, [1] * len(pos) + [-1] * len(neg)
    with pytest.warns(UserWarning, match="labelled negatives"):
        a = _fit_pair(xs, ys, True)
    b = _fit_pair(xs, ys, False)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_device_loop_other_sampler_uses_per_batch_path():
    import skge_amd as S
    trip, _ = make_kg(60, 4, 300, seed=4)
    xs = [tuple(x) for x in trip.tolist()]
    mk = lambda m: S.RandomModeSampler(2, [0, 1], xs, (60, 60, 4))   # two negatives per mode
    with pytest.warns(UserWarning, match="RandomModeSampler"):
        a = _fit_pair(xs, [1] * len(xs), True, sampler=mk)
    b = _fit_pair(xs, [1] * len(xs), False, sampler=mk)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_device_loop_reference_sampler_runs_on_device():
    import skge_amd as S
    trip, _ = make_kg(60, 4, 300, seed=4)
    xs = [tuple(x) for x in trip.tolist()]
    np.random.seed(42)
    m = S.TransE((60, 60, 4), 16)
    smp = S.RandomModeSampler(1, [0, 1], xs, (60, 60, 4))
    tr = S.PairwiseStochasticTrainer(m, nbatches=4, max_epochs=1, margin=1.0, device_loop=True,
                                     samplef=smp.sample, file_grad=None, file_embed=None)
    tr.fit(xs, [1] * len(xs))
    assert tr._runner is not None and tr._on_device


def test_device_loop_without_sampler_or_with_foreign_set_stays_on_host():
    """samplef None is the reference's labelled-negatives branch and a sampler
    over another triple set rejects other draws: neither runs the device loop."""
    import skge_amd as S
    trip, _ = make_kg(60, 4, 300, seed=4)
    xs = [tuple(x) for x in trip.tolist()]
    np.random.seed(42)
    m = S.TransE((60, 60, 4), 16)
    tr = S.PairwiseStochasticTrainer(m, nbatches=4, max_epochs=1, margin=1.0, device_loop=True,
                                     file_grad=None, file_embed=None)
    from skge_amd.device import device_sampler_args
    ok, _, why = device_sampler_args(tr, xs, [1] * len(xs))
    assert not ok and "samplef is None" in why
    smp = S.RandomModeSampler(1, [0, 1], xs[:-5], (60, 60, 4))   # train minus five triples
    tr2 = S.PairwiseStochasticTrainer(m, nbatches=4, max_epochs=1, margin=1.0, device_loop=True,
                                      samplef=smp.sample, file_grad=None, file_embed=None)
    ok, _, why = device_sampler_args(tr2, xs, [1] * len(xs))
    assert not ok and "rejection set" in why


def test_device_loop_file_grad_auto_keeps_counters(tmp_path):
    """device_runner='auto' with file_grad set: the pair loop, whose per-row
    counters fill the #(violations) / #(updates) columns."""
    import skge_amd as S
    from skge_amd.device import PairLoopRunner
    trip, _ = make_kg(60, 4, 300, seed=4)
    xs = [tuple(x) for x in trip.tolist()]
    for mk in (lambda: S.TransE((60, 60, 4), 16), lambda: S.HolE((60, 60, 4), 16)):
        np.random.seed(42)
        m = mk()
        tr = S.PairwiseStochasticTrainer(m, nbatches=4, max_epochs=1, margin=1.0, device_loop=True,
                                         samplef=S.RandomModeSampler(1, [0, 1], xs, (60, 60, 4)).sample,
                                         file_grad=str(tmp_path / "g.txt"), file_embed=None)
        tr.fit(xs, [1] * len(xs))
        assert isinstance(tr._runner, PairLoopRunner)
        assert int(np.asarray(m.E.updateCounts).sum()) > 0


def test_outputs_neighbours_accumulate_and_branches(tmp_path):
    import skge_amd as S
    trip, _ = make_kg(50, 3, 200, seed=6)
    xs = [tuple(x) for x in trip.tolist()]
    np.random.seed(42)
    m = S.TransE((50, 50, 3), 8)
    smp = S.RandomModeSampler(1, [0, 1], xs, (50, 50, 3))
    fg = tmp_path / "g.txt"
    tr = S.PairwiseStochasticTrainer(m, nbatches=2, max_epochs=1, margin=1.0, samplef=smp.sample,
                                     file_grad=str(fg), file_embed=None)
    tr.fit(xs, [1] * len(xs))
    tr.fit(xs, [1] * len(xs))
    deg = np.bincount(trip[:, 0], minlength=50) + np.bincount(trip[:, 1], minlength=50)
    np.testing.assert_array_equal(m.E.neighbours, 2 * deg)   # base.py:1364-1367, per fit
    # labelled-negatives branch (samplef None): the reference writes nothing
    fg2 = tmp_path / "g2.txt"
    fe2 = tmp_path / "e2.txt"
    m2 = S.TransE((50, 50, 3), 8)
    tr2 = S.PairwiseStochasticTrainer(m2, nbatches=2, max_epochs=1, margin=1.0,
                                      file_grad=str(fg2), file_embed=str(fe2))
    neg = [(s, (o + 1) % 50, p) for (s, o, p) in xs]
    tr2.fit(xs + neg, [1] * len(xs) + [-1] * len(neg))
    for f in (tr2.file_gradients, tr2.file_embeddings, tr2.pickle_file_embeddings):
        f.flush()
    assert fg2.read_text() == "" and fe2.read_text() == ""
    assert m2.E.neighbours is None


def test_pair_runner_holds_captured_buffers():
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    np.random.seed(3)
    m = S.HolE((80, 80, 4), 16)
    m.add_hyperparam("margin", 0.2)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
    trip, _ = make_kg(80, 4, 400, seed=2)
    kg = DeviceKG(trip, m.device)
    r = PairLoopRunner(m, upd, kg, nbatches=4, seed=1)
    old = m.accumulator("E").touched
    m.accumulator("E").ensure_slots(old.numel() * 8)   # a later, larger per-batch call
    assert m.accumulator("E").touched is not old
    assert any(t[2] is old for t in r._captured if isinstance(t, tuple))
    r.run(1)
    r.synchronize()
    assert np.isfinite(np.asarray(m.E)).all()


def test_sharded_dominant_relation_uses_copies_and_matches_runner():
    """The row-sharded runner's packed relation sums are all-reduced over the
    ranks' batches: a relation holding half the triples gets accumulator
    copies, and G = 1 still equals the two-launch device runner bit for bit."""
    import skge_amd as S
    from skge_amd.shard import ShardedRunner
    trip = _dominant_kg(3000, 7, 24000, 0.7, seed=4)
    E1, R1, v1, r1 = _train(trip, 3000, 7, 64, 2, epochs=2, seed=11, pipelined=False)
    assert r1.packed and r1.accR.replicas >= 2
    np.random.seed(11)
    m = S.TransE((3000, 3000, 7), 64)
    sr = ShardedRunner(3000, m.E.data.clone(), m.R.data.clone(),
                       torch.as_tensor(trip, device=m.device), 2, lr=0.1, margin=2.0, seed=3)
    assert sr.accR.replicas >= 2
    sr.run(2)
    sr.synchronize()
    assert int(sr.nviol_total.item()) == v1 > 0
    assert np.array_equal(sr.E.data.cpu().numpy(), E1)
    assert np.array_equal(sr.R.data.cpu().numpy(), R1)
