"""Device pair loop (skge_pair_runner_*, GPU) for every model.

The runner draws the epoch's permutation and negatives on the device; the
same draws are exposed by skge_epoch_sample, so each test replays them on the
host the way PairwiseStochasticTrainer._process_batch builds its pairs
(skge/base.py:1394-1427: positive x, then its s-corrupted and o-corrupted
negatives, a negative missing after ntries draws dropping that pair,
skge/sample.py:41-46) and feeds them to model._pairwise_step on a twin model.
SGD keeps the comparison linear: only float-atomic summation order differs,
so |diff| <= 1e-5 + 1e-5 |want|; violation totals are compared exactly.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ATOL = RTOL = 1e-5


def make_kg(n_ent, n_rel, T, seed=0):
    rs = np.random.RandomState(seed)
    seen, out = set(), []
    while len(out) < T:
        t = (int(rs.randint(n_ent)), int(rs.randint(n_ent)), int(rs.randint(n_rel)))
        if t not in seen:
            seen.add(t)
            out.append(t)
    return out


def make_model(kind, sz, d):
    import skge_amd as S
    np.random.seed(42)
    if kind == "transe_l1":
        return S.TransE(sz, d, l1=True)
    if kind == "transe_l2":
        return S.TransE(sz, d, l1=False)
    if kind == "hole":
        return S.HolE(sz, d, rparam=0.05)
    return S.RESCAL(sz, d, rparam=0.05)


def host_pairs(rec, n1, start, count):
    pos, neg = [], []
    for j in range(start, start + count):
        s, o, p, a = (int(x) for x in rec[j])
        b = int(n1[j])
        if a >= 0:
            pos.append((s, o, p))
            neg.append((a, o, p))
        if b >= 0:
            pos.append((s, o, p))
            neg.append((s, b, p))
    return pos, neg


def replay(model, upd, kg, n_ent, nbatches, epochs, seed, ntries):
    from skge_amd.device import batch_sizes, epoch_records
    dev = model.device
    nv = torch.zeros(1, dtype=torch.int32, device=dev)
    total = 0
    for e in range(epochs):
        rec, n1 = epoch_records(kg, n_ent, seed, e, ntries)
        rec, n1 = rec.cpu().numpy(), n1.cpu().numpy()
        start = 0
        for c in batch_sizes(kg.T, nbatches):
            pos, neg = host_pairs(rec, n1, start, c)
            start += c
            if not pos:
                continue
            nv.zero_()
            model._pairwise_step(torch.tensor(pos, dtype=torch.int32, device=dev),
                                 torch.tensor(neg, dtype=torch.int32, device=dev), upd, nv)
            total += int(nv.item())
    return total


@pytest.mark.parametrize("kind,d,dense", [("transe_l1", 32, False), ("transe_l2", 24, False),
                                          ("hole", 32, False), ("rescal", 16, False),
                                          ("hole", 16, True), ("rescal", 8, True),
                                          ("hole", 100, False), ("hole", 200, False),
                                          ("hole", 30, False)])
def test_pair_loop_matches_host_replay(kind, d, dense, monkeypatch):
    import skge_amd as S
    # the per-positive HolE kernel with the explicit-pair kernel's direct
    # correlations (same arithmetic -> same margin decisions); its FFT form is
    # checked against this one in test_hole_fft_matches_direct
    monkeypatch.setenv("SKGE_HOLE_DIRECT", "1")
    from skge_amd.device import DeviceKG, PairLoopRunner
    if dense:   # 70% of all triples: many negatives not found in 3 draws -> skipped pairs
        n_ent, n_rel, T, ntries = 12, 2, 200, 3
    else:
        n_ent, n_rel, T, ntries = 300, 7, 2000, 100
    xs = make_kg(n_ent, n_rel, T)
    sz = (n_ent, n_ent, n_rel)
    nb, epochs, seed, margin = 7, 2, 11, 0.5
    a = make_model(kind, sz, d)
    b = make_model(kind, sz, d)
    for m in (a, b):
        m.add_hyperparam("margin", margin)
    upd_a = {pid: S.SGD(p, 0.05) for pid, p in a.params.items()}
    upd_b = {pid: S.SGD(p, 0.05) for pid, p in b.params.items()}
    kg = DeviceKG(xs, a.device)
    r = PairLoopRunner(a, upd_a, kg, nb, seed=seed, ntries=ntries)
    with torch.cuda.stream(r.stream):
        r.run(epochs)
    r.synchronize()
    want_nv = replay(b, upd_b, kg, n_ent, nb, epochs, seed, ntries)
    torch.cuda.synchronize()
    assert int(r.nviol_total.item()) == want_nv
    assert want_nv > 0
    for pid in a.params:
        np.testing.assert_allclose(a.params[pid].data.cpu().numpy(),
                                   b.params[pid].data.cpu().numpy(), rtol=RTOL, atol=ATOL,
                                   err_msg="%s %s" % (kind, pid))
    for acc in a._acc.values():   # accumulators drained after every batch
        assert int(acc.cnt.abs().sum().item()) == 0


def test_dense_kg_skips_pairs():
    """The dense case really exercises skipped pairs: some negatives are
    missing (-1) in the draws the runner uses."""
    from skge_amd.device import DeviceKG, epoch_records
    xs = make_kg(12, 2, 200)
    import skge_amd as S
    m = make_model("hole", (12, 12, 2), 16)
    kg = DeviceKG(xs, m.device)
    rec, n1 = epoch_records(kg, 12, 11, 0, 3)
    rec, n1 = rec.cpu().numpy(), n1.cpu().numpy()
    assert (rec[:, 3] < 0).sum() > 0 and (n1 < 0).sum() > 0
    assert (rec[:, 3] >= 0).sum() > 0
    # accepted negatives are never training triples
    known = set(xs)
    for (s, o, p, a), b in zip(rec.tolist(), n1.tolist()):
        assert a < 0 or (a, o, p) not in known
        assert b < 0 or (s, b, p) not in known
    assert sorted(map(tuple, rec[:, :3].tolist())) == sorted(xs)   # a permutation
    del S


def test_pair_loop_transe_agrees_with_epoch_runner():
    """TransE-L1 through the pair loop and through the fused two-launch
    runner (fp32 sums): same draws, same batches -> same parameters."""
    import skge_amd as S
    from skge_amd.device import DeviceKG, EpochRunner, PairLoopRunner
    n_ent, n_rel, T = 400, 9, 3000
    xs = make_kg(n_ent, n_rel, T)
    models = [make_model("transe_l1", (n_ent, n_ent, n_rel), 32) for _ in range(2)]
    runners = []
    for i, m in enumerate(models):
        m.add_hyperparam("margin", 1.0)
        upd = {pid: S.SGD(p, 0.05) for pid, p in m.params.items()}
        kg = DeviceKG(xs, m.device)
        if i == 0:
            r = PairLoopRunner(m, upd, kg, 10, seed=3)
        else:
            r = EpochRunner(m, upd, kg, 10, seed=3, force_f32=True, pipelined=False)
        with torch.cuda.stream(r.stream):
            r.run(2)
        r.synchronize()
        runners.append(r)
    assert int(runners[0].nviol_total.item()) == int(runners[1].nviol_total.item())
    for pid in ("E", "R"):
        np.testing.assert_allclose(models[0].params[pid].data.cpu().numpy(),
                                   models[1].params[pid].data.cpu().numpy(), rtol=RTOL,
                                   atol=ATOL, err_msg=pid)


@pytest.mark.parametrize("kind", ["hole", "rescal"])
def test_trainer_device_loop_any_model(kind):
    """PairwiseStochasticTrainer(device_loop=True) trains HolE / RESCAL with
    AdaGrad through the pair loop; callbacks see per-epoch violations."""
    import skge_amd as S
    n_ent, n_rel = 200, 5
    xs = make_kg(n_ent, n_rel, 1500)
    m = make_model(kind, (n_ent, n_ent, n_rel), 16)
    E0 = m.E.data.clone()
    seen = []
    tr = S.PairwiseStochasticTrainer(m, nbatches=10, max_epochs=3, learning_rate=0.1,
                                     margin=0.2, device_loop=True, device_runner="pairs",
                                     samplef=S.RandomModeSampler(1, [0, 1], xs,
                                                                 (n_ent, n_ent, n_rel)).sample,
                                     file_grad=None, file_embed=None,
                                     post_epoch=[lambda t: seen.append(t.nviolations) or True])
    tr.fit(xs, [1] * len(xs))
    assert len(seen) == 3 and all(v > 0 for v in seen)
    assert not torch.equal(E0, m.E.data)
    assert np.isfinite(m.E.data.cpu().numpy()).all()
    assert int(m.E.updateCounts.sum()) > 0


@pytest.mark.parametrize("d", [32, 200])
def test_hole_positive_kernel_matches_explicit_pairs(d, monkeypatch):
    """The HolE pair loop's positive kernel (k_hole_pos: both pairs of a
    positive per wave) against the explicit-pair kernels (SKGE_HOLE_PAIRS=1)
    on the same draws: equal violation totals (the scores use the same
    arithmetic), parameters within the fp32 tolerance."""
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    n_ent, n_rel, T = 300, 7, 2000
    xs = make_kg(n_ent, n_rel, T)
    out = []
    monkeypatch.setenv("SKGE_HOLE_DIRECT", "1")   # the explicit-pair kernel's arithmetic
    for pairs in ("0", "1"):
        monkeypatch.setenv("SKGE_HOLE_PAIRS", pairs)
        m = make_model("hole", (n_ent, n_ent, n_rel), d)
        m.add_hyperparam("margin", 0.5)
        upd = {pid: S.SGD(p, 0.05) for pid, p in m.params.items()}
        r = PairLoopRunner(m, upd, DeviceKG(xs, m.device), 7, seed=5)
        with torch.cuda.stream(r.stream):
            r.run(2)
        r.synchronize()
        out.append((int(r.nviol_total.item()),
                    {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()}))
    assert out[0][0] == out[1][0] > 0
    for pid in out[0][1]:
        np.testing.assert_allclose(out[0][1][pid], out[1][1][pid], rtol=RTOL, atol=ATOL,
                                   err_msg=pid)


@pytest.mark.parametrize("d", [16, 64])
def test_rescal_positive_path_matches_explicit_pairs(d, monkeypatch):
    """The RESCAL pair loop's deduplicated form (each positive once in the
    GEMMs and dW, both pairs per scatter wave) against the explicit pairs
    (SKGE_RESCAL_PAIRS=1) on the same draws: equal violation totals (the scores
    are the same per-item sums), parameters within the fp32 tolerance."""
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    n_ent, n_rel, T = 300, 7, 2000
    xs = make_kg(n_ent, n_rel, T)
    out = []
    for pairs in ("0", "1"):
        monkeypatch.setenv("SKGE_RESCAL_PAIRS", pairs)
        m = make_model("rescal", (n_ent, n_ent, n_rel), d)
        m.add_hyperparam("margin", 0.5)
        upd = {pid: S.SGD(p, 0.05) for pid, p in m.params.items()}
        r = PairLoopRunner(m, upd, DeviceKG(xs, m.device), 7, seed=5)
        with torch.cuda.stream(r.stream):
            r.run(2)
        r.synchronize()
        out.append((int(r.nviol_total.item()),
                    {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()}))
    assert out[0][0] == out[1][0] > 0
    for pid in out[0][1]:
        np.testing.assert_allclose(out[0][1][pid], out[1][1][pid], rtol=RTOL, atol=ATOL,
                                   err_msg=pid)


@pytest.mark.parametrize("kind,env", [("hole", "SKGE_HOLE_PAIRS"), ("rescal", "SKGE_RESCAL_PAIRS")])
def test_per_positive_paths_at_wn18_batch_geometry(kind, env, monkeypatch):
    """WN18's entity count, relation count, d=200 and batch size (1414
    positives, 10 batches): the per-positive kernels against the explicit-pair
    kernels on the same draws -- equal violation totals, parameters within the
    fp32 tolerance (SGD, margin 0.2 as in the reference's HolE/RESCAL runs)."""
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    n_ent, n_rel, T, nb = 40943, 18, 14140, 10
    xs = make_kg(n_ent, n_rel, T, seed=3)
    out = []
    monkeypatch.setenv("SKGE_HOLE_DIRECT", "1")   # the explicit-pair kernel's arithmetic
    for pairs in ("0", "1"):
        monkeypatch.setenv(env, pairs)
        m = make_model(kind, (n_ent, n_ent, n_rel), 200)
        m.add_hyperparam("margin", 0.2)
        upd = {pid: S.SGD(p, 0.1) for pid, p in m.params.items()}
        r = PairLoopRunner(m, upd, DeviceKG(xs, m.device), nb, seed=9)
        with torch.cuda.stream(r.stream):
            r.run(1)
        r.synchronize()
        out.append((int(r.nviol_total.item()),
                    {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()}))
    assert out[0][0] == out[1][0] > 0
    for pid in out[0][1]:
        np.testing.assert_allclose(out[0][1][pid], out[1][1][pid], rtol=RTOL, atol=ATOL,
                                   err_msg="%s %s" % (kind, pid))


def _hole_epochs(runner_cls, xs, n_ent, n_rel, d, nb, epochs, margin=0.2, seed=9, opt="sgd"):
    import skge_amd as S
    from skge_amd.device import DeviceKG
    m = make_model("hole", (n_ent, n_ent, n_rel), d)
    m.add_hyperparam("margin", margin)
    U = S.SGD if opt == "sgd" else S.AdaGrad
    upd = {pid: U(p, 0.1) for pid, p in m.params.items()}
    r = runner_cls(m, upd, DeviceKG(xs, m.device), nb, seed=seed)
    with torch.cuda.stream(r.stream):
        r.run(epochs)
    r.synchronize()
    return (int(r.nviol_total.item()), int(r.epoch_key.item()),
            {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()})


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb,epochs,opt", [
    (300, 7, 2000, 32, 7, 2, "sgd"),        # ragged remainder batch
    (40, 3, 1200, 200, 4, 2, "sgd"),        # tiny graph: most rows pending every batch
    (500, 5, 3000, 64, 10, 3, "adagrad"),   # AdaGrad state through the hand-off
    (40943, 18, 14140, 200, 10, 1, "sgd"),  # WN18 entity count, d, batch size
    (3000, 7, 14000, 32, 2, 2, "sgd"),  # 7000 positives per batch: 4 relation replicas
])
def test_hole_pipelined_runner_matches_pair_loop(n_ent, n_rel, T, d, nb, epochs, opt):
    """The pipelined HolE runner (launch g scores batch b while batch b-1's
    rows are applied beside it) against the two-launch device pair loop on
    the same draws: the same pairs and scores up to fp32 summation order, so
    violation totals agree (within a tie or two) and parameters within the
    fp32 tolerance (rparam 0.05: the relation rows' rout term included)."""
    from skge_amd.device import HolePipeRunner, PairLoopRunner
    xs = make_kg(n_ent, n_rel, T, seed=3)
    a = _hole_epochs(PairLoopRunner, xs, n_ent, n_rel, d, nb, epochs, opt=opt)
    b = _hole_epochs(HolePipeRunner, xs, n_ent, n_rel, d, nb, epochs, opt=opt)
    assert a[1] == b[1] == epochs
    assert a[0] > 0 and abs(a[0] - b[0]) <= 2, (a[0], b[0])
    for pid in a[2]:
        np.testing.assert_allclose(b[2][pid], a[2][pid], rtol=RTOL, atol=ATOL,
                                   err_msg="%s (%d, %d)" % (pid, a[0], b[0]))


def test_hole_pipelined_runner_relation_replicas_forced(monkeypatch):
    """Relation accumulator replicas (positive w adds into replica w % reps,
    every reader sums them in a fixed order) forced to 3 at a small batch:
    the same training as the pair loop up to fp32 summation order."""
    from skge_amd.device import HolePipeRunner, PairLoopRunner
    xs = make_kg(300, 7, 2000, seed=3)
    a = _hole_epochs(PairLoopRunner, xs, 300, 7, 32, 7, 2)
    monkeypatch.setenv("SKGE_HPIPE_RREPS", "3")
    b = _hole_epochs(HolePipeRunner, xs, 300, 7, 32, 7, 2)
    assert a[0] > 0 and abs(a[0] - b[0]) <= 2, (a[0], b[0])
    for pid in a[2]:
        np.testing.assert_allclose(b[2][pid], a[2][pid], rtol=RTOL, atol=ATOL, err_msg=pid)


def test_hole_pipelined_runner_profile_trains_like_run():
    """HolePipeRunner.profile() (the bench's per-launch timing: one eager
    epoch with events) trains exactly like run(1) on a twin model and returns
    one duration per launch."""
    import skge_amd as S
    from skge_amd.device import DeviceKG, HolePipeRunner
    xs = make_kg(300, 7, 2000, seed=3)
    outs = []
    for prof in (False, True):
        m = make_model("hole", (300, 300, 7), 32)
        m.add_hyperparam("margin", 0.2)
        upd = {pid: S.SGD(p, 0.1) for pid, p in m.params.items()}
        r = HolePipeRunner(m, upd, DeviceKG(xs, m.device), 7, seed=9)
        if prof:
            us, stats = r.profile()
            assert len(us) == r.nlaunches and (us > 0).all()
        else:
            r.run(1)
        r.synchronize()
        outs.append((int(r.nviol_total.item()),
                     {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()}))
    assert outs[0][0] > 0 and abs(outs[0][0] - outs[1][0]) <= 2   # float atomics: a tie or two
    for pid in outs[0][1]:
        np.testing.assert_allclose(outs[1][1][pid], outs[0][1][pid], rtol=RTOL, atol=ATOL)


def test_rescal_split_k_dw_matches_fused(monkeypatch):
    """RESCAL dW split over K (batches with >= 4 groups of 128 items per
    relation: partial tiles summed in split order by a finishing kernel)
    against the single fused dW kernel (SKGE_RESCAL_FORM=nosplit) on the same draws:
    equal violation totals, parameters within the fp32 tolerance (SGD)."""
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    n_ent, n_rel, T, nb, d = 3000, 3, 6000, 2, 40   # 3000 positives / batch: ~3000 items / relation
    xs = make_kg(n_ent, n_rel, T, seed=4)
    out = []
    for form in ("nosplit", ""):
        monkeypatch.setenv("SKGE_RESCAL_FORM", form)
        m = make_model("rescal", (n_ent, n_ent, n_rel), d)
        m.add_hyperparam("margin", 0.5)
        upd = {pid: S.SGD(p, 0.05) for pid, p in m.params.items()}
        r = PairLoopRunner(m, upd, DeviceKG(xs, m.device), nb, seed=5)
        with torch.cuda.stream(r.stream):
            r.run(2)
        r.synchronize()
        out.append((int(r.nviol_total.item()),
                    {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()}))
    assert out[0][0] == out[1][0] > 0
    for pid in out[0][1]:
        np.testing.assert_allclose(out[1][1][pid], out[0][1][pid], rtol=RTOL, atol=ATOL,
                                   err_msg=pid)


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb", [
    (300, 7, 2000, 32, 7),          # M = 16 = 4 x 4
    (300, 7, 2000, 24, 7),          # M = 12 = 4 x 3
    (300, 7, 2000, 40, 7),          # M = 20 = 4 x 5
    (300, 7, 2000, 60, 7),          # M = 30 = 2 x 3 x 5
    (300, 7, 2000, 28, 7),          # M = 14 = 2 x 7: no FFT plan, direct sums
    (300, 7, 2000, 4, 7),           # M = 2: one radix-2 stage, the middle pair only
    (300, 7, 2000, 8, 7),           # M = 4
    (300, 7, 2000, 240, 7),         # M = 120 = 4 x 2 x 3 x 5, 61 lanes of pairs
    (40943, 18, 14140, 200, 10),    # WN18 entity count, d = 200 (M = 100 = 4 x 5 x 5)
])
def test_hole_fft_matches_direct(n_ent, n_rel, T, d, nb, monkeypatch):
    """The per-positive HolE kernel with its correlations through the wave FFT
    (skge_hole_fft.h: Stockham radix 4/2/3/5 over M = d/2, real rows packed as
    complex, Hermitian sums for the scores) against the direct O(d^2) sums on
    the same draws.  The scores differ by fp32 rounding only, so the margin
    decisions agree but for a near-tie or two; parameters within the fp32
    tolerance (SGD, rparam 0.05) wherever the decisions agree."""
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    xs = make_kg(n_ent, n_rel, T, seed=6)
    out = []
    for direct in ("1", "0"):
        monkeypatch.setenv("SKGE_HOLE_DIRECT", direct)
        m = make_model("hole", (n_ent, n_ent, n_rel), d)
        m.add_hyperparam("margin", 0.2)
        upd = {pid: S.SGD(p, 0.1) for pid, p in m.params.items()}
        r = PairLoopRunner(m, upd, DeviceKG(xs, m.device), nb, seed=9)
        with torch.cuda.stream(r.stream):
            r.run(2 if n_ent < 1000 else 1)
        r.synchronize()
        out.append((int(r.nviol_total.item()),
                    {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()}))
    (va, pa), (vb, pb) = out
    assert va > 0 and abs(va - vb) <= 2, (va, vb)
    for pid in pa:
        close = np.abs(pb[pid] - pa[pid]) <= ATOL + RTOL * np.abs(pa[pid])
        if va == vb:
            assert close.all(), (pid, float(np.abs(pb[pid] - pa[pid]).max()))
        else:   # a flipped near-tie moves the rows of that one pair
            assert close.mean() > 0.999, (pid, close.mean())


@pytest.mark.parametrize("d", [32, 200])
def test_hole_explicit_pair_fft_matches_direct(d, monkeypatch):
    """The explicit-pair HolE kernel (the reference-protocol / per-batch path)
    in the frequency domain against its direct sums, through the pair loop's
    explicit-pair form (SKGE_HOLE_PAIRS=1) on the same draws."""
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    n_ent, n_rel, T = 300, 7, 2000
    xs = make_kg(n_ent, n_rel, T, seed=8)
    monkeypatch.setenv("SKGE_HOLE_PAIRS", "1")
    out = []
    for direct in ("1", "0"):
        monkeypatch.setenv("SKGE_HOLE_DIRECT", direct)
        m = make_model("hole", (n_ent, n_ent, n_rel), d)
        m.add_hyperparam("margin", 0.2)
        upd = {pid: S.SGD(p, 0.1) for pid, p in m.params.items()}
        r = PairLoopRunner(m, upd, DeviceKG(xs, m.device), 7, seed=2)
        with torch.cuda.stream(r.stream):
            r.run(2)
        r.synchronize()
        out.append((int(r.nviol_total.item()),
                    {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()}))
    (va, pa), (vb, pb) = out
    assert va > 0 and abs(va - vb) <= 2, (va, vb)
    for pid in pa:
        close = np.abs(pb[pid] - pa[pid]) <= ATOL + RTOL * np.abs(pa[pid])
        if va == vb:
            assert close.all(), (pid, float(np.abs(pb[pid] - pa[pid]).max()))
        else:
            assert close.mean() > 0.999, (pid, close.mean())


def test_hole_device_loop_auto_selects_pipelined_runner():
    import skge_amd as S
    from skge_amd.device import HolePipeRunner
    xs = make_kg(200, 5, 1500)
    m = make_model("hole", (200, 200, 5), 16)
    tr = S.PairwiseStochasticTrainer(m, nbatches=10, max_epochs=2, margin=0.2, device_loop=True,
                                     samplef=S.RandomModeSampler(1, [0, 1], xs, (200, 200, 5)).sample,
                                     file_grad=None, file_embed=None)
    tr.fit(xs, [1] * len(xs))
    assert isinstance(tr._runner, HolePipeRunner)
    assert np.isfinite(m.E.data.cpu().numpy()).all()


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb", [
    (300, 7, 2000, 16, 7),          # ragged remainder batch
    (40943, 18, 14140, 200, 10),    # WN18 entity / relation counts, d, batch size
])
def test_rescal_epoch_buckets_match_per_batch_buckets(n_ent, n_rel, T, d, nb, monkeypatch):
    """The RESCAL pair loop with every batch's relation buckets built once per
    epoch (three launches per epoch) against per-batch bucketing on the same
    draws: the buckets are the same stable order, so violation totals are
    equal and parameters agree to the entity sums' float-atomic rounding."""
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    xs = make_kg(n_ent, n_rel, T, seed=2)
    out = []
    for eb in ("0", "1"):
        monkeypatch.setenv("SKGE_RESCAL_EPOCH_BUCKETS", eb)
        m = make_model("rescal", (n_ent, n_ent, n_rel), d)
        m.add_hyperparam("margin", 0.2)
        # SGD keeps the comparison linear (AdaGrad turns rounding-level
        # differences of a near-zero first gradient into +-lr steps)
        upd = {pid: S.SGD(p, 0.1) for pid, p in m.params.items()}
        r = PairLoopRunner(m, upd, DeviceKG(xs, m.device), nb, seed=4)
        with torch.cuda.stream(r.stream):
            r.run(2)
        r.synchronize()
        out.append((int(r.nviol_total.item()),
                    {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()}))
    assert out[0][0] == out[1][0] > 0
    for pid in out[0][1]:
        np.testing.assert_allclose(out[1][1][pid], out[0][1][pid], rtol=RTOL, atol=ATOL,
                                   err_msg=pid)


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb,fsplit,order", [
    (300, 7, 2000, 16, 7, "1", "1"),          # ragged remainder batch
    (300, 7, 2000, 36, 3, "2", "0"),          # d % 4 == 0, two dW splits, dW grid first
    (300, 5, 2000, 30, 3, "1", "3"),          # d % 4 != 0, interleaved roles
    (40943, 18, 14140, 200, 10, "1", "1"),    # WN18 entity / relation counts, d, batch size
    (40943, 18, 14140, 200, 10, "1", "9"),    # interleave clamped to the grid
])
def test_rescal_fused_front_matches_unfused(n_ent, n_rel, T, d, nb, fsplit, order, monkeypatch):
    """The RESCAL pair loop's fused front (Linear: dW contraction and GEMMs in
    one launch, dW coefficients written with the epoch's buckets, the W step
    after the scatter) against the unfused kernels (SKGE_RESCAL_FORM=unfused) on the
    same draws: equal violation totals, parameters within the fp32 tolerance
    (the entity sums are float atomics in both)."""
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    xs = make_kg(n_ent, n_rel, T, seed=3)
    out = []
    for fused in ("unfused,", ""):
        monkeypatch.setenv("SKGE_RESCAL_FORM", "%sfsplit=%s,order=%s" % (fused, fsplit, order))
        m = make_model("rescal", (n_ent, n_ent, n_rel), d)
        m.add_hyperparam("margin", 0.2)
        upd = {pid: S.SGD(p, 0.1) for pid, p in m.params.items()}
        r = PairLoopRunner(m, upd, DeviceKG(xs, m.device), nb, seed=6)
        with torch.cuda.stream(r.stream):
            r.run(2)
        r.synchronize()
        out.append((int(r.nviol_total.item()),
                    {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()}))
    assert out[0][0] == out[1][0] > 0
    for pid in out[0][1]:
        np.testing.assert_allclose(out[1][1][pid], out[0][1][pid], rtol=RTOL, atol=ATOL,
                                   err_msg=pid)


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb,af", [
    (300, 7, 2000, 16, 7, "linear"),          # ragged remainder batch, fused front
    (300, 7, 2000, 30, 3, "sigmoid"),         # d % 4 != 0, unfused kernels (scores drive dW)
    (200, 3, 130, 24, 2, "linear"),           # batches of < 64 positives (padded blocks)
    (40943, 18, 14140, 200, 10, "linear"),    # WN18 entity / relation counts, d, batch size
    (40943, 18, 14140, 200, 10, "sigmoid"),
])
def test_rescal_dedup_gemm_rows_match_three_rows(n_ent, n_rel, T, d, nb, af, monkeypatch):
    """The RESCAL pair loop's deduplicated GEMM rows (W E_o once per (o, p) of a
    positive and its s-corrupted negative, E_s W once per (s, p) of a positive
    and its o-corrupted negative: 2 rows per positive and product instead of
    3) against three rows per positive (SKGE_RESCAL_FORM=nodedup) on the same draws:
    the scores are the same values, so violation totals are equal; dW sums
    its items in another bucket order, so parameters agree to fp32 rounding."""
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    xs = make_kg(n_ent, n_rel, T, seed=5)
    out = []
    for form in ("nodedup", ""):
        monkeypatch.setenv("SKGE_RESCAL_FORM", form)
        np.random.seed(42)
        m = S.RESCAL((n_ent, n_ent, n_rel), d, rparam=0.05, af=af)
        m.add_hyperparam("margin", 0.2)
        upd = {pid: S.SGD(p, 0.1) for pid, p in m.params.items()}
        r = PairLoopRunner(m, upd, DeviceKG(xs, m.device), nb, seed=7)
        with torch.cuda.stream(r.stream):
            r.run(2)
        r.synchronize()
        out.append((int(r.nviol_total.item()),
                    {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()}))
    assert out[0][0] == out[1][0] > 0
    for pid in out[0][1]:
        np.testing.assert_allclose(out[1][1][pid], out[0][1][pid], rtol=RTOL, atol=ATOL,
                                   err_msg=pid)


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb", [
    (300, 7, 2000, 16, 7),          # ragged remainder batch
    (300, 5, 2000, 30, 3),          # d % 4 != 0
    (3000, 3, 6000, 40, 2),         # >= 4 item groups per relation: split-K partial tiles
    (40943, 18, 14140, 200, 10),    # WN18 entity / relation counts, d, batch size
])
def test_rescal_combined_dw_matches_three_items(n_ent, n_rel, T, d, nb, monkeypatch):
    """The fused front's combined dW (a positive and its o-corrupted negative
    as ONE outer product E_s (x) (-(k0 + k1) E_o + E_o'), its s-corrupted
    negative as E_s' (x) E_o: two outer products per positive instead of
    three) against three items per positive (SKGE_RESCAL_FORM=dw3) on the same
    draws: equal violation totals, parameters within the fp32 tolerance."""
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    xs = make_kg(n_ent, n_rel, T, seed=9)
    out = []
    for form in ("dw3", ""):
        monkeypatch.setenv("SKGE_RESCAL_FORM", form)
        m = make_model("rescal", (n_ent, n_ent, n_rel), d)
        m.add_hyperparam("margin", 0.2)
        upd = {pid: S.SGD(p, 0.1) for pid, p in m.params.items()}
        r = PairLoopRunner(m, upd, DeviceKG(xs, m.device), nb, seed=8)
        with torch.cuda.stream(r.stream):
            r.run(2)
        r.synchronize()
        out.append((int(r.nviol_total.item()),
                    {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()}))
    assert out[0][0] == out[1][0] > 0
    for pid in out[0][1]:
        np.testing.assert_allclose(out[1][1][pid], out[0][1][pid], rtol=RTOL, atol=ATOL,
                                   err_msg=pid)


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb,opt", [
    (300, 7, 2000, 16, 7, "sgd"),            # ragged remainder batch
    (300, 40, 2000, 24, 50, "adagrad"),      # ~40 positives / batch: most relations absent
    (300, 5, 2000, 30, 3, "adagrad"),        # d % 4 != 0
    (40943, 18, 14140, 200, 10, "sgd"),      # WN18 entity / relation counts, d, batch size
    (40943, 18, 14140, 200, 9, "sgd"),       # odd number of batches: W ends in the 2nd buffer
    (300, 7, 2000, 25, 5, "adagrad"),        # odd d, M d^2 % 4 == 3: the W sync's scalar tail
])
def test_rescal_in_front_w_step_matches_apply_side(n_ent, n_rel, T, d, nb, opt, monkeypatch):
    """The W step inside the fused front (written speculatively into a second
    W / state buffer, made current by the apply when the batch has violations,
    copied back into the model's W at the epoch's end) against the W step in
    the entity apply's launch (SKGE_RESCAL_FORM=wapply) on the same draws: equal
    violation totals, parameters and W's AdaGrad state within the fp32
    tolerance after 2 epochs.  (AdaGrad only at small sizes: at WN18's, the
    entity sums' float-atomic order turns rounding-level differences of a
    near-zero first gradient into +-lr steps, as in the tests above.)"""
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    xs = make_kg(n_ent, n_rel, T, seed=10)
    out = []
    for form in ("wapply", ""):
        monkeypatch.setenv("SKGE_RESCAL_FORM", form)
        m = make_model("rescal", (n_ent, n_ent, n_rel), d)
        m.add_hyperparam("margin", 0.2)
        cls = S.SGD if opt == "sgd" else S.AdaGrad
        upd = {pid: cls(p, 0.1) for pid, p in m.params.items()}
        r = PairLoopRunner(m, upd, DeviceKG(xs, m.device), nb, seed=11)
        with torch.cuda.stream(r.stream):
            r.run(2)
        r.synchronize()
        state = {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()}
        if opt == "adagrad":
            state["W_p2"] = upd["W"].p2.cpu().numpy().copy()
        out.append((int(r.nviol_total.item()), state))
    assert out[0][0] == out[1][0] > 0
    for k in out[0][1]:
        np.testing.assert_allclose(out[1][1][k], out[0][1][k], rtol=RTOL, atol=ATOL, err_msg=k)


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb,opt", [
    (300, 7, 2000, 16, 7, "sgd"),            # ragged remainder batch
    (300, 40, 2000, 24, 50, "adagrad"),      # ~40 positives / batch: most relations absent
    (300, 5, 2000, 30, 3, "adagrad"),        # d % 4 != 0
    (60, 3, 3000, 20, 8, "adagrad"),         # 375 positives over 60 rows: ~25 slots per row
    (40943, 18, 14140, 200, 10, "sgd"),      # WN18 entity / relation counts, d, batch size
    (40943, 18, 14140, 200, 9, "sgd"),       # odd number of batches: W ends in the 2nd buffer
])
def test_rescal_row_grouped_apply_matches_scatter(n_ent, n_rel, T, d, nb, opt, monkeypatch):
    """The row-grouped entity update (k_rescal_fold: one wave per distinct
    entity row of the batch sums its slots' contributions in registers, in
    slot order, from the WE / EW rows and partial scores; no scatter launch,
    no entity atomics; the epoch's row grouping by k_rs_rows_ep) against the
    scatter's float atomics + the apply launch (SKGE_RESCAL_FORM=scatter) on the
    same draws: equal violation totals, parameters and AdaGrad states within
    the fp32 tolerance after 2 epochs.  (AdaGrad at small sizes only: at
    WN18's the atomics' summation order turns rounding-level differences of a
    near-zero first gradient into +-lr steps, as in the tests above; the
    runner oracle tests hold the WN18 AdaGrad case to the oracle.)"""
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    xs = make_kg(n_ent, n_rel, T, seed=14)
    out = []
    for form in ("scatter", ""):
        monkeypatch.setenv("SKGE_RESCAL_FORM", form)
        m = make_model("rescal", (n_ent, n_ent, n_rel), d)
        m.add_hyperparam("margin", 0.2)
        cls = S.SGD if opt == "sgd" else S.AdaGrad
        upd = {pid: cls(p, 0.1) for pid, p in m.params.items()}
        r = PairLoopRunner(m, upd, DeviceKG(xs, m.device), nb, seed=15)
        with torch.cuda.stream(r.stream):
            r.run(2)
        r.synchronize()
        state = {pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()}
        if opt == "adagrad":
            state["W_p2"] = upd["W"].p2.cpu().numpy().copy()
            state["E_p2"] = upd["E"].p2.cpu().numpy().copy()
        out.append((int(r.nviol_total.item()), state))
    assert out[0][0] == out[1][0] > 0
    for k in out[0][1]:
        np.testing.assert_allclose(out[1][1][k], out[0][1][k], rtol=RTOL, atol=ATOL, err_msg=k)


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb,det", [
    (40943, 18, 14140, 200, 10, False),   # WN18 geometry: rows of 1-4 slots, merged in order
    (60, 3, 3000, 20, 8, True),           # ~25 slots per row: hub rows, fixed-point atomics
])
def test_rescal_row_grouped_apply_is_deterministic(n_ent, n_rel, T, d, nb, det, monkeypatch):
    """The row-grouped apply sums each row's contributions in slot order and a
    row's items' partial sums in item order (no float atomics while a row has
    at most 16 slots in a batch); hub rows past that add through the entity
    accumulator, exact in the deterministic mode.  Two runs from the same
    state give the same bits."""
    import skge_amd as S
    from skge_amd.device import DeviceKG, PairLoopRunner
    monkeypatch.delenv("SKGE_RESCAL_FORM", raising=False)
    xs = make_kg(n_ent, n_rel, T, seed=16)
    out = []
    prev = S.deterministic()
    S.set_deterministic(det)
    try:
        out = _two_runs(S, DeviceKG, PairLoopRunner, xs, n_ent, n_rel, d, nb)
    finally:
        S.set_deterministic(prev)
    for pid in out[0]:
        assert np.array_equal(out[0][pid], out[1][pid]), pid


def _two_runs(S, DeviceKG, PairLoopRunner, xs, n_ent, n_rel, d, nb):
    out = []
    for _ in range(2):
        m = make_model("rescal", (n_ent, n_ent, n_rel), d)
        m.add_hyperparam("margin", 0.2)
        upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
        r = PairLoopRunner(m, upd, DeviceKG(xs, m.device), nb, seed=17)
        with torch.cuda.stream(r.stream):
            r.run(2)
        r.synchronize()
        out.append({pid: p.data.cpu().numpy().copy() for pid, p in m.params.items()})
    return out
