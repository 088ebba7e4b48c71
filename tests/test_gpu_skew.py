"""Skewed KGs (SURVEY 8(d)'s Zipf variant, bench.make_zipf_kg): a few entity
rows take a large share of every batch, so nearly every scoring wave of the
pipelined runners meets a row the previous batch touched (the claim / wait
hand-off), many slot records name the same row (duplicate claims), and the
hot rows' per-batch counts leave the int8x4 range (the runner falls back to
int16x4 sums).  The runners must still reproduce their references: the
pipelined TransE runner the two-launch loop bit for bit, the pipelined HolE
runner (two waves per positive at d = 200) the device pair loop within fp32
tolerance.  (With AdaGrad over two epochs the hot rows' fp32 sums, added in
a different order by the two HolE runners, drift far enough apart to flip a
few dozen of ~37k margin tests -- measured at N = 2000 -- so the HolE cases
use SGD, as the uniform-KG ones mostly do.)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb,fused", [
    (2000, 11, 12000, 64, 10, "1"),       # hot rows in every batch (k_pipe_fused: no replicas)
    (2000, 11, 12000, 64, 10, "0"),       # the same on k_pipe_batch: hot-row replicas
    (2000, 11, 12000, 512, 10, None),     # two quads per lane (hot rows at KQ = 2)
    (1000, 5, 6000, 1024, 6, None),       # the widest packed row (KQ = 4)
    (40943, 18, 141442, 200, 100, None),  # WN18 geometry, skewed (hot-row replicas)
    (40943, 18, 141442, 200, 10, None),   # WN18 skewed at nb = 10: 14k positives per batch,
                                          # packed sums from the per-batch (binomial) count bound
])
def test_pipelined_transe_bitwise_equals_two_launch_on_zipf(n_ent, n_rel, T, d, nb, fused,
                                                            monkeypatch):
    """k_pipe_batch gives the hub rows HOT_REPS = 4 replicas of their sums and
    counts (csrc/skge_pipe.h),
    and every scoring wave that reads a hub computes its value itself
    (hot_value, the applier's code): still the two-launch loop bit for bit."""
    from bench import make_zipf_kg
    from test_gpu_device_loop import _runner_result
    if fused is not None:
        monkeypatch.setenv("SKGE_PIPE_FUSED", fused)
    trip = make_zipf_kg(n_ent, n_rel, T, seed=3)
    top = np.bincount(np.concatenate([trip[:, 0], trip[:, 1]])).max()
    assert top > 10 * 2 * T / n_ent   # the KG is skewed: the hottest row is far above average
    a, _ = _runner_result(n_ent, n_rel, T, d, nb, pipelined=False, trip=trip)
    b, _ = _runner_result(n_ent, n_rel, T, d, nb, pipelined=True, trip=trip)
    assert (b["hot"] > 0) == (fused != "1"), b["hot"]
    assert a["key"] == b["key"] == 2
    assert a["nviol"] == b["nviol"] > 0
    for k in ("E", "R", "pE", "pR"):
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("d,fused", [(200, "0"), (64, "1")])
def test_pipelined_hot_rows_across_runs(d, fused, monkeypatch):
    """State that lives in the runner between launches must be back in the
    caller's tables after every run(): the hand-off kernel's hot rows (in the
    runner's own buffers during a run, copied in before the first launch and
    back after the flush) and the fused kernel's rows in its second buffer
    (k_fused_fin copies them back, incl. the AdaGrad state, and the meta
    words are cleared).  Two run(1) calls must equal one run(2) bit for bit,
    and the tables between runs must hold the trained values."""
    import skge_amd as S
    from bench import make_zipf_kg
    from skge_amd.device import DeviceKG, EpochRunner
    monkeypatch.setenv("SKGE_PIPE_FUSED", fused)

    def train(calls):
        np.random.seed(5)
        m = S.TransE((2000, 2000, 11), d)
        m.add_hyperparam("margin", 2.0)
        upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
        kg = DeviceKG(make_zipf_kg(2000, 11, 12000, seed=3), m.device)
        r = EpochRunner(m, upd, kg, nbatches=10, seed=7, pipelined=True)
        assert (r.hot_rows > 0) == (fused == "0")
        mid = None
        for k, n in enumerate(calls):
            r.run(n)
            r.synchronize()
            if k == 0:
                mid = m.E.data.cpu().numpy().copy()
        return m.E.data.cpu().numpy().copy(), upd["E"].p2.cpu().numpy().copy(), mid
    e2, a2, _ = train([2])
    e11, a11, mid = train([1, 1])
    e1, _, _ = train([1])
    assert np.array_equal(mid, e1)
    assert np.array_equal(e2, e11) and np.array_equal(a2, a11)


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb,epochs,opt", [
    (2000, 11, 12000, 200, 10, 2, "sgd"),       # pair form, hot rows
    (40943, 18, 14140, 200, 10, 1, "sgd"),      # WN18 entity count and batch size, skewed
    (2000, 11, 12000, 32, 10, 2, "sgd"),        # the generic-d transform (one wave per positive)
])
def test_hole_pipelined_matches_pair_loop_on_zipf(n_ent, n_rel, T, d, nb, epochs, opt):
    from bench import make_zipf_kg
    from skge_amd.device import HolePipeRunner, PairLoopRunner
    from test_gpu_pairloop import ATOL, RTOL, _hole_epochs
    xs = [tuple(t) for t in make_zipf_kg(n_ent, n_rel, T, seed=5).tolist()]
    a = _hole_epochs(PairLoopRunner, xs, n_ent, n_rel, d, nb, epochs, opt=opt)
    b = _hole_epochs(HolePipeRunner, xs, n_ent, n_rel, d, nb, epochs, opt=opt)
    assert a[1] == b[1] == epochs
    assert a[0] > 0 and abs(a[0] - b[0]) <= 2, (a[0], b[0])
    for pid in a[2]:
        np.testing.assert_allclose(b[2][pid], a[2][pid], rtol=RTOL, atol=ATOL,
                                   err_msg="%s (%d, %d)" % (pid, a[0], b[0]))
