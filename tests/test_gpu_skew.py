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


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb", [
    (2000, 11, 12000, 64, 10),        # hot rows in every batch
    (40943, 18, 141442, 200, 100),    # WN18 geometry, skewed
    (40943, 18, 141442, 200, 10),     # WN18 skewed at nb = 10: 14k positives per batch, packed
                                      # sums from the per-batch (binomial) count bound
])
def test_pipelined_transe_bitwise_equals_two_launch_on_zipf(n_ent, n_rel, T, d, nb):
    from bench import make_zipf_kg
    from test_gpu_device_loop import _runner_result
    trip = make_zipf_kg(n_ent, n_rel, T, seed=3)
    top = np.bincount(np.concatenate([trip[:, 0], trip[:, 1]])).max()
    assert top > 10 * 2 * T / n_ent   # the KG is skewed: the hottest row is far above average
    a, _ = _runner_result(n_ent, n_rel, T, d, nb, pipelined=False, trip=trip)
    b, _ = _runner_result(n_ent, n_rel, T, d, nb, pipelined=True, trip=trip)
    assert a["key"] == b["key"] == 2
    assert a["nviol"] == b["nviol"] > 0
    for k in ("E", "R", "pE", "pR"):
        assert np.array_equal(a[k], b[k]), k


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
