"""The deterministic reduce mode (skge_amd.set_deterministic, SKGE_ACC_FX64).

The reference's segment mean is a CSR mat-vec (skge/util.py:53-101): the same
inputs give the same bits every run.  The default fp32-atomic accumulators of
the float-valued models (HolE, RESCAL entity rows, TransE-L2) add in arrival
order, so E is not run-to-run reproducible there.  With the mode on, every
contribution is rounded once to a 2^-40 fixed-point grid and summed with exact
integer atomics: two runs of the same epochs must give the same bits, and the
step must still match the fp64 oracle within the 1e-5 bar.
"""
import numpy as np
import pytest
import torch

import parity_util
from oracle import skge_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture
def det():
    import skge_amd as S
    S.set_deterministic(True)
    yield S
    S.set_deterministic(False)


def _pair_loop(S, kind, xs, n_ent, n_rel, d, nb, epochs=2):
    from skge_amd import _lib as L
    from skge_amd.device import DeviceKG, make_runner
    np.random.seed(42)
    m = (S.HolE if kind == "hole" else S.RESCAL)((n_ent, n_ent, n_rel), d, rparam=0.05)
    m.add_hyperparam("margin", 0.2)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
    r = make_runner(m, upd, DeviceKG(xs, m.device), nb, seed=3)
    assert type(r).__name__ == "PairLoopRunner"
    assert m.accumulator("E").mode == L.SKGE_ACC_FX64
    with torch.cuda.stream(r.stream):
        r.run(epochs)
    r.synchronize()
    return int(r.nviol_total.item()), {pid: p.data.cpu().numpy().copy()
                                       for pid, p in m.params.items()}


@pytest.mark.parametrize("kind", ["hole", "rescal"])
def test_pair_loop_bitwise_reproducible(det, kind):
    from test_gpu_pairloop import make_kg
    n_ent, n_rel, T, d, nb = 40943, 18, 14140, 200, 10   # WN18 rows, d, batch size
    xs = make_kg(n_ent, n_rel, T, seed=4)
    a = _pair_loop(det, kind, xs, n_ent, n_rel, d, nb)
    b = _pair_loop(det, kind, xs, n_ent, n_rel, d, nb)
    assert a[0] == b[0] > 0
    for pid in a[1]:
        assert np.array_equal(a[1][pid], b[1][pid]), pid


def test_transe_l2_epoch_runner_bitwise_reproducible(det):
    from skge_amd import _lib as L
    from skge_amd.device import DeviceKG, EpochRunner
    from test_gpu_device_loop import make_kg
    trip, _ = make_kg(3000, 11, 12000)
    out = []
    for _ in range(2):
        np.random.seed(7)
        m = det.TransE((3000, 3000, 11), 64, l1=False)
        m.add_hyperparam("margin", 2.0)
        upd = {pid: det.AdaGrad(p, 0.1) for pid, p in m.params.items()}
        r = EpochRunner(m, upd, DeviceKG(trip, m.device), nbatches=6, seed=2)
        assert not r.packed and r.accE.mode == L.SKGE_ACC_FX64
        r.run(2)
        r.synchronize()
        out.append((int(r.nviol_total.item()), m.E.data.cpu().numpy().copy(),
                    m.R.data.cpu().numpy().copy()))
    assert out[0][0] == out[1][0] > 0
    assert np.array_equal(out[0][1], out[1][1]) and np.array_equal(out[0][2], out[1][2])


@pytest.mark.parametrize("kind", ["hole", "rescal"])
def test_deterministic_step_matches_oracle(det, kind):
    """The fixed-point sums still meet the 1e-5 bar against the fp64 oracle
    (per batch from the device state, as tests/test_gpu_models.py)."""
    from test_gpu_models import _run
    _run(kind, 400, 18, 200, 700 if kind == "rescal" else 500, nb=2)


@pytest.mark.parametrize("mag", [1.0, 5.0e6])
def test_fx64_range_flag(mag):
    """FX64 sums wrap past 2^23 gradient units.  An apply that
    decodes a sum at or past 2^22 (half the range) sets skge_device_error
    bit 4 (a wrap itself is caught at the add, below), which
    check_device_error (every runner's synchronize) raises; ordinary sums do
    not."""
    import skge_amd as S
    from skge_amd import _lib as L
    from skge_amd.param import Accumulator, table_struct
    dev = torch.device("cuda", 0)
    rows, d = 8, 64
    P = S.param.Parameter(None, name="W", value=torch.zeros((rows, d), device=dev))
    acc = Accumulator(rows, d, dev, slots=4, mode=L.SKGE_ACC_FX64)
    x = acc.sum.view(torch.int64).view(rows, d)
    x[3] = int(mag * 2 ** 40)           # one row's fixed-point sum, count 1
    acc.cnt[3] = 1
    acc.touched[0] = 3
    t = table_struct(P, None, acc, opt=L.SKGE_SGD, post=L.SKGE_POST_NONE, lr=1.0)
    L.lib().skge_device_error(L.stream_ptr(), 1)
    L.check(L.lib().skge_accum_apply(L.stream_ptr(), (L.SkgeTable * 1)(t), 1, L.int_array(4)),
            "apply")
    if mag < 2 ** 22:
        L.check_device_error(L.stream_ptr(), "fx64")
        assert float(P.data[3, 0].item()) == -mag
    else:
        with pytest.raises(L.SkgeError, match="FX64"):
            L.check_device_error(L.stream_ptr(), "fx64")


@pytest.mark.parametrize("preset", [0, 2 ** 63 - 1])
def test_fx64_wrap_caught_when_added(det, preset):
    """the decode-time range check alone misses a sum that wraps
    back inside half the range.  Every fixed-point add is a returned atomic
    that checks its own signed overflow (acc_row): a row whose sums sit at
    the top of the range and receive positive contributions sets
    skge_device_error bit 4 in the producer itself -- no apply or collect
    (which would decode) runs here; from zero nothing is flagged."""
    from skge_amd import _lib as L
    np.random.seed(5)
    n, nr, d, P = 50, 3, 64, 40
    m = det.TransE((n, n, nr), d, l1=False)
    m.add_hyperparam("margin", 1.0e9)           # every pair violates
    rs = np.random.RandomState(1)
    s, o, p = rs.randint(0, n, P), rs.randint(0, n, P), rs.randint(0, nr, P)
    s[:] = 7                                    # row 7 in every positive
    pos = torch.tensor(np.stack([s, o, p], 1), dtype=torch.int32, device="cuda")
    neg = torch.tensor(np.stack([s, rs.randint(0, n, P), p], 1), dtype=torch.int32,
                       device="cuda")
    te, tr = m._tables("pairwise", slots=m._pair_slots(P))
    acc = m.accumulator("E")
    assert acc.mode == L.SKGE_ACC_FX64
    x = acc.sum.view(torch.int64).view(-1, d)
    x.zero_()
    x[7] = preset
    nviol = torch.zeros(1, dtype=torch.int32, device="cuda")
    L.lib().skge_device_error(L.stream_ptr(), 1)
    L.check(L.lib().skge_pair_grad(L.stream_ptr(), m._kernel_model(), m._af_code(), te, tr, d,
                                   L.ptr(pos), L.ptr(neg), P, 1.0e9, None, None, None,
                                   L.ptr(nviol)), "pair_grad")
    torch.cuda.synchronize()
    assert int(nviol.item()) == P
    if preset == 0:
        L.check_device_error(L.stream_ptr(), "fx64")
    else:
        with pytest.raises(L.SkgeError, match="FX64"):
            L.check_device_error(L.stream_ptr(), "fx64")
    L.lib().skge_device_error(L.stream_ptr(), 1)   # leave the global error word clean
