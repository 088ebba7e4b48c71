"""The shipped benchmark runners against the fp64 oracle at WN18 geometry.

The bench lines of configs 2 / 3 / 4 run
  * TransE-L1: the pipelined runner (EpochRunner, k_pipe_batch: one launch
    scores batch b while batch b-1's rows are applied, packed exact sums),
  * HolE: HolePipeRunner (k_hole_pipe, the wave-FFT correlations),
  * RESCAL: PairLoopRunner's fused front (relation-grouped fp32 MFMA GEMMs +
    split-K dW, in-front W step, deduplicated rows).
Each is checked here DIRECTLY against oracle.pairwise_step
(skge/transe.py:48-165, skge/hole.py:44-100, skge/rescal.py:78-139 with
skge/param.py:140-174), not through another HIP path:

  WN18's entity and relation counts (N = 40943, M = 18), d = 200 and batch
  size (B = 1414 positives, 2828 pairs); the KG holds 3 x 1414 triples so one
  epoch is exactly 3 batches.  One epoch is trained first (AdaGrad state
  non-zero, tables moved), the device state is snapshotted, one more epoch
  runs, and the oracle replays that epoch's 3 batches -- the pairs the
  device drew (skge_epoch_sample, the same keyed draws the runners make) in
  the order PairwiseStochasticTrainer._process_batch builds them
  (skge/base.py:1394-1427) -- from the snapshot.

Bar: violation totals EXACTLY equal; parameters and AdaGrad state within
1e-5 + 1e-5|x| (+ the propagated AdaGrad rounding lr*1e-8/max(sqrt(p2),1e-7),
tests/parity_util.py), headroom recorded.
"""
import numpy as np
import pytest
import torch

import parity_util
from oracle import skge_oracle as O

pytestmark = pytest.mark.gpu

N, M, D, B = 40943, 18, 200, 1414
NB = 3
T = NB * B


def _kg(seed=21):
    rs = np.random.RandomState(seed)
    seen, out = set(), []
    while len(out) < T:
        t = (int(rs.randint(N)), int(rs.randint(N)), int(rs.randint(M)))
        if t not in seen:
            seen.add(t)
            out.append(t)
    return np.array(out, dtype=np.int32)


def _pairs(rec, n1, start, count):
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
    return np.array(pos, dtype=np.int64), np.array(neg, dtype=np.int64)


def _snapshot(m, upd):
    params = {pid: p.data.detach().cpu().numpy().astype(np.float64) for pid, p in m.params.items()}
    state = {pid: upd[pid].p2.detach().cpu().numpy().astype(np.float64) for pid in m.params}
    return params, state


def _replay_and_check(kind, m, upd, runner, kg, seed, **kw):
    from skge_amd.device import batch_sizes, epoch_records
    runner.run(1)                       # epoch 1: moves the tables, fills the AdaGrad state
    runner.synchronize()
    params, state = _snapshot(m, upd)
    v0 = int(runner.nviol_total.item())
    rec, n1 = epoch_records(kg, N, seed, 1)   # epoch 2's draws (epoch key 1)
    rec, n1 = rec.cpu().numpy(), n1.cpu().numpy()
    runner.run(1)
    runner.synchronize()
    got_v = int(runner.nviol_total.item()) - v0
    want_v = 0
    start = 0
    sizes = batch_sizes(kg.T, NB)
    assert sizes == [B] * NB
    for c in sizes:
        pos, neg = _pairs(rec, n1, start, c)
        start += c
        assert len(pos) == 2 * c          # WN18-sparse: every negative found
        want_v += O.pairwise_step(kind, params, state, pos, neg, 0.1, float(m.margin), "adagrad",
                                  **kw)[2]
    assert got_v == want_v > 0, (kind, got_v, want_v)
    for pid in m.params:
        parity_util.check(m.params[pid].data, params[pid], "%s runner %s" % (kind, pid),
                          lr=0.1, p2=state[pid])
        parity_util.check(upd[pid].p2, state[pid], "%s runner p2 %s" % (kind, pid))
    return got_v


def _setup(cls, **kw):
    import skge_amd as S
    from skge_amd.device import DeviceKG
    np.random.seed(42)
    m = cls((N, N, M), D, **kw)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
    kg = DeviceKG(_kg(), m.device)
    return m, upd, kg


def test_transe_pipelined_runner_vs_oracle():
    import skge_amd as S
    from skge_amd.device import EpochRunner
    m, upd, kg = _setup(S.TransE, l1=True)
    m.add_hyperparam("margin", 2.0)
    r = EpochRunner(m, upd, kg, nbatches=NB, seed=31)
    assert r.pipelined and r.packed
    with torch.cuda.stream(r.stream):
        _replay_and_check("transe", m, upd, r, kg, 31, l1=True)


def test_hole_pipe_runner_vs_oracle():
    import skge_amd as S
    from skge_amd.device import HolePipeRunner
    m, upd, kg = _setup(S.HolE)
    m.add_hyperparam("margin", 0.2)
    r = HolePipeRunner(m, upd, kg, NB, seed=32)
    with torch.cuda.stream(r.stream):
        _replay_and_check("hole", m, upd, r, kg, 32, af=O.Sigmoid)


def test_rescal_fused_front_runner_vs_oracle():
    import skge_amd as S
    from skge_amd.device import make_runner, PairLoopRunner
    m, upd, kg = _setup(S.RESCAL)
    m.add_hyperparam("margin", 0.2)
    r = make_runner(m, upd, kg, NB, seed=33)          # auto: the fused-front pair loop
    assert isinstance(r, PairLoopRunner)
    with torch.cuda.stream(r.stream):
        _replay_and_check("rescal", m, upd, r, kg, 33, af=O.Linear)
