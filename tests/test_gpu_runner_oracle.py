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
  size (B = 1414 positives, 2828 pairs).  The oracle replays the pairs the
  device drew (skge_epoch_sample, the same keyed draws the runners make) in
  the order PairwiseStochasticTrainer._process_batch builds them
  (skge/base.py:1394-1427), from the device state snapshotted before them:
  (a) AdaGrad, the bench's updater: one batch per epoch, each batch from the
      device state right before it;
  (b) one epoch of 3 batches (the pipelined hand-off between batches), SGD.

Bar: violation totals EXACTLY equal; parameters and AdaGrad state within
1e-5 + 1e-5|x|, plus for one AdaGrad step the gradient's fp32 rounding
propagated through the step and the row projection (parity_util.check_step:
lr * eps / max(sqrt(p2), 1e-7), eps = 1e-8 + 4 ulps of the gradient row's
norm; a projected row's scale carries its elements' allowance to the whole
row), headroom recorded.
"""
import numpy as np
import pytest
import torch

import parity_util
from oracle import skge_oracle as O

pytestmark = pytest.mark.gpu

N, M, D, B = 40943, 18, 200, 1414


def _kg(T, seed=21):
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
    state = {pid: upd[pid].p2.detach().cpu().numpy().astype(np.float64)
             for pid in m.params if getattr(upd[pid], "p2", None) is not None}
    return params, state


def _epoch_vs_oracle(kind, m, upd, runner, kg, seed, epoch, nb, opt, what, **kw):
    """Run epoch `epoch` (0-based; the runner's key is at it) on the device and
    replay its batches through the oracle from the device state before it."""
    from skge_amd.device import batch_sizes, epoch_records
    params, state = _snapshot(m, upd)
    if opt == "sgd":
        state = {k: np.zeros_like(v) for k, v in params.items()}
    v0 = int(runner.nviol_total.item())
    rec, n1 = epoch_records(kg, N, seed, epoch)
    rec, n1 = rec.cpu().numpy(), n1.cpu().numpy()
    runner.run(1)
    runner.synchronize()
    got_v = int(runner.nviol_total.item()) - v0
    want_v, start = 0, 0
    sizes = batch_sizes(kg.T, nb)
    assert sizes == [B] * nb
    for c in sizes:
        pos, neg = _pairs(rec, n1, start, c)
        start += c
        assert len(pos) == 2 * c          # WN18-sparse: every negative found
        before = {k: v.copy() for k, v in params.items()}
        _, _, nv, grads = O.pairwise_step(kind, params, state, pos, neg, 0.1, float(m.margin),
                                          opt, **kw)
        want_v += nv
    assert got_v == want_v, (what, got_v, want_v)
    for pid in m.params:
        if nb == 1:     # one step from the snapshot: the step-aware bound (parity_util.check_step)
            parity_util.check_step(m.params[pid].data, params[pid], before[pid],
                                   grads[pid] if grads else None, state[pid], 0.1,
                                   "%s %s" % (what, pid), post=parity_util.POSTS[kind].get(pid),
                                   opt=opt)
        else:
            parity_util.check(m.params[pid].data, params[pid], "%s %s" % (what, pid),
                              lr=0.1 if opt == "adagrad" else None,
                              p2=state[pid] if opt == "adagrad" else None)
        if opt == "adagrad":
            parity_util.check(upd[pid].p2, state[pid], "%s p2 %s" % (what, pid))
    return got_v


def _setup(cls, T, opt, d=D, lr=0.1, no_post=False, **kw):
    import skge_amd as S
    from skge_amd.device import DeviceKG
    np.random.seed(42)
    m = cls((N, N, M), d, **kw)
    if no_post:          # gradient probe: the rows' projection off (see test below)
        for p in m.params.values():
            p.post = None
    U = S.AdaGrad if opt == "adagrad" else S.SGD
    upd = {pid: U(p, lr) for pid, p in m.params.items()}
    kg = DeviceKG(_kg(T), m.device)
    return m, upd, kg


def _runner(kind, m, upd, kg, nb, seed):
    from skge_amd.device import EpochRunner, HolePipeRunner, PairLoopRunner, make_runner
    if kind == "transe":
        r = EpochRunner(m, upd, kg, nbatches=nb, seed=seed)
        assert r.pipelined and r.packed
    elif kind == "hole":
        r = HolePipeRunner(m, upd, kg, nb, seed=seed)
    else:
        r = make_runner(m, upd, kg, nb, seed=seed)      # auto: the fused-front pair loop
        assert isinstance(r, PairLoopRunner)
    return r


CASES = {"transe": ("TransE", {"l1": True}, 2.0, {"l1": True}),
         "hole": ("HolE", {}, 0.2, {"af": O.Sigmoid}),
         "rescal": ("RESCAL", {}, 0.2, {"af": O.Linear})}


@pytest.mark.parametrize("kind", ["transe", "hole", "rescal"])
def test_runner_adagrad_batches_vs_oracle_from_device_state(kind):
    """AdaGrad (the bench configuration): one batch of B = 1414 positives per
    epoch, 3 epochs; every batch replayed from the device state (parameters
    AND AdaGrad state) right before it, so rounding-level differences of a
    near-zero first gradient are not compounded through p2 across batches."""
    import skge_amd as S
    name, ckw, margin, okw = CASES[kind]
    m, upd, kg = _setup(getattr(S, name), B, "adagrad", **ckw)
    m.add_hyperparam("margin", margin)
    r = _runner(kind, m, upd, kg, 1, 41)
    with torch.cuda.stream(r.stream):
        viol = [_epoch_vs_oracle(kind, m, upd, r, kg, 41, e, 1, "adagrad",
                                 "%s runner adagrad e%d" % (kind, e), **okw) for e in range(3)]
    assert viol[0] > 0      # (a later epoch may separate every pair by the margin)


@pytest.mark.parametrize("kind", ["transe", "hole", "rescal"])
def test_runner_epoch_of_three_batches_vs_oracle(kind):
    """One epoch of 3 batches (B = 1414): the pipelined hand-off between
    batches (rows of batch b-1 applied while batch b is scored) in the chain.
    SGD keeps the 3-batch oracle chain linear (AdaGrad's per-element divisor
    would compound rounding of near-zero first gradients across batches, see
    the test above); an epoch is trained first so the tables have moved."""
    import skge_amd as S
    name, ckw, margin, okw = CASES[kind]
    m, upd, kg = _setup(getattr(S, name), 3 * B, "sgd", **ckw)
    m.add_hyperparam("margin", margin)
    r = _runner(kind, m, upd, kg, 3, 42)
    with torch.cuda.stream(r.stream):
        r.run(1)
        r.synchronize()
        assert _epoch_vs_oracle(kind, m, upd, r, kg, 42, 1, 3, "sgd",
                                "%s runner sgd 3 batches" % kind, **okw) > 0


def test_config1_padded_runner_three_batches_vs_oracle():
    """BASELINE configs[0] (run_transe_wn18.sh:3-5): TransE-L1 d = 50, SGD, the
    bench's runner -- the pipelined runner on zero-padded d = 64 tables --
    one epoch of 3 batches of B = 1414 against the oracle (after a first
    epoch so the tables have moved)."""
    import skge_amd as S
    m, upd, kg = _setup(S.TransE, 3 * B, "sgd", d=50, l1=True)
    m.add_hyperparam("margin", 2.0)
    r = _runner("transe", m, upd, kg, 3, 43)
    assert r._pad and r.d_pad == 64      # device.padded_width: whole 128-B lines
    with torch.cuda.stream(r.stream):
        r.run(1)
        r.synchronize()
        assert _epoch_vs_oracle("transe", m, upd, r, kg, 43, 1, 3, "sgd",
                                "config1 padded runner sgd 3 batches", l1=True) > 0


@pytest.mark.parametrize("kind", ["transe", "hole"])
def test_runner_skewed_kg_hot_rows_vs_oracle(kind):
    """SURVEY 8(d)'s skew variant (bench.make_zipf_kg: entity ids Zipf(1.1),
    WN18's entity and relation counts) on the shipped runners with their
    hub rows in replicated sums whose updated values every reader computes
    itself (TransE: k_pipe_batch's hot rows; HolE: k_hole_pipe's pair form):
    one epoch of 3 batches of B = 1414, SGD, after a first epoch, replayed
    DIRECTLY by the oracle -- not only against another HIP runner
    (test_gpu_skew.py)."""
    import skge_amd as S
    from bench import make_zipf_kg
    from skge_amd.device import DeviceKG
    name, ckw, margin, okw = CASES[kind]
    np.random.seed(42)
    m = getattr(S, name)((N, N, M), D, **ckw)
    m.add_hyperparam("margin", margin)
    upd = {pid: S.SGD(p, 0.1) for pid, p in m.params.items()}
    kg = DeviceKG(make_zipf_kg(N, M, 3 * B, seed=7), m.device)
    r = _runner(kind, m, upd, kg, 3, 45)
    assert r.hot_rows > 0, "the skewed KG must give the runner hub rows"
    with torch.cuda.stream(r.stream):
        r.run(1)
        r.synchronize()
        assert _epoch_vs_oracle(kind, m, upd, r, kg, 45, 1, 3, "sgd",
                                "%s runner zipf hot rows sgd 3 batches" % kind, **okw) > 0


GRAD_CASES = [("transe", 200), ("transe", 50), ("hole", 200), ("rescal", 200)]


@pytest.mark.parametrize("kind,d", GRAD_CASES)
def test_runner_gradients_vs_oracle(kind, d):
    """Gradient-level parity of the SHIPPED runners (k_pipe_batch incl. config
    1's padded tables, k_hole_pipe, RESCAL's fused front) at WN18 geometry,
    at the plain north-star bar 1e-5 + 1e-5|g| -- no AdaGrad amplification term.

    Gradient probe: the same runner with its updaters set to SGD(lr = 1) and
    the rows' projection off, one batch of B = 1414 positives from the tables
    after one AdaGrad-free training epoch.  The apply then computes
    P' = fl(P - g) with g the device's segment mean (accumulated sums / counts,
    skge/util.py:53-101), so P - P' (exact in fp64) is g to within half an ulp
    of |P'| (<= 6e-8 here).  Compared with oracle.pairwise_step's (grad, idx)
    rows (transe.py:48-165, hole.py:44-100, rescal.py:78-139); rows outside
    idx must be unchanged, violations exactly equal."""
    import skge_amd as S
    from skge_amd.device import epoch_records
    name, ckw, margin, okw = CASES[kind]
    # HolE / RESCAL: warm the tables up with one ordinary epoch (shipped updater,
    # projection on); TransE from its initial tables (after one SGD epoch only
    # ~10 of its 2828 pairs still violate the margin of 2)
    m0, upd0, kg = _setup(getattr(S, name), B, "sgd", d=d, **ckw)
    m0.add_hyperparam("margin", margin)
    if kind != "transe":
        r0 = _runner(kind, m0, upd0, kg, 1, 44)
        r0.run(1)
        r0.synchronize()
        del r0
    warm = {pid: p.data.clone() for pid, p in m0.params.items()}
    m, upd, _ = _setup(getattr(S, name), 1, "sgd", d=d, lr=1.0, no_post=True, **ckw)
    m.add_hyperparam("margin", margin)
    for pid, p in m.params.items():
        p.data.copy_(warm[pid])
    r = _runner(kind, m, upd, kg, 1, 44)
    if kind == "transe":
        assert r.pipelined and (r._pad == (d % 4 != 0))
    before = {pid: p.data.detach().cpu().numpy().astype(np.float64) for pid, p in m.params.items()}
    rec, n1 = epoch_records(kg, N, 44, 0)
    rec, n1 = rec.cpu().numpy(), n1.cpu().numpy()
    with torch.cuda.stream(r.stream):
        r.run(1)
        r.synchronize()
    torch.cuda.synchronize()
    got_v = int(r.nviol_total.item())
    pos, neg = _pairs(rec, n1, 0, B)
    params = {k: v.copy() for k, v in before.items()}
    state = {k: np.zeros_like(v) for k, v in before.items()}
    _, _, want_v, grads = O.pairwise_step(kind, params, state, pos, neg, 1.0, margin, "sgd", **okw)
    assert got_v == want_v > (200 if kind == "transe" else 0)
    for pid, p in m.params.items():
        after = p.data.detach().cpu().numpy().astype(np.float64)
        g_dev = before[pid] - after
        rows, idx = grads[pid]
        idx = np.asarray(idx, dtype=np.int64)
        mask = np.ones(g_dev.shape[0], dtype=bool)
        mask[idx] = False
        assert np.array_equal(after[mask], before[pid][mask]), "%s %s: untouched rows moved" % (kind, pid)
        parity_util.check(g_dev[idx], np.asarray(rows, dtype=np.float64),
                          "%s d%d runner gradient %s" % (kind, d, pid))
