"""Fused explicit-pair steps of every model on random batches at sizes the
golden fixtures do not reach (many relations, ragged d, duplicate rows), vs
the oracle; RESCAL runs on the relation-grouped fp32 MFMA path for d <= 480
(skge_rescal.hip).  Tolerances 1e-5 + 1e-5|x| plus, for the AdaGrad steps,
the fp32 gradient rounding propagated through the step and the projection
(tests/parity_util.py check_step); violation counts exact."""
import numpy as np
import pytest
import torch

from oracle import skge_oracle as O
import parity_util
from test_gpu_parity import close, close_adagrad

pytestmark = pytest.mark.gpu


def _batch(rs, n_ent, n_rel, P, diff_rel=0.1):
    pos = np.stack([rs.randint(n_ent, size=P), rs.randint(n_ent, size=P),
                    rs.randint(n_rel, size=P)], axis=1).astype(np.int32)
    neg = pos.copy()
    mode = rs.randint(2, size=P)
    neg[mode == 0, 0] = rs.randint(n_ent, size=int((mode == 0).sum()))
    neg[mode == 1, 1] = rs.randint(n_ent, size=int((mode == 1).sum()))
    flip = rs.rand(P) < diff_rel            # some pairs with a different negative relation
    neg[flip, 2] = rs.randint(n_rel, size=int(flip.sum()))
    return pos, neg


def _model(name, n_ent, n_rel, d, seed=3, rparam=0.0):
    import skge_amd as S
    np.random.seed(seed)
    sz = (n_ent, n_ent, n_rel)
    if name == "rescal":
        m = S.RESCAL(sz, d, rparam=rparam)
        m.add_hyperparam("margin", 0.2)
    elif name == "hole":
        m = S.HolE(sz, d, rparam=rparam)
        m.add_hyperparam("margin", 0.2)
    else:
        m = S.TransE(sz, d)
        m.add_hyperparam("margin", 2.0)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
    return m, upd


def _run(name, n_ent, n_rel, d, P, nb, rparam=0.0, seed=5):
    """nb steps; each step is compared with one oracle step taken from the
    device's own state before it (AdaGrad's first step moves an element by
    lr*sign(g), so an element whose gradient is ~0 at fp32 rounding level
    may legitimately land on either side; chaining oracle steps across
    batches would compound such an element into unrelated later errors)."""
    m, upd = _model(name, n_ent, n_rel, d, rparam=rparam)
    rs = np.random.RandomState(seed)
    nviol = torch.zeros(1, dtype=torch.int32, device=m.device)
    for b in range(nb):
        params = {pid: p.data.detach().cpu().numpy().astype(np.float64)
                  for pid, p in m.params.items()}
        state = {pid: upd[pid].p2.detach().cpu().numpy().astype(np.float64) for pid in m.params}
        pos, neg = _batch(rs, n_ent, n_rel, P)
        nviol.zero_()
        m._pairwise_step(torch.as_tensor(pos, device=m.device), torch.as_tensor(neg, device=m.device),
                         upd, nviol)
        kw = {"rparam": rparam} if name != "transe" else {"l1": True}
        before = {k: v.copy() for k, v in params.items()}
        _, _, nv, grads = O.pairwise_step(name, params, state, pos, neg, 0.1, float(m.margin),
                                          "adagrad", **kw)
        assert int(nviol.item()) == nv, (name, b)
        for pid in m.params:
            parity_util.check_step(m.params[pid].data, params[pid], before[pid],
                                   grads[pid] if grads else None, state[pid], 0.1,
                                   "%s b%d %s" % (name, b, pid),
                                   post=parity_util.POSTS[name].get(pid))
            close(upd[pid].p2, state[pid], "%s b%d p2 %s" % (name, b, pid))
    return m


@pytest.mark.parametrize("n_ent,n_rel,d,P", [(300, 7, 40, 600),     # ragged d (not a multiple of 16)
                                             (400, 18, 200, 700),   # WN18 width and relations
                                             (50, 3, 64, 900),      # many duplicate rows
                                             (200, 40, 8, 300)])    # more relations than 16-tiles
def test_rescal_mfma_step_vs_oracle(n_ent, n_rel, d, P):
    _run("rescal", n_ent, n_rel, d, P, nb=3)


def test_rescal_mfma_rparam():
    _run("rescal", 300, 5, 32, 400, nb=2, rparam=0.05)


def test_rescal_mfma_relation_gradient_deterministic():
    """Stable buckets + fixed MFMA k order + plain stores: W after one step is
    bitwise reproducible (entity sums use float atomics, so E is not)."""
    outs = []
    for _ in range(2):
        m = _run("rescal", 300, 9, 48, 500, nb=1)
        outs.append(m.params["W"].data.cpu().numpy().copy())
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("n_ent,n_rel,d,P", [(300, 7, 40, 600), (400, 18, 200, 500)])
def test_hole_step_vs_oracle(n_ent, n_rel, d, P):
    _run("hole", n_ent, n_rel, d, P, nb=2)


def _run_logistic(name, n_ent, n_rel, d, B, nb, rparam=0.0, seed=9):
    """StochasticTrainer-style steps (B positives y=+1 and their two sampler
    corruptions y=-1, skge/base.py:1293-1304) vs one oracle logistic step from
    the device's state before each."""
    m, upd = _model(name, n_ent, n_rel, d, rparam=rparam)
    rs = np.random.RandomState(seed)
    loss = torch.zeros(1, dtype=torch.float32, device=m.device)
    for b in range(nb):
        params = {pid: p.data.detach().cpu().numpy().astype(np.float64)
                  for pid, p in m.params.items()}
        state = {pid: upd[pid].p2.detach().cpu().numpy().astype(np.float64) for pid in m.params}
        pos, neg = _batch(rs, n_ent, n_rel, B, diff_rel=0.0)
        trip = np.concatenate([pos, neg]).astype(np.int32)
        ys = np.concatenate([np.ones(B), -np.ones(B)]).astype(np.float32)
        loss.zero_()
        m._logistic_step(torch.as_tensor(trip, device=m.device),
                         torch.as_tensor(ys, device=m.device), upd, loss)
        _, want_loss, _ = O.logistic_step(name, params, state, trip, ys.astype(np.float64), 0.1,
                                          "adagrad", rparam=rparam)
        np.testing.assert_allclose(float(loss.item()), want_loss, rtol=1e-5)
        for pid in m.params:
            close_adagrad(m.params[pid].data, params[pid], state[pid], 0.1,
                          "%s logistic b%d %s" % (name, b, pid))
            close(upd[pid].p2, state[pid], "%s logistic b%d p2 %s" % (name, b, pid))


@pytest.mark.parametrize("n_ent,n_rel,d,B", [(300, 7, 40, 300), (400, 18, 200, 350)])
def test_rescal_logistic_mfma_vs_oracle(n_ent, n_rel, d, B):
    _run_logistic("rescal", n_ent, n_rel, d, B, nb=2)


def test_rescal_logistic_rparam():
    _run_logistic("rescal", 300, 5, 32, 200, nb=2, rparam=0.05)


@pytest.mark.parametrize("n_ent,n_rel,d,B", [(300, 7, 40, 300), (400, 18, 200, 250)])
def test_hole_logistic_vs_oracle(n_ent, n_rel, d, B):
    _run_logistic("hole", n_ent, n_rel, d, B, nb=2)


@pytest.mark.parametrize("name", ["transe", "hole", "rescal"])
def test_empty_batch_is_a_no_op(name):
    """A batch with no pairs (every negative draw rejected) or no triples: the
    reference would fail unpacking empty lists (unzip_triples of []); here
    _pairwise_gradients returns None with no violations, the fused steps
    launch nothing harmful, and the parameters do not move."""
    m, upd = _model(name, 50, 3, 16)
    before = {pid: p.data.clone() for pid, p in m.params.items()}
    assert m._pairwise_gradients([], []) is None
    assert m.nviolations == 0
    nviol = torch.zeros(1, dtype=torch.int32, device=m.device)
    empty = torch.zeros((0, 3), dtype=torch.int32, device=m.device)
    m._pairwise_step(empty, empty, upd, nviol)
    torch.cuda.synchronize()
    assert int(nviol.item()) == 0
    for pid, p in m.params.items():
        assert torch.equal(p.data, before[pid]), pid
