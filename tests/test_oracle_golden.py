"""Pin the CPU oracle (oracle/skge_oracle.py) against the reference's golden vectors.

The fixtures were produced by running the reference's own trainer loop
(tools/gen_golden.py); every mini-batch of every case is replayed here through
the oracle from the same fp32-rounded initial parameters.
"""
import os

import numpy as np
import pytest

from golden_util import GOLDEN, Case, case_names, tol_for
from oracle import skge_oracle as O


def _close(got, exp, what):
    rtol, atol = tol_for(exp)
    np.testing.assert_allclose(got, exp.astype(np.float64), rtol=rtol, atol=atol, err_msg=what)


def replay_oracle(c):
    params = c.init_params()
    state = {pid: np.zeros_like(v) for pid, v in params.items()}
    for b in range(c.nbatch):
        bt = c.batch(b)
        if c.mode == "pairwise":
            kw = {"l1": c.l1} if c.model == "transe" else {"rparam": c.rparam}
            ps, ns, nv, g = O.pairwise_step(c.model, params, state, bt["pos"], bt["neg"],
                                            c.lr, c.margin, c.opt, **kw)
            _close(ps, bt["pscore"], "%s b%d pscore" % (c.name, b))
            _close(ns, bt["nscore"], "%s b%d nscore" % (c.name, b))
            assert nv == int(bt["nviol"]), (c.name, b)
            assert (g is not None) == bool(int(bt["has_grads"]))
        else:
            sc, loss, g = O.logistic_step(c.model, params, state, bt["trip"], bt["y"],
                                          c.lr, c.opt, rparam=c.rparam)
            _close(sc, bt["score"], "%s b%d score" % (c.name, b))
            np.testing.assert_allclose(loss, float(bt["loss"]), rtol=1e-9)
        if g is not None:
            for pid, (gv, gi) in g.items():
                if "g_" + pid in bt:
                    np.testing.assert_array_equal(gi, bt["gidx_" + pid])
                    _close(gv, bt["g_" + pid], "%s b%d grad %s" % (c.name, b, pid))
        for pid in c.param_ids:
            if "after_" + pid in bt:
                _close(params[pid], bt["after_" + pid], "%s b%d %s" % (c.name, b, pid))
            if "state_" + pid in bt:
                _close(state[pid], bt["state_" + pid], "%s b%d state %s" % (c.name, b, pid))


@pytest.mark.parametrize("name", case_names())
def test_oracle_matches_reference_fixture(name):
    replay_oracle(Case(name))


def test_init_quirks_and_fft():
    z = np.load(os.path.join(GOLDEN, "init_quirks.npz"))
    np.testing.assert_allclose(O.normalize(z["raw"].copy(), None), z["normalize_none"], rtol=1e-12)
    np.testing.assert_allclose(O.normless1(z["normless1_none_in"].copy(), None), z["normless1_none"],
                               rtol=1e-12)
    np.testing.assert_allclose(O.normless1(z["normless1_idx_in"].copy(), z["normless1_idx_idx"]),
                               z["normless1_idx"], rtol=1e-12)
    np.testing.assert_allclose(O.normalize(z["raw"].copy(), z["normless1_idx_idx"]),
                               z["normalize_idx"], rtol=1e-12)
    np.testing.assert_allclose(O.ccorr(z["cc_a"], z["cc_b"]), z["ccorr"], atol=1e-12)
    np.testing.assert_allclose(O.cconv(z["cc_a"], z["cc_b"]), z["cconv"], atol=1e-12)
    np.testing.assert_allclose(O.ccorr_direct(z["cc_a"], z["cc_b"]), z["ccorr"], atol=1e-12)
    np.testing.assert_allclose(O.cconv_direct(z["cc_a"], z["cc_b"]), z["cconv"], atol=1e-12)


def test_init_sequence_matches_reference_constructors():
    """Model constructors draw E then R (or W slices) from numpy's global RNG
    and apply the post projection at init (skge/base.py:1160-1164,
    skge/param.py:57-86)."""
    z = np.load(os.path.join(GOLDEN, "init_quirks.npz"))
    np.random.seed(42)
    E = O.normalize(O.init_nunif((50, 8)), None)
    R = O.init_nunif((4, 8))
    np.testing.assert_allclose(E, z["transe_E"], rtol=1e-12)
    np.testing.assert_allclose(R, z["transe_R"], rtol=1e-12)
    np.random.seed(42)
    E = O.normless1(O.init_nunif((50, 8)), None)
    R = O.init_nunif((4, 8))
    np.testing.assert_allclose(E, z["hole_E"], rtol=1e-12)
    np.testing.assert_allclose(R, z["hole_R"], rtol=1e-12)
    np.random.seed(42)
    E = O.init_nunif((50, 4))
    W = np.array([O.init_nunif((4, 4)) for _ in range(3)])
    np.testing.assert_allclose(E, z["rescal_E"], rtol=1e-12)
    np.testing.assert_allclose(W, z["rescal_W"], rtol=1e-12)


def test_batch_bounds_match_np_split():
    for T, nb in [(141442, 100), (200, 3), (120, 3), (7, 7), (10, 3)]:
        idx = np.arange(T)
        bs = T // nb
        ref = np.split(idx, np.arange(bs, T, bs))
        got = O.batch_bounds(T, nb)
        assert [(int(r[0]), int(r[-1]) + 1) for r in ref] == got
