"""Device filtered ranking (skge_rank) against the positions of the
reference's own evaluators (tests/golden/eval_*.npz) and the oracle."""
import os

import numpy as np
import pytest
import torch

from oracle import skge_oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _model(name, n_ent, n_rel, d, E=None, R=None, seed=1):
    import skge_amd as S
    np.random.seed(seed)
    sz = (n_ent, n_ent, n_rel)
    m = {"transe": S.TransE, "hole": S.HolE, "rescal": S.RESCAL}[name](sz, d)
    rid = "W" if name == "rescal" else "R"
    if E is not None:
        m.params["E"].data.copy_(torch.as_tensor(E, dtype=torch.float32))
        m.params[rid].data.copy_(torch.as_tensor(R, dtype=torch.float32))
    return m


@pytest.mark.parametrize("name", ["transe", "hole"])
def test_ranks_match_reference_positions(name):
    import skge_amd as S
    z = np.load(os.path.join(GOLD, "eval_%s.npz" % name))
    E, R = z["E"], z["R"]
    m = _model(name, E.shape[0], R.shape[0], E.shape[1], E, R)
    ev = (S.TransEEval if name == "transe" else S.HolEEval)(z["queries"].tolist(),
                                                            z["known"].tolist())
    pos, fpos = ev.positions(m)
    r = ev.last_ranks
    np.testing.assert_array_equal(r[:, 0], z["tail_raw"])
    np.testing.assert_array_equal(r[:, 1], z["tail_filt"])
    np.testing.assert_array_equal(r[:, 2], z["head_raw"])
    np.testing.assert_array_equal(r[:, 3], z["head_filt"])
    # the reference's structure: {p: {'head': [...], 'tail': [...]}}
    k = 0
    for p, sos in ev.idx.items():
        assert pos[p]["tail"] == z["tail_raw"][k:k + len(sos)].tolist()
        assert fpos[p]["head"] == z["head_filt"][k:k + len(sos)].tolist()
        k += len(sos)


@pytest.mark.parametrize("name,d", [("transe", 40), ("hole", 32), ("rescal", 24)])
def test_ranks_vs_oracle(name, d):
    import skge_amd as S
    rs = np.random.RandomState(4)
    n_ent, n_rel = 300, 5
    known = np.unique(np.stack([rs.randint(n_ent, size=3000), rs.randint(n_ent, size=3000),
                                rs.randint(n_rel, size=3000)], axis=1), axis=0).astype(np.int32)
    test = known[rs.choice(len(known), 120, replace=False)]
    m = _model(name, n_ent, n_rel, d)
    ev = S.FilteredRankingEval(test.tolist(), known.tolist())
    r = ev.ranks(m)
    q = np.asarray([(s, o, p) for p, sos in ev.idx.items() for (s, o) in sos])
    rid = "W" if name == "rescal" else "R"
    want = O.filtered_ranks(name, m.params["E"].data.cpu().numpy().astype(np.float64),
                            m.params[rid].data.cpu().numpy().astype(np.float64), q, known)
    # fp32 vs fp64 scores: a rank may move only if another entity ties the true
    # score to fp32 rounding; allow such rare near-ties
    diff = np.abs(r - want)
    assert (diff == 0).mean() >= 0.99, diff.max()
    assert diff.max() <= 2


def test_wn18_scale_ranking_runs():
    import skge_amd as S
    rs = np.random.RandomState(0)
    n_ent, n_rel = 40943, 18
    known = np.stack([rs.randint(n_ent, size=150000), rs.randint(n_ent, size=150000),
                      rs.randint(n_rel, size=150000)], axis=1).astype(np.int32)
    test = known[:5000]
    m = _model("transe", n_ent, n_rel, 200)
    ev = S.TransEEval(test.tolist(), known.tolist())
    torch.cuda.synchronize()
    r = ev.ranks(m)
    assert r.shape == (5000, 4)
    assert (r >= 1).all() and (r <= n_ent).all()
    assert (r[:, 1] <= r[:, 0]).all() and (r[:, 3] <= r[:, 2]).all()   # filtering only removes
    (mrr, mean, hits), (fmrr, fmean, fhits) = S.ranking_scores(*ev.positions(m))
    assert 0 < mrr <= fmrr <= 1


@pytest.mark.parametrize("name,d,n_ent", [("transe", 200, 3000), ("hole", 200, 3000),
                                          ("rescal", 37, 1500), ("transe", 30, 5000)])
def test_known_answer_ranks_equal_triple_set_ranks(name, d, n_ent, monkeypatch):
    """The all-entity pass over entity slices with the filter applied from the
    queries' known answers (skge_rank_known) against the triple-set form
    (skge_rank): identical positions, raw and filtered, both directions --
    incl. d % 4 != 0 and a KG dense enough that queries have many answers."""
    import skge_amd as S
    rs = np.random.RandomState(7)
    n_rel = 4
    known = np.unique(np.stack([rs.randint(n_ent // 10, size=20000), rs.randint(n_ent, size=20000),
                                rs.randint(n_rel, size=20000)], axis=1), axis=0).astype(np.int32)
    test = known[rs.choice(len(known), 700, replace=False)]
    m = _model(name, n_ent, n_rel, d)
    out = []
    for env in ("1", "0"):
        monkeypatch.setenv("SKGE_RANK_SET", env)
        ev = S.FilteredRankingEval(test.tolist(), known.tolist())
        out.append(ev.ranks(m))
    np.testing.assert_array_equal(out[0], out[1])
    assert (out[1][:, 1] < out[1][:, 0]).any()   # the filter removed some known answers
