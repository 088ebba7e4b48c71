"""Model files on the device (GPU): a reference model file loads into a
device model with the reference's posts, trains, and is written back in the
reference layout; skge_amd's own Model.save / load round-trips."""
import os

import numpy as np
import pytest
import torch

from golden_util import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["transe", "hole", "rescal"])
def test_load_reference_file_then_save_back(name, tmp_path):
    import skge_amd as S
    from skge_amd.checkpoint import read_reference_state
    z = np.load(os.path.join(GOLDEN, "ckpt_%s.npz" % name), allow_pickle=False)
    m = S.load_reference(os.path.join(GOLDEN, "ckpt_%s.pkl" % name))
    assert type(m).__name__ == str(z["class_name"])
    for pid, p in m.params.items():
        assert p.data.is_cuda
        np.testing.assert_array_equal(np.asarray(p), z["param_" + pid].astype(np.float32))
    want_post = {"transe": S.normalize, "hole": S.normless1, "rescal": None}[name]
    assert m.E.post is want_post
    # one device training step from the loaded state, then write it back
    m.add_hyperparam("margin", 0.5)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
    pos = torch.tensor([[0, 1, 0], [2, 3, 1], [4, 5, 2]], dtype=torch.int32, device=m.device)
    neg = torch.tensor([[6, 1, 0], [2, 7, 1], [8, 5, 2]], dtype=torch.int32, device=m.device)
    nv = torch.zeros(1, dtype=torch.int32, device=m.device)
    m._pairwise_step(pos, neg, upd, nv)
    out = tmp_path / "model.pkl"
    m.save_reference(str(out), updaters=upd)
    with open(out, "rb") as f:
        cname, hp, params, st = read_reference_state(f)
    assert cname == type(m).__name__
    for pid, p in m.params.items():
        np.testing.assert_array_equal(params[pid], np.asarray(p).astype(np.float64))
        np.testing.assert_array_equal(st["adagrad"][pid], upd[pid].p2.cpu().numpy())
    assert hp["margin"] == 0.5


def test_own_save_load_round_trip(tmp_path):
    import skge_amd as S
    np.random.seed(42)
    m = S.HolE((30, 30, 4), 16, rparam=0.1)
    f = tmp_path / "m.pkl"
    m.save(str(f))
    m2 = S.Model.load(str(f))
    assert type(m2) is S.HolE and m2.E.post is S.normless1 and m2.rparam == 0.1
    for pid in m.params:
        torch.testing.assert_close(m2.params[pid].data, m.params[pid].data, rtol=0, atol=0)
