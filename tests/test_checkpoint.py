"""Model files in the reference's pickle layout (skge/base.py:1170-1192,
278-288): the fixtures tests/golden/ckpt_*.pkl were written by the reference's
own Model.save / callback pickler (tools/gen_golden_ckpt.py, which also checks
that the reference reads skge_amd's files).  Read here only through the
restricted unpickler of skge_amd.checkpoint."""
import io
import os
import pickle
import pickletools

import numpy as np
import pytest

from golden_util import GOLDEN

MODELS = ("transe", "hole", "rescal")


def _fixture(name):
    z = np.load(os.path.join(GOLDEN, "ckpt_%s.npz" % name), allow_pickle=False)
    return {k: z[k] for k in z.files}


def _globals(data):
    """'module name' of every GLOBAL (protocol <= 3) and STACK_GLOBAL
    (protocol >= 4: the two strings pushed just before it; the reference's
    own writer never memo-fetches them) in a pickle."""
    out, strs = set(), []
    for op, arg, _ in pickletools.genops(io.BytesIO(data)):
        if op.name == "GLOBAL":
            out.add(arg)
        elif op.name in ("SHORT_BINUNICODE", "BINUNICODE", "UNICODE"):
            strs.append(arg)
        elif op.name == "STACK_GLOBAL":
            out.add("%s %s" % (strs[-2], strs[-1]))
    return out


@pytest.mark.parametrize("cb", [False, True])
@pytest.mark.parametrize("name", MODELS)
def test_read_reference_model_file(name, cb):
    from skge_amd import actfun
    from skge_amd.checkpoint import read_reference_state
    fx = _fixture(name)
    path = os.path.join(GOLDEN, "ckpt_%s%s.pkl" % (name, "_cb" if cb else ""))
    with open(path, "rb") as f:
        cname, hp, params, _ = read_reference_state(f)
    assert cname == str(fx["class_name"])
    pids = sorted(k[len("param_"):] for k in fx if k.startswith("param_"))
    assert sorted(params) == pids
    for pid in pids:
        assert params[pid].dtype == np.float64
        np.testing.assert_array_equal(params[pid], fx["param_" + pid])
    for k, v in fx.items():
        if k.startswith("hp_") and k != "hp_af_class":
            want = v.tolist()
            got = hp[k[3:]]
            assert (list(got) if isinstance(got, tuple) else got) == want, k
    if "hp_af_class" in fx:
        assert hp["af"] is getattr(actfun, str(fx["hp_af_class"]))


@pytest.mark.parametrize("name", MODELS)
def test_written_file_matches_reference_layout(name):
    from skge_amd import actfun
    from skge_amd.checkpoint import read_reference_state, reference_state_bytes
    fx = _fixture(name)
    with open(os.path.join(GOLDEN, "ckpt_%s.pkl" % name), "rb") as f:
        ref_bytes = f.read()
    _, hp, params, _ = read_reference_state(ref_bytes)
    ours = reference_state_bytes(str(fx["class_name"]), hp, params)
    # same model class global as the reference's own file, and the activation
    # class (HolE) under skge.actfun
    model_global = [g for g in _globals(ref_bytes) if g.startswith("skge.") and
                    not g.startswith(("skge.param", "skge.actfun"))]
    assert model_global and set(model_global) <= _globals(ours)
    assert all(g.startswith(("skge.", "numpy", "_codecs ")) for g in _globals(ours)), _globals(ours)
    if "hp_af_class" in fx:
        assert "skge.actfun %s" % fx["hp_af_class"] in _globals(ours)
    # round trip
    cname, hp2, params2, _ = read_reference_state(ours)
    assert cname == str(fx["class_name"])
    for pid in params:
        np.testing.assert_array_equal(params2[pid], params[pid])
    assert hp2 == hp
    assert all(not isinstance(v, type) or issubclass(v, actfun.ActivationFunction)
               for v in hp2.values())


def test_restricted_unpickler_rejects_other_globals():
    from skge_amd.checkpoint import read_reference_state
    evil = b"\x80\x02cos\nsystem\nq\x00X\x04\x00\x00\x00trueq\x01\x85q\x02Rq\x03."
    with pytest.raises(pickle.UnpicklingError):
        read_reference_state(evil)
    with pytest.raises(ValueError):
        read_reference_state(pickle.dumps({"model": 3}, protocol=2))
