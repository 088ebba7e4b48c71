"""Model files in the reference's pickle layout (skge/base.py:1170-1192).

The reference pickles a model as an instance of ``skge.<module>.<Class>``
whose state is ``{'hyperparams': {...}, 'params': {pid: Parameter}}``
(``Model.__getstate__`` base.py:1170-1174; ``save`` uses the highest protocol,
the experiment callback pickles ``{'model': m, 'pos test': ...}`` with
protocol 2, base.py:278-288).  This module reads and writes exactly that
layout, so a model trained on the device can be handed to the reference's
evaluation scripts, and a reference model file can be trained further here:

* ``reference_state_bytes`` / ``save_reference``: write a model as the
  reference would (class ``skge.transe.TransE`` etc., params as float64
  ndarrays, activation classes as ``skge.actfun.*``).  The reference's
  ``__setstate__`` (base.py:1176-1182) rebuilds it with ``add_param(...,
  value=p)``.  The pickle is produced without importing ``skge``: stand-in
  classes are registered under the reference's module names for the duration
  of the dump only.
* ``read_reference_state`` / ``load_reference``: read a reference model file
  (or a callback dict holding one under ``'model'``) with a restricted
  unpickler that resolves only the reference's model, activation and
  Parameter classes and numpy's array reconstruction -- nothing else in the
  file can name a callable.  Reference Parameters (ndarray subclasses) come
  back as plain float arrays.

The AdaGrad state is not part of the reference layout (its updaters are not
pickled); ``save_reference(..., updaters=...)`` can add it under the extra
key ``'adagrad'``, which the reference's ``__setstate__`` ignores.
"""
import contextlib
import io
import pickle
import sys
import types

import numpy as np

from . import actfun as AF

MODEL_MODULES = {"TransE": "skge.transe", "HolE": "skge.hole", "RESCAL": "skge.rescal"}
_ACTFUNS = ("ActivationFunction", "Linear", "Sigmoid", "Tanh", "ReLU", "Softplus")
_NUMPY_GLOBALS = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    ("numpy", "ndarray"), ("numpy", "dtype"),
    ("_codecs", "encode"),   # protocol 2 spells bytes as _codecs.encode(str, 'latin1')
}


# ---------------------------------------------------------------------------
# writing
# ---------------------------------------------------------------------------

class _StandinModel(object):
    """Instance pickled as skge.<module>.<Class> with the given state."""

    def __init__(self, state):
        self._state = state

    def __getstate__(self):
        return self._state


@contextlib.contextmanager
def _reference_names():
    """Register stand-in classes under the reference's module names, so the
    pickler writes GLOBAL 'skge.transe TransE' etc.; restore sys.modules after."""
    names = ["skge", "skge.actfun"] + sorted(set(MODEL_MODULES.values()))
    saved = {n: sys.modules.get(n) for n in names}
    mods = {n: types.ModuleType(n) for n in names}
    classes = {}
    for cname, mname in MODEL_MODULES.items():
        cls = type(cname, (_StandinModel,), {"__module__": mname})
        cls.__qualname__ = cname
        setattr(mods[mname], cname, cls)
        classes[cname] = cls
    for aname in _ACTFUNS:
        cls = type(aname, (object,), {"__module__": "skge.actfun"})
        cls.__qualname__ = aname
        setattr(mods["skge.actfun"], aname, cls)
        classes["af." + aname] = cls
    try:
        sys.modules.update(mods)
        yield classes
    finally:
        for n, m in saved.items():
            if m is None:
                sys.modules.pop(n, None)
            else:
                sys.modules[n] = m


def _export_value(v, classes):
    if isinstance(v, type) and issubclass(v, AF.ActivationFunction):
        return classes["af." + v.__name__]
    return v


def reference_state_bytes(class_name, hyperparams, params, extra=None, protocol=2):
    """Pickle bytes of a reference model: class skge.<module>.<class_name>,
    state {'hyperparams', 'params' (float64 ndarrays)} (+ `extra` keys)."""
    if class_name not in MODEL_MODULES:
        raise ValueError("no reference model class %r" % (class_name,))
    with _reference_names() as classes:
        state = {"hyperparams": {k: _export_value(v, classes) for k, v in hyperparams.items()},
                 "params": {pid: np.asarray(p, dtype=np.float64) for pid, p in params.items()}}
        if extra:
            state.update(extra)
        return pickle.dumps(classes[class_name](state), protocol=protocol)


def save_reference(model, fname, updaters=None, protocol=2):
    """Write `model` (an skge_amd model) as the reference's model pickle.
    With `updaters` (trainer._updaters), their AdaGrad state is added under
    'adagrad' (ignored by the reference)."""
    extra = None
    if updaters is not None:
        extra = {"adagrad": {pid: u.p2.detach().cpu().numpy().astype(np.float64)
                             for pid, u in updaters.items() if hasattr(u, "p2")}}
    data = reference_state_bytes(type(model).__name__, model.hyperparams,
                                 {pid: np.asarray(p) for pid, p in model.params.items()},
                                 extra=extra, protocol=protocol)
    with open(fname, "wb") as f:
        f.write(data)


# ---------------------------------------------------------------------------
# reading
# ---------------------------------------------------------------------------

class _LoadedModel(object):
    model_class = None

    def __setstate__(self, st):
        self.state = st


class _RefUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if MODEL_MODULES.get(name) == module:
            return type(name, (_LoadedModel,), {"model_class": name})
        if module == "skge.actfun" and name in _ACTFUNS:
            return getattr(AF, name)
        if module == "skge.param" and name == "Parameter":
            return np.ndarray
        if (module, name) in _NUMPY_GLOBALS:
            return getattr(sys.modules[module] if module in sys.modules else
                           __import__(module, fromlist=[name]), name)
        raise pickle.UnpicklingError("reference model file names %s.%s, which is not a "
                                     "reference model, activation or array type" % (module, name))


def read_reference_state(data):
    """(class name, hyperparams, params {pid: float64 ndarray}, state) of a
    reference model pickle (bytes or file object).  A callback dict
    (skge/base.py:278-288) is accepted: its 'model' entry is read."""
    f = io.BytesIO(data) if isinstance(data, (bytes, bytearray)) else data
    obj = _RefUnpickler(f).load()
    if isinstance(obj, dict) and "model" in obj:
        obj = obj["model"]
    if not isinstance(obj, _LoadedModel):
        raise ValueError("not a reference model pickle (got %s)" % type(obj).__name__)
    st = obj.state
    params = {pid: np.asarray(p, dtype=np.float64) for pid, p in st["params"].items()}
    return obj.model_class, dict(st["hyperparams"]), params, st


def load_reference(fname):
    """Build an skge_amd model (parameters on the GPU) from a reference model
    file written by skge's Model.save or experiment callback."""
    from .hole import HolE
    from .rescal import RESCAL
    from .transe import TransE
    with open(fname, "rb") as f:
        cname, hp, params, _ = read_reference_state(f)
    cls = {"TransE": TransE, "HolE": HolE, "RESCAL": RESCAL}[cname]
    m = cls.__new__(cls)
    m.__setstate__({"hyperparams": hp, "params": params})
    return m
