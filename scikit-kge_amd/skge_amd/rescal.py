"""RESCAL (mirrors skge/rescal.py): score E[s] . (W[p] E[o]).

Entity part of the gradients -> skge_pair_grad / skge_triple_grad; the d x d
relation gradient -> skge_rescal_wgrad.  Reference quirks kept: in the
pairwise loss dW uses ALL pairs and is divided by 2 (skge/rescal.py:113-125)
and rparam sits inside the entity mean (rescal.py:299-302); in the logistic
loss rparam is added outside the means (rescal.py:70, 239)."""
from . import _lib as L
from . import actfun as af
from .base import Model


class RESCAL(Model):
    model_code = L.SKGE_RESCAL
    rel_id = "W"

    def __init__(self, *args, **kwargs):
        super(RESCAL, self).__init__(*args, **kwargs)
        self.add_hyperparam("sz", args[0])
        self.add_hyperparam("ncomp", args[1])
        self.add_hyperparam("rparam", kwargs.pop("rparam", 0.0))
        aff = kwargs.pop("af", "linear")
        self.add_hyperparam("af", af.afuns[aff])
        self.add_param("E", (self.sz[0], self.ncomp))
        self.add_param("W", (self.sz[2], self.ncomp, self.ncomp))

    def _af_code(self):
        return af.af_code(self.af)

    def _reg(self, mode):
        r = float(self.rparam)
        if mode == "pairwise":
            return {"E": (r, 0.0, 0.0), "W": (r, 0.0, 2.0)}
        return {"E": (0.0, r, 0.0), "W": (0.0, r, 0.0)}
