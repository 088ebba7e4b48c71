"""HolE (mirrors skge/hole.py): score sum_k R[p]_k ccorr(E[s], E[o])_k.

_gradients (logistic, skge/hole.py:22-42) -> skge_triple_grad;
_pairwise_gradients (skge/hole.py:44-100) -> skge_pair_grad.  Circular
correlation / convolution are evaluated directly in LDS by the kernels."""
from . import _lib as L
from . import actfun as af
from .base import Model
from .param import normless1


class HolE(Model):
    default_posts = {"E": normless1}   # posts restored when loading a reference file
    model_code = L.SKGE_HOLE
    rel_id = "R"

    def __init__(self, *args, **kwargs):
        super(HolE, self).__init__(*args, **kwargs)
        self.add_hyperparam("sz", args[0])
        self.add_hyperparam("ncomp", args[1])
        self.add_hyperparam("rparam", kwargs.pop("rparam", 0.0))
        self.add_hyperparam("af", kwargs.pop("af", af.Sigmoid))
        self.add_param("E", (self.sz[0], self.ncomp), post=normless1)
        self.add_param("R", (self.sz[2], self.ncomp))

    def _af_code(self):
        return af.af_code(self.af)

    def _reg(self, mode):
        # pairwise: dR += rparam*R (hole.py:83), dE has none (hole.py:98)
        # logistic: both + rparam * param outside the mean (hole.py:33, 40)
        r = float(self.rparam)
        if mode == "pairwise":
            return {"E": (0.0, 0.0, 0.0), "R": (0.0, r, 0.0)}
        return {"E": (0.0, r, 0.0), "R": (0.0, r, 0.0)}
