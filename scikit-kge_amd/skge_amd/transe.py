"""TransE (mirrors skge/transe.py): score -||E[s] + R[p] - E[o]||_1 (or the
squared L2 norm), pairwise margin gradients.  The scoring, margin test,
sign sub-gradients and segment sums of ``_pairwise_gradients``
(skge/transe.py:48-165) run in skge_pair_grad (csrc/skge_grad.hip)."""
import logging

from . import _lib as L
from .base import Model
from .param import normalize

log = logging.getLogger("EX-KG")


class TransE(Model):
    """Translational Embeddings of Knowledge Graphs (skge/transe.py:9-23)."""
    default_posts = {"E": normalize}   # posts restored when loading a reference file
    rel_id = "R"

    def __init__(self, *args, **kwargs):
        super(TransE, self).__init__(*args, **kwargs)
        self.add_hyperparam("sz", args[0])
        self.add_hyperparam("ncomp", args[1])
        self.add_hyperparam("l1", kwargs.pop("l1", True))
        self.add_param("E", (self.sz[0], self.ncomp), post=normalize)
        self.add_param("R", (self.sz[2], self.ncomp))

    def _kernel_model(self):
        return L.SKGE_TRANSE_L1 if self.l1 else L.SKGE_TRANSE_L2

    def _gradients(self, xys):
        raise NotImplementedError("TransE has no logistic loss in the reference")
