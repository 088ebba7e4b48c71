"""skge_amd -- MI355X-native (HIP/gfx950) scikit-kge training hot path.

Drop-in for skge's model / updater / trainer protocol: TransE, HolE, RESCAL,
StochasticTrainer, PairwiseStochasticTrainer, SGD, AdaGrad,
RandomModeSampler.  Every numeric step runs in libskgehip.so."""
from .version import __version__
from .base import Model, StochasticTrainer, PairwiseStochasticTrainer, set_deterministic, deterministic
from .transe import TransE
from .hole import HolE
from .rescal import RESCAL
from .param import Parameter, SGD, AdaGrad, normalize, normless1
from .sample import RandomModeSampler
from .eval import FilteredRankingEval, TransEEval, HolEEval, compute_scores, ranking_scores
from .checkpoint import save_reference, load_reference, read_reference_state
