"""Negative samplers (mirrors skge/sample.py).

RandomModeSampler here is the reference's host sampler, statement for
statement (same numpy global RNG stream, so a seeded run draws the same
negatives as the reference).  The throughput path samples on the device
instead (skge_transe_sample_grad, used by PairwiseStochasticTrainer with
device_loop=True)."""
from numpy.random import randint


class Sampler(object):
    """skge/sample.py:11-25"""

    def __init__(self, n, modes, ntries=100):
        self.n = n
        self.modes = modes
        self.ntries = ntries

    def sample(self, xys):
        res = []
        for x, _ in xys:
            for _ in range(self.n):
                for mode in self.modes:
                    t = self._sample(x, mode)
                    if t is not None:
                        res.append(t)
        return res


class RandomModeSampler(Sampler):
    """Corrupt s (mode 0) or o (mode 1) with up to ntries rejection draws
    against the training set (skge/sample.py:28-46)."""

    def __init__(self, n, modes, xs, sz):
        super(RandomModeSampler, self).__init__(n, modes)
        self.xs = set(tuple(int(v) for v in x) for x in xs)
        self.sz = sz

    def _sample(self, x, mode):
        nex = list(x)
        res = None
        for _ in range(self.ntries):
            nex[mode] = randint(self.sz[mode])
            if tuple(nex) not in self.xs:
                res = (tuple(nex), -1.0)
                break
        return res
