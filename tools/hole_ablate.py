#!/usr/bin/env python3
"""Time skge_pair_grad for HolE d=200 on a WN18-sized batch (2828 pairs):
score only (margin -inf), all violating (margin +1e9: 8 correlations +
contribution atomics), and the apply; HIP events on the current stream."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scikit-kge_amd"))
import skge_amd as S  # noqa: E402
from skge_amd import _lib as L  # noqa: E402

N, M, d, P = 40943, 18, int(os.environ.get("D", "200")), 2828
np.random.seed(42)
m = S.HolE((N, N, M), d)
m.add_hyperparam("margin", 0.2)
dev = m.device
rs = np.random.RandomState(0)
pos = torch.tensor(np.stack([rs.randint(N, size=P), rs.randint(N, size=P), rs.randint(M, size=P)], 1),
                   dtype=torch.int32, device=dev)
neg = pos.clone()
neg[:, 0] = torch.tensor(rs.randint(N, size=P), dtype=torch.int32, device=dev)
lib = L.lib()
upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


nv = torch.zeros(1, dtype=torch.int32, device=dev)
te, tr = m._tables("pairwise", upd, slots=m._pair_slots(P))
tabs = (L.SkgeTable * 2)(te, tr)


def grad(margin):
    def f():
        L.check(lib.skge_pair_grad(L.stream_ptr(), L.SKGE_HOLE, m._af_code(), te, tr, d, L.ptr(pos),
                                   L.ptr(neg), P, margin, None, None, None, L.ptr(nv)))
        L.check(lib.skge_accum_reset(L.stream_ptr(), te, 4 * P))
        L.check(lib.skge_accum_reset(L.stream_ptr(), tr, 2 * P))
    return f


def reset_only():
    L.check(lib.skge_accum_reset(L.stream_ptr(), te, 4 * P))
    L.check(lib.skge_accum_reset(L.stream_ptr(), tr, 2 * P))


def step():
    nv.zero_()
    m._pairwise_step(pos, neg, upd, nv)


t_reset = timeit(reset_only)
print("reset only          %.1f us" % t_reset)
print("score only (-inf)   %.1f us" % (timeit(grad(float("-inf"))) - t_reset))
print("all violate + atom  %.1f us" % (timeit(grad(1e9)) - t_reset))
print("margin 0.2 grad     %.1f us" % (timeit(grad(0.2)) - t_reset))
print("full pair_step      %.1f us (nviol %d)" % (timeit(step), int(nv.item())))
