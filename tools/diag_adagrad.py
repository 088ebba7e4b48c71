"""Diagnostic: where the fp32 device step departs from the fp64 oracle after
AdaGrad (tests/test_gpu_runner_oracle.py geometry).  For the elements using
more than half the parity budget prints the error, the AdaGrad divisor H,
the oracle's gradient element and its row's norm (from the oracle's own
gradient rows), so the gradient-rounding term of the tolerance can be sized."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "scikit-kge_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import test_gpu_runner_oracle as T   # noqa: E402
from oracle import skge_oracle as O  # noqa: E402


def main(kind):
    import skge_amd as S
    from skge_amd.device import batch_sizes, epoch_records
    name, ckw, margin, okw = T.CASES[kind]
    m, upd, kg = T._setup(getattr(S, name), T.B, "adagrad", **ckw)
    m.add_hyperparam("margin", margin)
    r = T._runner(kind, m, upd, kg, 1, 41)
    with torch.cuda.stream(r.stream):
        for e in range(2):
            params, state = T._snapshot(m, upd)
            p2_before = {k: v.copy() for k, v in state.items()}
            rec, n1 = epoch_records(kg, T.N, 41, e)
            rec, n1 = rec.cpu().numpy(), n1.cpu().numpy()
            r.run(1)
            r.synchronize()
            pos, neg = T._pairs(rec, n1, 0, T.B)
            _, _, nv, grads = O.pairwise_step(kind, params, state, pos, neg, 0.1, float(m.margin),
                                              "adagrad", **okw)
            g, idx = grads["E"]
            got = m.E.data.cpu().numpy().astype(np.float64)
            want = params["E"]
            H = np.maximum(np.sqrt(state["E"]), 1e-7)
            tol = 1e-5 + 1e-5 * np.abs(want) + 0.1 * 1e-8 / H
            err = np.abs(got - want)
            ratio = err / tol
            print("%s e%d: nviol %d, max ratio %.3f, elements > 0.5: %d" % (
                kind, e, nv, ratio.max(), int((ratio > 0.5).sum())))
            gfull = np.zeros_like(want)
            gfull[idx] = g
            rown = np.zeros(want.shape[0])
            rown[idx] = np.sqrt((g ** 2).sum(axis=1))
            bad = np.argwhere(ratio > 0.5)
            for i, j in bad[np.argsort(-ratio[ratio > 0.5])][:12]:
                print("  row %6d col %3d err %.3g tol %.3g H %.3g p2_before %.3g g %.3g |g_row| %.3g "
                      "err*H/lr %.3g" % (i, j, err[i, j], tol[i, j], H[i, j], p2_before["E"][i, j],
                                         gfull[i, j], rown[i], err[i, j] * H[i, j] / 0.1))


if __name__ == "__main__":
    for k in sys.argv[1:] or ["hole", "rescal"]:
        main(k)
