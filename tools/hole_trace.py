#!/usr/bin/env python3
"""Per-wave timeline of one pipelined HolE batch launch (diagnostics).

The config-3 bench workload (WN18 shape, HolE d=200, AdaGrad, margin 0.2,
nb=100) on HolePipeRunner: warm up, then one eager epoch with HIP events
around every launch and s_memrealtime stamps (10 ns) from every wave of
launch --launch (k_hole_pipe's trace hooks).  Prints the per-launch event
durations and percentiles of each scoring-wave phase and of the apply waves,
relative to the earliest wave start.
Usage: python tools/hole_trace.py [--launch 50] [--warmup 2]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scikit-kge_amd"))
sys.path.insert(0, ROOT)


def pct(x):
    import numpy as np
    if len(x) == 0:
        return "-"
    q = np.percentile(x, [0, 10, 50, 90, 100]) / 100.0   # 10 ns ticks -> us
    return " ".join("%6.2f" % v for v in q)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launch", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--d", type=int, default=200)
    ap.add_argument("--nb", type=int, default=100)
    args = ap.parse_args()
    import numpy as np
    import torch
    import skge_amd as S
    from skge_amd.device import DeviceKG, HolePipeRunner
    from bench import make_wn18_kg, N_ENT, N_REL
    dev = torch.device("cuda", 0)
    trip = make_wn18_kg()
    np.random.seed(42)
    m = S.HolE((N_ENT, N_ENT, N_REL), args.d)
    m.add_hyperparam("margin", 0.2)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
    kg = DeviceKG(trip, dev)
    r = HolePipeRunner(m, upd, kg, args.nb, seed=5)
    r.run(args.warmup)
    r.synchronize()
    for rep in range(2):
        us, stats, tr = r.profile(trace_launch=args.launch)
        r.synchronize()
        print("per-launch event us: p10 %.2f p50 %.2f p90 %.2f sum %.1f (launches %d)" % (
            np.percentile(us[1:-1], 10), np.percentile(us[1:-1], 50),
            np.percentile(us[1:-1], 90), us.sum(), len(us)))
        nb_, na = int(tr[0]), int(tr[1])
        B = tr[2:2 + 6 * nb_].reshape(nb_, 6).astype(np.int64)
        inv = B[:, 5] >> 16                   # violating: inverse-transform phase (10 ns ticks)
        B[:, 5] = B[:, 5] & 0xffff
        A = tr[2 + 6 * nb_:2 + 6 * nb_ + 2 * na].reshape(na, 2).astype(np.int64)
        A = A[A[:, 0] > 0]
        t0 = min(B[:, 0].min(), A[:, 0].min() if len(A) else B[:, 0].min())
        pend = B[:, 5] & 0xf
        viol = (B[:, 5] >> 8) & 1
        v0 = (B[:, 5] >> 9) & 1
        v1 = (B[:, 5] >> 10) & 1
        print("launch %d: event %.2f us, B waves %d (violating positives %d: v0 only %d, "
              "v1 only %d, both %d; waves with pending rows %d), A waves %d" % (
                  args.launch, us[args.launch], nb_, viol.sum(), (v0 & (1 - v1)).sum(),
                  (v1 & (1 - v0)).sum(), (v0 & v1).sum(), (pend != 0).sum(), len(A)))
        print("percentiles (us)           p0     p10    p50    p90    p100")
        print("B start                  ", pct(B[:, 0] - t0))
        print("B record+rows+marks      ", pct(B[:, 1] - B[:, 0]))
        print("B settle (pending)       ", pct((B[:, 2] - B[:, 1])[pend != 0]))
        print("B settle (none pending)  ", pct((B[:, 2] - B[:, 1])[pend == 0]))
        print("B stage+2 corr+scores    ", pct(B[:, 3] - B[:, 2]))
        print("B rows+atomics (viol)    ", pct((B[:, 4] - B[:, 3])[viol == 1]))
        print("  of which H + inverse   ", pct(inv[viol == 1]))
        print("  then rows' atomics     ", pct((B[:, 4] - B[:, 3] - inv)[viol == 1]))
        print("B end (not violating)    ", pct((B[:, 4] - t0)[viol == 0]))
        print("B end (violating)        ", pct((B[:, 4] - t0)[viol == 1]))
        if len(A):
            print("A start                  ", pct(A[:, 0] - t0))
            print("A duration               ", pct(A[:, 1] - A[:, 0]))
            print("A end                    ", pct(A[:, 1] - t0))
        print("last end %.2f us" % ((max(B[:, 4].max(), A[:, 1].max() if len(A) else 0) - t0) / 100))


if __name__ == "__main__":
    main()
