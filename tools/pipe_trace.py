#!/usr/bin/env python3
"""Per-wave timeline of one pipelined batch launch (diagnostics).

Runs the WN18-shaped bench workload, warms up, then profiles one epoch with
s_memrealtime stamps (10 ns) recorded by every wave of batch launch --launch.
Prints percentiles of each scoring-wave phase and of the apply waves,
relative to the earliest wave start.
Usage: python tools/pipe_trace.py [--launch 50] [--warmup 2]
"""
import argparse
import json
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
    ap.add_argument("--skew", choices=("none", "zipf"), default="none")
    args = ap.parse_args()
    import numpy as np
    import torch
    import skge_amd as S
    from skge_amd.device import DeviceKG, EpochRunner
    from bench import make_wn18_kg, make_zipf_kg, N_ENT, N_REL
    dev = torch.device("cuda", 0)
    trip = make_zipf_kg() if args.skew == "zipf" else make_wn18_kg()
    np.random.seed(42)
    m = S.TransE((N_ENT, N_ENT, N_REL), args.d)
    m.add_hyperparam("margin", 2.0)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
    kg = DeviceKG(trip, dev)
    r = EpochRunner(m, upd, kg, nbatches=args.nb, seed=5)
    r.run(args.warmup)
    r.synchronize()
    for rep in range(2):
        us, stats, tr = r.profile(trace_launch=args.launch)
        r.synchronize()
        nb_, na = int(tr[0]), int(tr[1])
        B = tr[2:2 + 6 * nb_].reshape(nb_, 6).astype(np.int64)
        A = tr[2 + 6 * nb_:2 + 6 * nb_ + 2 * na].reshape(na, 2).astype(np.int64)
        A = A[A[:, 0] > 0]
        t0 = min(B[:, 0].min(), A[:, 0].min() if len(A) else B[:, 0].min())
        pend = (B[:, 5] & 0x1f)
        viol = (B[:, 5] >> 8) & 1
        print("launch %d: event %.2f us, B waves %d (viol %d, pending entity rows: any %d, "
              "1 %d, 2+ %d), A waves %d, stats %s" % (
                  args.launch, us[args.launch], nb_, viol.sum(), (pend != 0).sum(),
                  (np.array([bin(int(x)).count("1") for x in pend]) == 1).sum(),
                  (np.array([bin(int(x)).count("1") for x in pend]) >= 2).sum(), len(A),
                  stats[args.launch].tolist()))
        print("percentiles (us)           p0     p10    p50    p90    p100")
        print("B start                  ", pct(B[:, 0] - t0))
        # (k_pipe_fused: "rows+marks" = record, rows, meta, the item's apply rows and
        # the relation row; "settle" = the item's applies + the pending rows' updates)
        print("B rows+marks (ballot)    ", pct(B[:, 1] - B[:, 0]))
        print("B settle (pending)       ", pct((B[:, 2] - B[:, 1])[pend != 0]))
        print("B settle (none pending)  ", pct((B[:, 2] - B[:, 1])[pend == 0]))
        print("B score (incl row wait)  ", pct(B[:, 3] - B[:, 2]))
        print("B atomics issue (viol)   ", pct((B[:, 4] - B[:, 3])[viol == 1]))
        print("B issue end             ", pct(B[:, 4] - t0))
        if len(A):
            print("A start                  ", pct(A[:, 0] - t0))
            print("A duration               ", pct(A[:, 1] - A[:, 0]))
            print("A end                    ", pct(A[:, 1] - t0))
        print("last end %.2f us" % ((max(B[:, 4].max(), A[:, 1].max() if len(A) else 0) - t0) / 100))


if __name__ == "__main__":
    main()
