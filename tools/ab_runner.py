#!/usr/bin/env python3
"""A/B of the TransE-L1 device runners (pipelined one-launch-per-batch vs
two-launch) at a given batch count, WN18 shape, d=200, AdaGrad: epochs/s
from the initial parameters.  Usage: python tools/ab_runner.py --nb 2 4 10 100"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scikit-kge_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nb", type=int, nargs="+", default=[2, 4, 10, 100])
    ap.add_argument("--epochs", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch
    import skge_amd as S
    from skge_amd.device import DeviceKG, EpochRunner
    from bench import make_wn18_kg, N_ENT, N_REL, N_TRIPLES
    dev = torch.device("cuda", 0)
    trip = make_wn18_kg()
    np.random.seed(42)
    m = S.TransE((N_ENT, N_ENT, N_REL), 200)
    m.add_hyperparam("margin", 2.0)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
    init = {pid: p.data.clone() for pid, p in m.params.items()}
    kg = DeviceKG(trip, dev)
    for nb in args.nb:
        for pipe in (True, False):
            r = EpochRunner(m, upd, kg, nbatches=nb, seed=7, pipelined=pipe)
            r.run(1)
            r.synchronize()
            for pid, p in m.params.items():
                p.data.copy_(init[pid])
                upd[pid].reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.run(args.epochs)
            r.synchronize()
            dt = (time.perf_counter() - t0) / args.epochs
            print("nb=%d %-10s %.1f M triples/s (%.3f ms/epoch)" % (
                nb, "pipelined" if r.pipelined else "two-launch", N_TRIPLES / dt / 1e6, dt * 1e3))
            del r


if __name__ == "__main__":
    main()
