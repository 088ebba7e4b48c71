#!/usr/bin/env python3
"""PCIe-inclusive rate of the reference-protocol boundary.

The drop-in path a reference user calls hands HOST buffers to the library:
per mini-batch, the pairs PairwiseStochasticTrainer._process_batch builds
(skge/base.py:1394-1427) arrive as host arrays, are copied to the device and
trained by model._pairwise_step (one fused skge_pair_step).  This times that
loop over one WN18-shaped epoch (TransE-L1 d=200 AdaGrad, nb=100) with the
pairs drawn beforehand by the reference-semantics host sampler (the sampler
itself is untimed, as in bench.py's cpu_baseline): host->device copy + step
per batch, synchronised at the end of the epoch.
Usage: python tools/bench_protocol.py [--epochs 3] [--model transe|hole|rescal]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scikit-kge_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--model", default="transe", choices=["transe", "hole", "rescal"])
    ap.add_argument("--d", type=int, default=200)
    ap.add_argument("--nb", type=int, default=100)
    args = ap.parse_args()
    import numpy as np
    import torch
    import skge_amd as S
    from bench import make_wn18_kg, N_ENT, N_REL
    from skge_amd.sample import RandomModeSampler
    dev = torch.device("cuda", 0)
    trip = make_wn18_kg()
    np.random.seed(42)
    sz = (N_ENT, N_ENT, N_REL)
    margin = 2.0 if args.model == "transe" else 0.2
    m = {"transe": lambda: S.TransE(sz, args.d), "hole": lambda: S.HolE(sz, args.d),
         "rescal": lambda: S.RESCAL(sz, args.d)}[args.model]()
    m.add_hyperparam("margin", margin)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
    xs = [tuple(t) for t in trip.tolist()]
    sampler = RandomModeSampler(1, [0, 1], xs, sz)   # skge/sample.py semantics, host RNG
    idx = np.arange(len(xs))
    np.random.shuffle(idx)
    bs = len(xs) // args.nb   # StochasticTrainer._optim's np.split geometry
    batches = []
    for a in range(0, len(xs), bs):
        pos, neg = [], []
        for j in idx[a:a + bs]:   # _process_batch: (x, nx) for each surviving negative
            for nx, _ in sampler.sample([(xs[j], 1.0)]):
                pos.append(xs[j])
                neg.append(nx)
        batches.append((np.ascontiguousarray(np.array(pos, dtype=np.int32)),
                        np.ascontiguousarray(np.array(neg, dtype=np.int32)),
                        len(idx[a:a + bs])))
    nv = torch.zeros(1, dtype=torch.int32, device=dev)
    times = []
    for e in range(args.epochs + 1):   # epoch 0: warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for pos, neg, _ in batches:
            m._pairwise_step(torch.from_numpy(pos).to(dev, non_blocking=False),
                             torch.from_numpy(neg).to(dev, non_blocking=False), upd, nv)
        torch.cuda.synchronize()
        if e:
            times.append(time.perf_counter() - t0)
    npos = sum(c for _, _, c in batches)
    best = min(times)
    print(json.dumps({"path": "reference protocol (host pairs -> H2D -> _pairwise_step per batch)",
                      "model": args.model, "d": args.d, "nbatches": args.nb,
                      "triples_per_s": round(npos / best, 1),
                      "ms_per_epoch": round(1e3 * best, 3),
                      "epochs_ms": [round(1e3 * t, 3) for t in times]}))


if __name__ == "__main__":
    main()
