#!/usr/bin/env python3
"""Filtered-ranking evaluation time at the WN18 geometry (5000 test triples,
|E|=40943, |R|=18, d=200; known triples = the synthetic KG): device
skge_rank vs the oracle (fp64 NumPy, the reference evaluators' arithmetic) on
a sample of queries, extrapolated.
Usage: python tools/bench_eval.py [--models transe,hole] [--cpu-queries 20]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scikit-kge_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="transe,hole")
    ap.add_argument("--cpu-queries", type=int, default=20)
    args = ap.parse_args()
    import numpy as np
    import torch
    import skge_amd as S
    from bench import make_wn18_kg, N_ENT, N_REL
    from oracle import skge_oracle as O
    trip = make_wn18_kg()
    test = trip[:5000]
    out = {}
    for name in args.models.split(","):
        np.random.seed(42)
        m = S.TransE((N_ENT, N_ENT, N_REL), 200) if name == "transe" else \
            S.HolE((N_ENT, N_ENT, N_REL), 200)
        ev = S.FilteredRankingEval(test, trip)
        ev.ranks(m)   # warm-up (also builds the known-triple set)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = ev.ranks(m)
        torch.cuda.synchronize()
        t_gpu = time.perf_counter() - t0
        E = m.params["E"].data.cpu().numpy().astype(np.float64)
        R = m.params["R"].data.cpu().numpy().astype(np.float64)
        q = np.asarray([(s, o, p) for p, sos in ev.idx.items() for (s, o) in sos])
        t0 = time.perf_counter()
        O.filtered_ranks(name, E, R, q[:args.cpu_queries], trip)
        t_cpu = (time.perf_counter() - t0) / args.cpu_queries * len(q)
        out[name] = {"queries": len(q), "gpu_s": round(t_gpu, 4), "cpu_oracle_s_est": round(t_cpu, 1),
                     "filtered_mrr": round(S.compute_scores(np.r_[r[:, 1], r[:, 3]])[0], 5)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
