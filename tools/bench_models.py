#!/usr/bin/env python3
"""Per-batch GPU time of the fused explicit-pair training step (skge_pair_step)
for every model at the WN18 geometry:
|E|=40943, |R|=18, d=200, B=1414 positives -> P=2828 pairs (RandomModeSampler
modes 0 and 1), AdaGrad lr 0.1.  Batches are pre-sampled on the host, the
steps are captured in a CUDA graph and replayed (HIP events on the stream).
Usage: python tools/bench_models.py [--models transe,hole,rescal] [--nb 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scikit-kge_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="transe,hole,rescal")
    ap.add_argument("--nb", type=int, default=20, help="batches per graph")
    ap.add_argument("--d", type=int, default=200)
    ap.add_argument("--B", type=int, default=1414)
    args = ap.parse_args()
    import numpy as np
    import torch
    import skge_amd as S
    from bench import make_wn18_kg, N_ENT, N_REL
    dev = torch.device("cuda", 0)
    trip = make_wn18_kg()
    rs = np.random.RandomState(1)
    B, d = args.B, args.d
    pos_b, neg_b = [], []
    for k in range(args.nb):
        idx = rs.randint(len(trip), size=B)
        p = trip[idx]
        n0, n1 = p.copy(), p.copy()
        n0[:, 0] = rs.randint(N_ENT, size=B)   # mode 0 corrupts s
        n1[:, 1] = rs.randint(N_ENT, size=B)   # mode 1 corrupts o
        pos_b.append(torch.from_numpy(np.concatenate([p, p])).to(dev).contiguous())
        neg_b.append(torch.from_numpy(np.concatenate([n0, n1])).to(dev).contiguous())
    out = {}
    for name in args.models.split(","):
        np.random.seed(42)
        if name == "transe":
            m = S.TransE((N_ENT, N_ENT, N_REL), d)
            m.add_hyperparam("margin", 2.0)
        elif name == "hole":
            m = S.HolE((N_ENT, N_ENT, N_REL), d)
            m.add_hyperparam("margin", 0.2)
        else:
            m = S.RESCAL((N_ENT, N_ENT, N_REL), d)
            m.add_hyperparam("margin", 0.2)
        upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
        nviol = torch.zeros(1, dtype=torch.int32, device=dev)
        st = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(st):
            for k in range(args.nb):   # warm-up: allocations, first touches
                nviol.zero_()
                m._pairwise_step(pos_b[k], neg_b[k], upd, nviol)
            st.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                for k in range(args.nb):
                    nviol.zero_()
                    m._pairwise_step(pos_b[k], neg_b[k], upd, nviol)
            g.replay()
            st.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            g.replay()
            e1.record(st)
            st.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.nb
        out[name] = {"us_per_batch": round(us, 2), "pos_triples_per_s": round(B / (us * 1e-6)),
                     "pairs": 2 * B, "d": d}
        del g
    print(json.dumps(out))


if __name__ == "__main__":
    main()
