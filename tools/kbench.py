#!/usr/bin/env python3
"""Fixed-workload kernel timing for the TransE device batch loop.

Times, at the WN18 geometry (B = 1414 positives, d = 200), inside hipGraphs of
N back-to-back launches:
  sample_all   skge_transe_sample_grad, every pair violating (margin +1e9)
  sample_none  skge_transe_sample_grad, no pair violating    (margin -1e9)
  pair_all     sample_grad (all violating) + skge_accum_apply
so apply = pair_all - sample_all.  Parameters do not change between launches
(no apply, or an apply whose effect is irrelevant for timing), so variants of
the library (SKGE_LIB_PATH) are compared on identical work.
Usage: python tools/kbench.py [--acc auto|f32] [--n 100]
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
    ap.add_argument("--acc", default="auto")
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--d", type=int, default=200)
    ap.add_argument("--nb", type=int, default=100)
    args = ap.parse_args()
    import numpy as np
    import torch
    import skge_amd as S
    from skge_amd import _lib as L
    from skge_amd.device import DeviceKG, EpochRunner
    from bench import make_wn18_kg, N_ENT, N_REL
    dev = torch.device("cuda", 0)
    trip = make_wn18_kg()
    np.random.seed(42)
    m = S.TransE((N_ENT, N_ENT, N_REL), args.d)
    m.add_hyperparam("margin", 2.0)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
    kg = DeviceKG(trip, dev)
    r = EpochRunner(m, upd, kg, nbatches=args.nb, seed=5, force_f32=args.acc == "f32")
    st = r.stream
    lib = L.lib()
    sp = L.stream_ptr(st)
    B = kg.T // args.nb
    tabs = (L.SkgeTable * 2)(r.te, r.tr)
    ns = L.int_array(4 * B, B)

    def sample(margin, start):
        L.check(lib.skge_transe_sample_grad(sp, 1, r.te, r.tr, args.d, L.ptr(kg.trip), kg.T,
                                            L.ptr(kg.slots), kg.capacity, start, B, 9,
                                            L.ptr(r.epoch_key), margin, 100, None, None, None))

    def apply():
        L.check(lib.skge_accum_apply(sp, tabs, 2, ns))

    def timed(fn):
        with torch.cuda.stream(st):
            for i in range(5):
                fn(i)
            st.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                for i in range(args.n):
                    fn(i)
            g.replay()
            st.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(st)
            g.replay()
            e1.record(st)
            st.synchronize()
            return e0.elapsed_time(e1) * 1e3 / args.n

    res = {}
    res["sample_none"] = timed(lambda i: sample(-1e9, (i % args.nb) * B))
    res["sample_all"] = timed(lambda i: sample(1e9, (i % args.nb) * B))
    res["pair_all"] = timed(lambda i: (sample(1e9, (i % args.nb) * B), apply()))
    res["apply_est"] = res["pair_all"] - res["sample_all"]
    res["packed"] = r.packed
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
