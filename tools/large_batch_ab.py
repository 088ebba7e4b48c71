"""Large-batch runner A/B (diagnostics): WN18-shaped TransE-L1 d=200 AdaGrad
at --nb (default 2), the pipelined runner vs the two-launch runner, timed over
--steps epochs after --warmup (graph replays, events on the runner stream).
The two-launch runner's dense entity apply is selected by SKGE_APPLY_DENSE in
the environment of the whole process.  Prints one JSON line per runner."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scikit-kge_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nb", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--runners", default="pipelined,two-launch")
    args = ap.parse_args()
    import numpy as np
    import torch
    import skge_amd as S
    from skge_amd.device import DeviceKG, EpochRunner
    from bench import make_wn18_kg, N_ENT, N_REL
    dev = torch.device("cuda", 0)
    trip = make_wn18_kg()
    for name in args.runners.split(","):
        np.random.seed(42)
        m = S.TransE((N_ENT, N_ENT, N_REL), 200)
        m.add_hyperparam("margin", 2.0)
        upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
        kg = DeviceKG(trip, dev)
        r = EpochRunner(m, upd, kg, nbatches=args.nb, seed=7, pipelined=(name == "pipelined"))
        r.run(args.warmup)
        r.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(r.stream)
        r.run(args.steps)
        e1.record(r.stream)
        r.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        print(json.dumps({"runner": name, "nb": args.nb, "dense": os.environ.get("SKGE_APPLY_DENSE", "0"),
                          "ms_per_epoch": round(ms, 4),
                          "triples_per_s": round(kg.T / (ms * 1e-3), 1),
                          "pipelined": bool(r.pipelined)}), flush=True)
        del r, m, upd, kg
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
