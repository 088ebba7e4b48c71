"""The data-parallel epoch at world size 1 under "nccl" (RCCL; the epoch and
its all-gathers captured in one graph) against the one-GPU pipelined
runner's epoch, same WN18-shaped KG, model and batches (nb = 100): the
protocol's own overhead (the exchange and the record writes), in one JSON
line.  Run as one process: python tools/dp_world1.py [--steps 20]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scikit-kge_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--nb", type=int, default=100)
    ap.add_argument("--d", type=int, default=200)
    args = ap.parse_args()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29533"),
                      WORLD_SIZE="1", RANK="0")
    import numpy as np
    import torch
    import torch.distributed as dist
    import skge_amd as S
    from skge_amd.device import DeviceKG, EpochRunner
    from skge_amd.dp import DataParallelRunner
    from bench import make_wn18_kg, N_ENT, N_REL
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="env://")
    dev = torch.device("cuda", 0)
    trip = make_wn18_kg()
    kg = DeviceKG(trip, dev)
    out = {}
    for name in ("pipelined_1gpu", "dp_world1_nccl"):
        np.random.seed(42)
        m = S.TransE((N_ENT, N_ENT, N_REL), args.d)
        m.add_hyperparam("margin", 2.0)
        upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
        init = {pid: p.data.clone() for pid, p in m.params.items()}
        if name == "pipelined_1gpu":
            r = EpochRunner(m, upd, kg, nbatches=args.nb, seed=7, pipelined=True)
        else:
            r = DataParallelRunner(m, upd, kg, args.nb, seed=7)
        r.run(2)                      # warm-up (DP: the first epoch also captures the graph)
        r.synchronize()
        for pid, p in m.params.items():
            p.data.copy_(init[pid])
            upd[pid].reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.run(args.steps)
        r.synchronize()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out[name] = {"ms_per_epoch": round(1000.0 * el / args.steps, 4),
                     "us_per_batch": round(1e6 * el / args.steps / (kg.T // (kg.T // args.nb) +
                                                                  (1 if kg.T % args.nb else 0)), 3),
                     "E_checksum": float(m.E.data.double().sum().item())}
        if name == "dp_world1_nccl":
            out[name]["captured_graph"] = r.graph is not None
        del r
    out["ratio_dp_over_1gpu"] = round(out["dp_world1_nccl"]["ms_per_epoch"] /
                                      out["pipelined_1gpu"]["ms_per_epoch"], 4)
    out["bitwise_same_tables"] = out["dp_world1_nccl"]["E_checksum"] == out["pipelined_1gpu"]["E_checksum"]
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
