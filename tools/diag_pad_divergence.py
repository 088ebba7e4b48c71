"""Where do config 1's two runners part ways?  (missing item 2)

Round 3 compared the padded pipelined TransE-L1 runner (d = 50 on zero-padded
d = 52 tables, packed exact sums, the fast reciprocal-sqrt projection of
skge_device.h proj_scale_fast) with the two-launch fp32 runner (fp32 sums,
correctly rounded projection) over one epoch of 10 batches and found 1,171 of
100,000 elements off by up to 0.068.  This replays the same comparison one
batch at a time (a KG of B = 1414 triples, nb = 1, so an epoch is one batch;
both runners draw the same negatives from the same keyed sampler) and, before
every batch, MEASURES from the two runners' current tables:

  flips      residual components (E[s] + R[p] - E[o] and the two negatives'
             residuals, skge/transe.py:32, 103-117) whose sign differs between
             the runners -- each flip moves that component's sub-gradient by 1
             (or 2) before the segment mean, i.e. by lr / count per flip;
  decisions  pairs whose margin test (strict >, transe.py:73) differs;

and after it: how many elements differ by more than 1e-5 and by how much.
Output: one JSON line per batch plus a summary (gpurun_out/diag_pad_div.json).
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scikit-kge_amd")]

N, M, D, B = 40943, 18, 50, 1414


def kg_triples(T, seed=21):
    rs = np.random.RandomState(seed)
    seen, out = set(), []
    while len(out) < T:
        t = (int(rs.randint(N)), int(rs.randint(N)), int(rs.randint(M)))
        if t not in seen:
            seen.add(t)
            out.append(t)
    return np.array(out, dtype=np.int32)


def residuals(E, R, rec, n1):
    s, o, p, a = rec[:, 0], rec[:, 1], rec[:, 2], rec[:, 3]
    b = n1
    vp = E[s] + R[p] - E[o]
    v0 = np.where((a >= 0)[:, None], E[np.maximum(a, 0)] + R[p] - E[o], 0.0)
    v1 = np.where((b >= 0)[:, None], E[s] + R[p] - E[np.maximum(b, 0)], 0.0)
    return vp, v0, v1


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=40943)
    ap.add_argument("--m", type=int, default=18)
    ap.add_argument("--batch", type=int, default=1414)
    ap.add_argument("--opt", default="sgd", choices=["sgd", "adagrad"])
    ap.add_argument("--batches", type=int, default=10)
    ap.add_argument("--tag", default="c1")
    args = ap.parse_args()
    global N, M, B
    N, M, B = args.n, args.m, args.batch
    batches, seed = args.batches, 7
    import skge_amd as S
    from skge_amd.device import DeviceKG, EpochRunner, epoch_records
    dev = torch.device("cuda", 0)
    trip = kg_triples(B)
    kg = DeviceKG(trip, dev)
    runs = []
    for f32 in (False, True):
        np.random.seed(42)
        m = S.TransE((N, N, M), D, l1=True)
        m.add_hyperparam("margin", 2.0)
        U = S.SGD if args.opt == "sgd" else S.AdaGrad
        upd = {pid: U(p, 0.1) for pid, p in m.params.items()}
        r = EpochRunner(m, upd, kg, nbatches=1, seed=seed, force_f32=f32)
        runs.append((m, r))
    assert runs[0][1].pipelined and runs[0][1]._pad and not runs[1][1].pipelined
    out = []
    for e in range(batches):
        rec, n1 = epoch_records(kg, N, seed, e)
        rec, n1 = rec.cpu().numpy(), n1.cpu().numpy()
        tabs = [(m.E.data.cpu().numpy(), m.R.data.cpu().numpy()) for m, _ in runs]
        ra = residuals(*tabs[0], rec, n1)
        rb = residuals(*tabs[1], rec, n1)
        flips = [int((np.sign(x) != np.sign(y)).sum()) for x, y in zip(ra, rb)]
        near = [int((np.minimum(np.abs(x), np.abs(y)) < 1e-6).sum()) for x, y in zip(ra, rb)]
        sa = [-np.abs(v).sum(1) for v in ra]
        sb = [-np.abs(v).sum(1) for v in rb]
        dec = int(((sa[1] + 2.0 > sa[0]) != (sb[1] + 2.0 > sb[0])).sum() +
                  ((sa[2] + 2.0 > sa[0]) != (sb[2] + 2.0 > sb[0])).sum())
        for m, r in runs:
            r.run(1)
            r.synchronize()
        dE = np.abs(runs[0][0].E.data.cpu().numpy().astype(np.float64) -
                    runs[1][0].E.data.cpu().numpy())
        dR = np.abs(runs[0][0].R.data.cpu().numpy().astype(np.float64) -
                    runs[1][0].R.data.cpu().numpy())
        line = {"tag": args.tag, "opt": args.opt, "n": N, "batch_size": B, "batch": e, "sign_flips_pos_neg0_neg1": flips,
                "components_below_1e-6": near, "margin_decision_flips": dec,
                "E_elems_gt_1e-5": int((dE > 1e-5).sum()), "E_rows_gt_1e-5": int((dE > 1e-5).any(1).sum()),
                "E_max": float(dE.max()), "R_elems_gt_1e-5": int((dR > 1e-5).sum()),
                "R_max": float(dR.max()), "E_elems_gt_0": int((dE > 0).sum())}
        print(json.dumps(line))
        out.append(line)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "diag_pad_div_%s.json" % args.tag), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
