#!/usr/bin/env python3
"""Per-epoch mean durations of the batch kernels in a rocprofv3 kernel trace
(config 5: the two-launch runner's k_transe_*_sample_grad / k_apply at the
full batch grid, `launches` per epoch, in dispatch order), so the bench
line's per-kernel times -- HIP events over the timed epochs -- can be checked
against the profiler epoch by epoch.
Usage: python tools/trace_epochs.py <rocprofv3 dir> <launches per epoch> [kernel prefixes...]
"""
import csv
import glob
import json
import os
import sys


def main():
    root, per = sys.argv[1], int(sys.argv[2])
    names = sys.argv[3:] or ["k_transe_l1_sample_grad", "k_apply", "k_pipe_batch"]
    f = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    out = {}
    for name in names:
        sel = [r for r in rows if r["Kernel_Name"].startswith(name)]
        if not sel:   # (this runner does not launch it)
            continue
        grids = {}
        for r in sel:
            g = r.get("Grid_Size_X") or r.get("Grid_Size")
            grids.setdefault(g, []).append(r)
        g, rs = max(grids.items(), key=lambda kv: len(kv[1]))   # the full-batch geometry
        v = sorted((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
                   for r in rs)
        out[name] = {"grid": g, "epochs": [
            {"epoch": e // per, "launches": len(v[e:e + per]),
             "avg_us": round(sum(x[1] for x in v[e:e + per]) / len(v[e:e + per]), 3),
             "sum_ms": round(sum(x[1] for x in v[e:e + per]) / 1e3, 3)}
            for e in range(0, len(v), per)]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
