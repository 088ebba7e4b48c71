#!/usr/bin/env python3
"""Per-epoch HBM traffic of the batch kernels from a `gpu_run.sh pmc` pass
(FETCH_SIZE and WRITE_SIZE runs, one row per dispatch): the launches of each
kernel at its full-batch grid in dispatch order, `launches` per epoch, with
MI355X_MICROARCH.md's gfx950 correction (traffic = 2 x FETCH_SIZE +
WRITE_SIZE, KB units).  Config 5: the bench line's timed epochs are epochs
W..W+K-1 of this list (epoch 0 = the warm-up).
Usage: python tools/pmc_epochs.py <pmc dir> <launches per epoch> [kernel prefixes...]
"""
import csv
import json
import os
import sys


def per_dispatch(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            out[int(r["Dispatch_Id"])] = (r["Kernel_Name"], r["Grid_Size"], float(r["Counter_Value"]))
    return out


def main():
    root, per = sys.argv[1], int(sys.argv[2])
    # the two-launch runner's kernels, or the pipelined runner's batch kernel
    names = sys.argv[3:] or ["k_transe_l1_sample_grad", "k_apply", "k_pipe_batch"]
    fetch = per_dispatch(os.path.join(root, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(root, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    res = {}
    for name in names:
        def rows(tab):
            sel = [(k, v) for k, v in sorted(tab.items()) if v[0].startswith(name)]
            grids = {}
            for k, v in sel:
                grids.setdefault(v[1], []).append(v[2])
            return max(grids.values(), key=len) if grids else []
        f, w = rows(fetch), rows(write)
        n = min(len(f), len(w))
        if n == 0:   # (this runner does not launch it)
            continue
        eps = []
        for e in range(0, n, per):
            fe, we = f[e:e + per], w[e:e + per]
            t = (2.0 * sum(fe) + sum(we)) * 1024.0 / len(fe)
            eps.append({"epoch": e // per, "launches": len(fe),
                        "fetch_kb_per_launch": round(sum(fe) / len(fe), 1),
                        "write_kb_per_launch": round(sum(we) / len(we), 1),
                        "traffic_bytes_per_launch": round(t)})
        res[name] = eps
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
