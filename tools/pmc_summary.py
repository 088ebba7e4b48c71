#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of tools/gpu_profile.sh into per-kernel numbers.

Per kernel: dispatches, average duration (kernel-trace stats), and per-launch
FETCH_SIZE / WRITE_SIZE (KB units, summed over the counter's instances).  The
HBM-traffic estimate follows MI355X_MICROARCH.md "HBM": on gfx950 FETCH_SIZE
reports half the bytes of wide (16 B/lane) coalesced reads, so
traffic = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes).  FETCH_SIZE derives from
the L2 memory-side requests, so Infinity-Cache hits are counted too.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def one(pattern):
    f = glob.glob(pattern, recursive=True)
    return f[0] if f else None


def grid_of(r):
    for key in ("Grid_Size_X", "Grid_Size", "Grid_Size_x"):
        if key in r and r[key] not in (None, ""):
            return int(float(r[key]))
    return None


def counters(d, name, by_grid=None):
    f = one(os.path.join(d, "**", "*counter_collection.csv"))
    out = defaultdict(list)
    if not f:
        return out
    per_dispatch = defaultdict(float)
    kname = {}
    kgrid = {}
    for r in csv.DictReader(open(f)):
        if r.get("Counter_Name") != name:
            continue
        key = r["Dispatch_Id"]
        per_dispatch[key] += float(r["Counter_Value"])
        kname[key] = r["Kernel_Name"]
        kgrid[key] = grid_of(r)
    for k, v in per_dispatch.items():
        out[kname[k]].append(v)
        if by_grid is not None:
            by_grid[(kname[k], kgrid[k])].append(v)
    return out


def trace_by_grid(d):
    """(kernel, grid size) -> list of durations (us) from the kernel trace: the
    same kernel launched at two geometries (e.g. the nb=100 epochs and the
    large-batch detail) is reported per geometry."""
    f = one(os.path.join(d, "**", "*kernel_trace.csv"))
    out = defaultdict(list)
    if not f:
        return out
    for r in csv.DictReader(open(f)):
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        out[(r["Kernel_Name"], grid_of(r))].append(dur)
    return out


def main(d):
    stats = {}
    f = one(os.path.join(d, "stats", "**", "*kernel_stats.csv"))
    if f:
        for r in csv.DictReader(open(f)):
            stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                "pct": float(r["Percentage"])}
    gfetch, gwrite = defaultdict(list), defaultdict(list)
    fetch = counters(os.path.join(d, "fetch"), "FETCH_SIZE", gfetch)
    write = counters(os.path.join(d, "write"), "WRITE_SIZE", gwrite)
    gtrace = trace_by_grid(os.path.join(d, "stats"))
    res = {}
    for k in set(stats) | set(fetch) | set(write):
        e = dict(stats.get(k, {}))
        if fetch.get(k):
            e["fetch_kb_per_launch"] = sum(fetch[k]) / len(fetch[k])
        if write.get(k):
            e["write_kb_per_launch"] = sum(write[k]) / len(write[k])
        if "fetch_kb_per_launch" in e and "write_kb_per_launch" in e:
            e["traffic_bytes_per_launch"] = 1024.0 * (2 * e["fetch_kb_per_launch"] +
                                                      e["write_kb_per_launch"])
        grids = sorted(g for (n, g) in gtrace if n == k)
        if len(grids) > 1:
            e["by_grid"] = {}
            for g in grids:
                t = gtrace[(k, g)]
                ge = {"calls": len(t), "avg_us": sum(t) / len(t)}
                if gfetch.get((k, g)) and gwrite.get((k, g)):
                    fk = sum(gfetch[(k, g)]) / len(gfetch[(k, g)])
                    wk = sum(gwrite[(k, g)]) / len(gwrite[(k, g)])
                    ge.update(fetch_kb_per_launch=fk, write_kb_per_launch=wk,
                              traffic_bytes_per_launch=1024.0 * (2 * fk + wk))
                e["by_grid"][str(g)] = ge
        res[k] = e
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
