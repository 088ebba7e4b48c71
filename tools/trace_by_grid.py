#!/usr/bin/env python3
"""Per-kernel, per-grid dispatch statistics from a rocprofv3 --kernel-trace
CSV (profiles/<round>/kernel_trace_by_grid.json): the same kernel runs at
several geometries in one bench command (the timed nb=100 epochs, the flush,
the nb=2 detail line), and the roofline is read at the one launched most.
Usage: python tools/trace_by_grid.py <rocprofv3 output dir> > kernel_trace_by_grid.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    files = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit("no *kernel_trace.csv under %s" % root)
    durs = defaultdict(lambda: defaultdict(list))
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "")
                short = name.split("(")[0].split("<")[0].replace("void ", "").split("::")[-1]
                grid = None
                for key in ("Grid_Size_X", "Grid_Size", "Grid_Size_x"):
                    if r.get(key) not in (None, ""):
                        grid = int(float(r[key]))
                        break
                us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
                durs[short][str(grid)].append(us)
    out = {}
    for k in sorted(durs):
        out[k] = {g: {"avg_us": sum(v) / len(v), "calls": len(v), "min_us": min(v),
                      "max_us": max(v)} for g, v in sorted(durs[k].items())}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
