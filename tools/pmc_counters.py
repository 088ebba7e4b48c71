#!/usr/bin/env python3
"""Per-kernel, per-grid averages of any rocprofv3 --pmc counters (one pass,
gpu_run.sh step `pmcx`): {kernel: {grid: {calls, counter: mean per dispatch}}}.
SQ_* cycle counters are in quad-cycles (MI355X_MICROARCH.md, "rocprofv3 PMC
slots"); derived: active_valu_frac = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES,
wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES, issue_stall_frac = SQ_WAIT_INST_ANY /
SQ_WAVE_CYCLES, valu_per_wave = SQ_INSTS_VALU / SQ_WAVES.
Usage: python tools/pmc_counters.py <rocprofv3 output dir>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        sys.exit("no counter_collection.csv under %s" % d)
    per = defaultdict(lambda: defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(f[0])):
        key = r["Dispatch_Id"]
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        g = None
        for k in ("Grid_Size_X", "Grid_Size", "Grid_Size_x"):
            if r.get(k) not in (None, ""):
                g = int(float(r[k]))
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        meta[key] = (name, g)
    agg = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    cnt = defaultdict(lambda: defaultdict(int))
    for key, cs in per.items():
        n, g = meta[key]
        cnt[n][g] += 1
        for c, v in cs.items():
            agg[n][g][c] += v
    out = {}
    for n in agg:
        out[n] = {}
        for g in agg[n]:
            k = cnt[n][g]
            e = {"calls": k}
            e.update({c: v / k for c, v in agg[n][g].items()})
            wc = e.get("SQ_WAVE_CYCLES")
            if wc:
                for c, name in (("SQ_ACTIVE_INST_VALU", "active_valu_frac"),
                                ("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "issue_stall_frac"),
                                ("SQ_ACTIVE_INST_ANY", "active_any_frac"),
                                ("SQ_WAIT_INST_LDS", "lds_issue_stall_frac")):
                    if c in e:
                        e[name] = e[c] / wc
            if e.get("SQ_WAVES") and "SQ_INSTS_VALU" in e:
                e["valu_per_wave"] = e["SQ_INSTS_VALU"] / e["SQ_WAVES"]
            out[n][str(g)] = e
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
