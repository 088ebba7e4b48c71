"""One GPU run showing that tests/test_gpu_device_loop.py's stream-ordering
regression test has teeth: the same dirty-allocator / delayed-zero-fill
scenario with the runner's ordering neutralised (the caller-stream sync after
the tables are built and run()'s wait_stream patched to no-ops) must differ
from the fresh run, while the scenario as shipped must not.  Prints one JSON
line.  Run once (not in a loop): python tools/race_check.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "scikit-kge_amd")]

from test_gpu_device_loop import race_scenario  # noqa: E402


def diff(a, b):
    return {k: int(np.sum(a[k] != b[k])) for k in ("E", "R", "pE")}


def main():
    out = {}
    for d in (200, 64):
        f, r = race_scenario(d=d)
        f2, u = race_scenario(d=d, unordered=True)
        out[str(d)] = {"ordered": {"diff_elems": diff(f, r), "err": r["err"],
                                   "nviol": [f["nviol"], r["nviol"]]},
                       "unordered": {"diff_elems": diff(f2, u), "err": u["err"],
                                     "nviol": [f2["nviol"], u["nviol"]]}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
