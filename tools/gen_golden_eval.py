#!/usr/bin/env python3
"""Golden fixtures for filtered-ranking evaluation,
made by running the reference's own evaluators in this container:
FilteredRankingEval.positions (skge/base.py:913-1031) with TransEEval
(skge/run_transe.py:15-29) and HolEEval (skge/run_hole.py:12-19), on small
random models (parameters rounded to fp32 first).  Same import shims as
tools/gen_golden.py.  Writes tests/golden/eval_<model>.npz: E, R, the known
triples, the test triples in the evaluator's iteration order, and their
raw / filtered tail and head positions.  One more harness shim: np.Inf is
aliased to np.inf (skge/base.py:977 and 1017 use the alias NumPy 2.0 removed).
Usage: python tools/gen_golden_eval.py [--out tests/golden]
"""
import argparse
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_golden import import_reference, make_kg   # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
    args = ap.parse_args()
    out = os.path.abspath(args.out)
    ref = import_reference()
    np.Inf = np.inf   # compat shim (NumPy 2.0 removed the alias)
    os.chdir(tempfile.mkdtemp())
    import run_transe   # noqa: F401  (skge/run_transe.py: TransEEval)
    import run_hole     # noqa: F401  (skge/run_hole.py: HolEEval)
    base = sys.modules["base"]   # the evaluators' own copy of skge/base.py
    for name, n_ent, n_rel, d in (("transe", 150, 4, 16), ("hole", 120, 3, 16)):
        trip = np.asarray(make_kg(n_ent, n_rel, 600, seed=11), dtype=np.int64)
        np.random.seed(42)
        if name == "transe":
            m = ref.TransE((n_ent, n_ent, n_rel), d)
            ev_cls = run_transe.TransEEval
        else:
            m = ref.HolE((n_ent, n_ent, n_rel), d)
            ev_cls = run_hole.HolEEval
        for pid in m.params:
            m.params[pid][:] = m.params[pid].astype(np.float32).astype(np.float64)
        rs = np.random.RandomState(3)
        test = trip[rs.choice(len(trip), 40, replace=False)]
        xs = [tuple(int(v) for v in t) for t in test]
        known = [tuple(int(v) for v in t) for t in trip]
        ev = ev_cls(xs, known)
        assert isinstance(ev, base.FilteredRankingEval)
        pos, fpos = ev.positions(m)
        q, tr, tf, hr, hf = [], [], [], [], []
        for p, sos in ev.idx.items():
            for k, (s, o) in enumerate(sos):
                q.append((s, o, p))
                tr.append(pos[p]["tail"][k])
                tf.append(fpos[p]["tail"][k])
                hr.append(pos[p]["head"][k])
                hf.append(fpos[p]["head"][k])
        np.savez_compressed(os.path.join(out, "eval_%s.npz" % name), model=name,
                            E=np.asarray(m.E, dtype=np.float64), R=np.asarray(m.R, dtype=np.float64),
                            known=np.asarray(known, dtype=np.int32),
                            queries=np.asarray(q, dtype=np.int32),
                            tail_raw=np.asarray(tr), tail_filt=np.asarray(tf),
                            head_raw=np.asarray(hr), head_filt=np.asarray(hf))
        print(name, "queries", len(q), "mean filtered tail rank", np.mean(tf))


if __name__ == "__main__":
    main()
