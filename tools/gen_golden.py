#!/usr/bin/env python3
"""Generate golden fixtures by importing the scikit-kge reference library layer.

Runs ONLY in the build container (the reference at /root/reference does not
travel to the GPU box).  It imports the reference unmodified, with the
harness-level shims listed in SURVEY.md section 8(c):

  1. sys.dont_write_bytecode (the tree is read-only)
  2. sys.path gets /root/reference and /root/reference/skge
     (skge/base.py:20 does a Py2-style ``from subgraphs import Subgraphs``)
  3. a stub ``trident`` module (skge/base.py:21; only get_all_triples uses it)
  4. collections.Hashable alias (skge/util.py:148, removed in Py3.10)
  5. a numpy proxy for skge.rescal whose array() retries with dtype=object
     (skge/rescal.py:84-85 builds ragged arrays, rejected since numpy 1.24)
  6. chdir to a scratch dir, file_grad=None / file_embed=None
  7. logging disabled

Every fixture drives the reference's own trainer loop
(``PairwiseStochasticTrainer._optim`` / ``StochasticTrainer._optim``,
skge/base.py:1242-1291) for one epoch over a small synthetic KG and records,
per mini-batch, the explicit (positive, negative) pairs the reference sampler
produced, the raw scores, the violation count, the gradient dicts returned by
the model (``{pid: (rows, sorted-unique idx)}``) and the parameters after
``_batch_step``.  Initial parameters are rounded to fp32 first so the fp32
HIP build and the fp64 reference see identical inputs.

Output: tests/golden/*.npz (inputs + expected outputs only, no code).
Usage:  python tools/gen_golden.py [--out tests/golden]
"""
import argparse
import collections
import collections.abc
import logging
import os
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"


def import_reference():
    sys.dont_write_bytecode = True
    sys.path[:0] = [REF, os.path.join(REF, "skge")]
    sys.modules["trident"] = types.ModuleType("trident")
    collections.Hashable = collections.abc.Hashable
    logging.disable(logging.CRITICAL)
    import warnings
    warnings.filterwarnings("ignore")
    import skge.base as base
    import skge.rescal as rescal
    from skge.transe import TransE
    from skge.hole import HolE
    from skge.param import AdaGrad, SGD
    from skge.sample import RandomModeSampler
    import skge.actfun as af

    class _NpProxy(types.ModuleType):
        def __getattr__(self, k):
            return getattr(np, k)

        @staticmethod
        def array(*a, **kw):
            try:
                return np.array(*a, **kw)
            except ValueError:
                kw["dtype"] = object
                return np.array(*a, **kw)

    rescal.np = _NpProxy("np_proxy")
    return types.SimpleNamespace(base=base, TransE=TransE, HolE=HolE,
                                 RESCAL=rescal.RESCAL, AdaGrad=AdaGrad, SGD=SGD,
                                 RandomModeSampler=RandomModeSampler, af=af)


def make_kg(n_ent, n_rel, n_triples, seed=0):
    """Unique uniform (s, o, p) triples, RandomState(seed) + rejection."""
    rs = np.random.RandomState(seed)
    seen, out = set(), []
    while len(out) < n_triples:
        t = (int(rs.randint(n_ent)), int(rs.randint(n_ent)), int(rs.randint(n_rel)))
        if t not in seen:
            seen.add(t)
            out.append(t)
    return out


def round_params_fp32(model):
    for pid, p in model.params.items():
        p[...] = np.asarray(p, dtype=np.float32).astype(np.float64)


def _store(arr, hi_precision):
    arr = np.asarray(arr)
    if arr.dtype.kind == "f" and not hi_precision:
        return arr.astype(np.float32)
    return arr


def run_case(R, name, model_kind, mode, opt, d, n_ent, n_rel, n_triples, nb,
             lr=0.1, margin=2.0, l1=True, rparam=0.0, afname=None, hi=True,
             seed_params=42, out_dir="tests/golden"):
    np.random.seed(seed_params)
    sz = (n_ent, n_ent, n_rel)
    if model_kind == "transe":
        model = R.TransE(sz, d, l1=l1)
    elif model_kind == "hole":
        model = R.HolE(sz, d, rparam=rparam)
    elif model_kind == "rescal":
        model = R.RESCAL(sz, d, rparam=rparam, af=afname or "linear")
    else:
        raise ValueError(model_kind)
    round_params_fp32(model)
    init = {pid: np.array(p, dtype=np.float32) for pid, p in model.params.items()}

    xs = make_kg(n_ent, n_rel, n_triples, seed=0)
    ys = np.ones(len(xs))
    sampler = R.RandomModeSampler(1, [0, 1], xs, sz)
    upd = {"adagrad": R.AdaGrad, "sgd": R.SGD}[opt]
    np.random.seed(7)
    if mode == "pairwise":
        trainer = R.base.PairwiseStochasticTrainer(
            model, nbatches=nb, margin=margin, max_epochs=1, learning_rate=lr,
            samplef=sampler.sample, post_epoch=[], param_update=upd,
            file_grad=None, file_embed=None)
    else:
        trainer = R.base.StochasticTrainer(
            model, nbatches=nb, max_epochs=1, learning_rate=lr,
            samplef=sampler.sample, post_epoch=[], param_update=upd)

    rec = []
    if mode == "pairwise":
        orig = model._pairwise_gradients

        def wrapped(pxs, nxs):
            pos = np.array([x for x, _ in pxs], dtype=np.int64)
            neg = np.array([x for x, _ in nxs], dtype=np.int64)
            ps = np.asarray(model._scores(pos[:, 0], pos[:, 2], pos[:, 1]), dtype=np.float64)
            ns = np.asarray(model._scores(neg[:, 0], neg[:, 2], neg[:, 1]), dtype=np.float64)
            g = orig(pxs, nxs)
            rec.append({"pos": pos, "neg": neg, "pscore": ps, "nscore": ns,
                        "nviol": int(model.nviolations),
                        "grads": None if g is None else
                        {k: (np.array(v[0], dtype=np.float64), np.array(v[1], dtype=np.int64))
                         for k, v in g.items()}})
            return g
        model._pairwise_gradients = wrapped
    else:
        orig = model._gradients

        def wrapped(xys):
            trip = np.array([x for x, _ in xys], dtype=np.int64)
            y = np.array([v for _, v in xys], dtype=np.float64)
            sc = np.asarray(model._scores(trip[:, 0], trip[:, 2], trip[:, 1]), dtype=np.float64)
            g = orig(xys)
            rec.append({"trip": trip, "y": y, "score": sc, "loss": float(model.loss),
                        "grads": {k: (np.array(v[0], dtype=np.float64), np.array(v[1], dtype=np.int64))
                                  for k, v in g.items()}})
            return g
        model._gradients = wrapped

    orig_bs = trainer._batch_step

    def bs(grads):
        orig_bs(grads)
        if len(rec) == 1 or True:
            rec[-1]["after"] = {pid: np.array(p, dtype=np.float64) for pid, p in model.params.items()}
            rec[-1]["state"] = {pid: np.array(u.p2, dtype=np.float64)
                                for pid, u in trainer._updaters.items() if hasattr(u, "p2")}
    trainer._batch_step = bs

    trainer.fit(xs, list(ys))

    out = {"meta_model": model_kind, "meta_mode": mode, "meta_opt": opt,
           "d": d, "n_ent": n_ent, "n_rel": n_rel, "lr": lr, "margin": margin,
           "l1": int(l1), "rparam": rparam, "af": afname or "",
           "nbatch": len(rec), "param_ids": np.array(list(model.params.keys()))}
    for pid, v in init.items():
        out["init_" + pid] = v
    out["triples"] = np.array(xs, dtype=np.int64)
    for b, r in enumerate(rec):
        pre = "b%d_" % b
        if mode == "pairwise":
            out[pre + "pos"] = r["pos"].astype(np.int32)
            out[pre + "neg"] = r["neg"].astype(np.int32)
            out[pre + "pscore"] = r["pscore"]
            out[pre + "nscore"] = r["nscore"]
            out[pre + "nviol"] = r["nviol"]
        else:
            out[pre + "trip"] = r["trip"].astype(np.int32)
            out[pre + "y"] = r["y"]
            out[pre + "score"] = r["score"]
            out[pre + "loss"] = r["loss"]
        out[pre + "has_grads"] = int(r["grads"] is not None)
        if r["grads"] is not None:
            for pid, (g, idx) in r["grads"].items():
                if b not in (0, len(rec) - 1) or (g.ndim == 3 and b > 0):
                    continue  # size: gradients of the first and last batch only
                out[pre + "g_" + pid] = _store(g, hi)
                out[pre + "gidx_" + pid] = idx.astype(np.int32)
        # parameters after the first batch and after the last one
        if (b == 0 or b == len(rec) - 1) and "after" in r:
            for pid, v in r["after"].items():
                out[pre + "after_" + pid] = _store(v, hi)
            for pid, v in r["state"].items():
                out[pre + "state_" + pid] = _store(v, hi)
    # the last batch that updated (trajectory end state)
    last = max([b for b, r in enumerate(rec) if "after" in r], default=-1)
    out["last_update_batch"] = last
    if last >= 0 and last != len(rec) - 1 and last != 0:
        r = rec[last]
        for pid, v in r["after"].items():
            out["b%d_after_%s" % (last, pid)] = _store(v, hi)
        for pid, v in r["state"].items():
            out["b%d_state_%s" % (last, pid)] = _store(v, hi)
    path = os.path.join(out_dir, name + ".npz")
    np.savez_compressed(path, **out)
    return path, len(rec), [r.get("nviol") for r in rec]


def init_quirks(R, out_dir):
    """Initialisation fixtures: TransE E row-normalised (skge/transe.py:21,
    skge/param.py:161-167 with idx=None) and HolE's column-wise normless1
    quirk (skge/hole.py:16, skge/param.py:170-174 with idx=None -> M[None])."""
    from skge import param as P
    np.random.seed(42)
    raw = P.init_nunif((64, 8))
    out = {"raw": raw.copy(),
           "normalize_none": P.normalize(raw.copy(), None),
           "normless1_none": P.normless1(raw.copy() * 3.0, None),
           "normless1_none_in": raw.copy() * 3.0}
    idx = np.array([1, 5, 9, 33], dtype=np.int64)
    m = raw.copy() * 3.0
    out["normless1_idx_in"] = m.copy()
    out["normless1_idx"] = P.normless1(m, idx)
    out["normless1_idx_idx"] = idx
    m = raw.copy()
    out["normalize_idx"] = P.normalize(m, idx)
    # model constructors: E / R after __init__ under np.random.seed(42)
    np.random.seed(42)
    t = R.TransE((50, 50, 4), 8)
    out["transe_E"] = np.array(t.E)
    out["transe_R"] = np.array(t.R)
    np.random.seed(42)
    h = R.HolE((50, 50, 4), 8)
    out["hole_E"] = np.array(h.E)
    out["hole_R"] = np.array(h.R)
    np.random.seed(42)
    rs = R.RESCAL((50, 50, 3), 4)
    out["rescal_E"] = np.array(rs.E)
    out["rescal_W"] = np.array(rs.W)
    # ccorr / cconv on random vectors (skge/util.py:8-50)
    rs2 = np.random.RandomState(3)
    a = rs2.randn(5, 12)
    b = rs2.randn(5, 12)
    from skge.util import ccorr, cconv
    out["cc_a"], out["cc_b"] = a, b
    out["ccorr"], out["cconv"] = ccorr(a, b), cconv(a, b)
    np.savez_compressed(os.path.join(out_dir, "init_quirks.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
    args = ap.parse_args()
    out_dir = os.path.abspath(args.out)
    os.makedirs(out_dir, exist_ok=True)
    R = import_reference()
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp())
    try:
        init_quirks(R, out_dir)
        sizes = {8: 512, 50: 256, 200: 128}
        cases = []
        for d, n in sizes.items():
            hi = d <= 8
            for l1 in (True, False):
                for opt in ("adagrad", "sgd"):
                    cases.append(("transe_%s_%s_d%d" % ("l1" if l1 else "l2", opt, d),
                                  dict(model_kind="transe", mode="pairwise", opt=opt, d=d,
                                       n_ent=n, n_rel=18, n_triples=200, nb=3, l1=l1,
                                       margin=2.0, hi=hi)))
            cases.append(("hole_pairwise_adagrad_d%d" % d,
                          dict(model_kind="hole", mode="pairwise", opt="adagrad", d=d, n_ent=n,
                               n_rel=18, n_triples=200, nb=3, margin=0.2, hi=hi)))
            cases.append(("hole_logistic_adagrad_d%d" % d,
                          dict(model_kind="hole", mode="logistic", opt="adagrad", d=d, n_ent=n,
                               n_rel=18, n_triples=200, nb=3, rparam=0.01, hi=hi)))
            m, nr, nt, rnb = {8: (18, n, 120, 3), 50: (6, n, 90, 3), 200: (2, 64, 60, 1)}[d]
            cases.append(("rescal_pairwise_adagrad_d%d" % d,
                          dict(model_kind="rescal", mode="pairwise", opt="adagrad", d=d, n_ent=nr,
                               n_rel=m, n_triples=nt, nb=rnb, margin=0.2, rparam=0.01, hi=d <= 8)))
            cases.append(("rescal_logistic_adagrad_d%d" % d,
                          dict(model_kind="rescal", mode="logistic", opt="adagrad", d=d, n_ent=nr,
                               n_rel=m, n_triples=nt, nb=rnb, rparam=0.01, hi=d <= 8)))
        # edge cases
        cases.append(("transe_l1_adagrad_noviol",
                      dict(model_kind="transe", mode="pairwise", opt="adagrad", d=8, n_ent=64,
                           n_rel=4, n_triples=60, nb=2, margin=-1e6)))
        cases.append(("transe_l1_adagrad_dups",
                      dict(model_kind="transe", mode="pairwise", opt="adagrad", d=16, n_ent=12,
                           n_rel=3, n_triples=120, nb=2, margin=2.0)))
        cases.append(("hole_pairwise_sgd_dups",
                      dict(model_kind="hole", mode="pairwise", opt="sgd", d=12, n_ent=12,
                           n_rel=3, n_triples=120, nb=2, margin=0.2)))
        cases.append(("hole_pairwise_adagrad_rparam",
                      dict(model_kind="hole", mode="pairwise", opt="adagrad", d=16, n_ent=64,
                           n_rel=5, n_triples=100, nb=2, margin=0.2, rparam=0.05)))
        for name, kw in cases:
            path, nbatch, nv = run_case(R, name, out_dir=out_dir, **kw)
            print("%-34s batches=%d nviol=%s %6.1f KB" % (name, nbatch, nv, os.path.getsize(path) / 1024))
    finally:
        os.chdir(cwd)


if __name__ == "__main__":
    main()
