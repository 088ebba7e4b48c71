"""Filtered link-prediction ranking on the device (mirrors FilteredRankingEval,
skge/base.py:737-1031, with the TransEEval / HolEEval scorers of
skge/run_transe.py:15-29 and skge/run_hole.py:12-19).

``positions(model)`` returns the reference's structures
``(pos, fpos)`` = ``{p: {'head': [...], 'tail': [...]}}`` (raw, filtered),
computed for every test triple in one ``skge_rank`` call
(csrc/skge_eval.hip).  A position is 1 + #entities scoring strictly higher
than the true one: the reference's descending-argsort position whenever no
other entity ties the true score exactly (among exact ties the reference
follows numpy's unstable argsort order).
"""
import os
from collections import defaultdict

import numpy as np
import torch

from . import _lib as L
from .device import DeviceKG
from .util import triples_array


def _model_code(model):
    from .transe import TransE
    from .hole import HolE
    from .rescal import RESCAL
    if isinstance(model, TransE):
        return L.SKGE_TRANSE_L1, model.params["R"]
    if isinstance(model, HolE):
        return L.SKGE_HOLE, model.params["R"]
    if isinstance(model, RESCAL):
        return L.SKGE_RESCAL, model.params["W"]
    raise NotImplementedError("no evaluator for %s" % type(model).__name__)


class FilteredRankingEval(object):
    """xs: test triples (s, o, p); true_triples: every known triple (the
    filter).  neval is accepted for signature compatibility (the reference
    computes it but evaluates every triple, base.py:955)."""

    def __init__(self, xs, true_triples, neval=-1):
        self.sz = len(xs)
        self.neval = neval
        idx = defaultdict(list)
        for s, o, p in triples_array(xs).tolist():
            idx[p].append((s, o))
        self.idx = dict(idx)
        self._true = triples_array(true_triples)
        self._kg = {}        # per device: the known-triple set
        self._answers = {}   # per device: the known-answer CSR
        self.last_ranks = None

    def _known_set(self, device):
        key = str(torch.device(device))
        if key not in self._kg:
            self._kg[key] = DeviceKG(self._true, device)
        return self._kg[key]

    def _known_answers(self, q, device):
        """Per query (s, o, p) its other known tails {o' != o: (s, o', p) known}
        and heads {s' != s: (s', o, p) known}, as int32 CSR on the device (the
        filter of skge/base.py:913-1031 as lists: a handful per query)."""
        key = str(torch.device(device))
        if key not in self._answers:
            tails, heads = defaultdict(set), defaultdict(set)
            for s, o, p in self._true.tolist():
                tails[(s, p)].add(o)
                heads[(o, p)].add(s)
            toff, tent, hoff, hent = [0], [], [0], []
            for s, o, p in q:
                tent.extend(sorted(x for x in tails.get((s, p), ()) if x != o))
                toff.append(len(tent))
                hent.extend(sorted(x for x in heads.get((o, p), ()) if x != s))
                hoff.append(len(hent))
            as_dev = lambda v: torch.as_tensor(np.asarray(v if v else [0], dtype=np.int32),
                                               device=device)
            self._answers[key] = (as_dev(toff), as_dev(tent), as_dev(hoff), as_dev(hent))
        return self._answers[key]

    def ranks(self, model):
        """[n, 4] int array: tail raw, tail filtered, head raw, head filtered,
        for the test triples in the evaluator's order (by relation, then
        insertion order, as positions() iterates)."""
        code, rel = _model_code(model)
        dev = model.device
        q = [(s, o, p) for p, sos in self.idx.items() for (s, o) in sos]
        if not q:
            return np.zeros((0, 4), dtype=np.int64)
        queries = torch.as_tensor(np.asarray(q, dtype=np.int32), device=dev)
        E = model.params["E"]
        lib = L.lib()
        out = torch.empty((len(q), 4), dtype=torch.int32, device=dev)
        if os.environ.get("SKGE_RANK_SET") == "1":   # A/B: the triple-set form (round 1)
            kg = self._known_set(dev)
            nbytes = lib.skge_rank_workspace_bytes(len(q), model.d)
            ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            L.check(lib.skge_rank(L.stream_ptr(), code, L.ptr(E.data), L.ptr(rel.data), E.rows,
                                  model.d, L.ptr(queries), len(q), L.ptr(kg.slots), kg.capacity,
                                  L.ptr(ws), nbytes, L.ptr(out)), "rank")
        else:
            toff, tent, hoff, hent = self._known_answers(q, dev)
            nbytes = lib.skge_rank_known_workspace_bytes(len(q), model.d)
            ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            L.check(lib.skge_rank_known(L.stream_ptr(), code, L.ptr(E.data), L.ptr(rel.data),
                                        E.rows, model.d, L.ptr(queries), len(q), L.ptr(toff),
                                        L.ptr(tent), L.ptr(hoff), L.ptr(hent), L.ptr(ws), nbytes,
                                        L.ptr(out)), "rank")
        self.last_ranks = out.cpu().numpy().astype(np.int64)
        return self.last_ranks

    def positions(self, mdl, plot=False, pagerankMap=None):
        r = self.ranks(mdl)
        pos, fpos = {}, {}
        k = 0
        for p, sos in self.idx.items():
            n = len(sos)
            pos[p] = {"tail": r[k:k + n, 0].tolist(), "head": r[k:k + n, 2].tolist()}
            fpos[p] = {"tail": r[k:k + n, 1].tolist(), "head": r[k:k + n, 3].tolist()}
            k += n
        return pos, fpos


class TransEEval(FilteredRankingEval):
    """skge/run_transe.py:13-29 (scores -sum|E[s] + R[p] - E|, either norm)."""


class HolEEval(FilteredRankingEval):
    """skge/run_hole.py:10-19 (scores ccorr(R[p], E) . E[s])."""


def compute_scores(pos, hits=10):
    """(MRR, mean position, hits@k in percent), skge/base.py:1099-1103."""
    pos = np.asarray(pos, dtype=np.float64)
    return float(np.mean(1.0 / pos)), float(np.mean(pos)), float(np.mean(pos <= hits) * 100)


def ranking_scores(pos, fpos):
    """Raw and filtered (MRR, mean position, hits@10) over heads and tails of
    every relation, as ranking_scores (skge/base.py:1050-1058) aggregates."""
    raw = [x for k in pos for x in pos[k]["head"] + pos[k]["tail"]]
    filt = [x for k in fpos for x in fpos[k]["head"] + fpos[k]["tail"]]
    return compute_scores(raw), compute_scores(filt)
