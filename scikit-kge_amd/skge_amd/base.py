"""Model base class and the mini-batch trainers (mirrors skge/base.py:1140-1427).

The trainers keep the reference's names, kwargs and batch geometry; every
numeric step of a batch runs as HIP kernels through libskgehip.so:

* default (``fused=True``): one ``skge_pair_step`` / triple-grad + apply per
  batch -- score, margin test, segment-sum scatter, mean, updater and
  projection, never materialising the gradient rows;
* ``fused=False``: the reference protocol step by step --
  ``model._pairwise_gradients`` returns ``{pid: (rows, sorted idx)}`` and the
  updaters are called by ``_batch_step`` (skge/base.py:1306-1316);
* ``device_loop=True`` (PairwiseStochasticTrainer, every model): the whole
  epoch runs on the device -- permutation, negative sampling, score,
  scatter, update -- captured once into a hipGraph by a native runner.
"""
import logging
import os
import pickle
import timeit
import warnings

import numpy as np
import torch
from numpy.random import shuffle

from . import _lib as L
from .param import AdaGrad, Accumulator, Parameter, ParameterUpdate
from .util import labels_array, to_device_triples

log = logging.getLogger("EX-KG")

_DEF_NBATCHES = 100
_DEF_POST_EPOCH = []
_DEF_LEARNING_RATE = 0.1
_DEF_SAMPLE_FUN = None
_DEF_MAX_EPOCHS = 1000
_DEF_MARGIN = 1.0
_FILE_GRADIENTS = "gradients.txt"
_FILE_EMBEDDINGS = "embeddings.txt"


_DETERMINISTIC = [os.environ.get("SKGE_DETERMINISTIC", "0") == "1"]


def set_deterministic(flag=True):
    """The deterministic reduce mode (off by default; env SKGE_DETERMINISTIC=1):
    models created afterwards sum their float gradient contributions as exact
    64-bit fixed-point integers (SKGE_ACC_FX64) instead of fp32 atomics, so
    HolE / RESCAL / TransE-L2 parameters are bitwise reproducible run to run,
    like the reference's CSR mat-vec (skge/util.py:53-101).  Costs 8 B of
    atomic traffic per element instead of 4; the device loops then run the
    pair loop (the pipelined HolE runner keeps fp32 sums)."""
    _DETERMINISTIC[0] = bool(flag)


def deterministic():
    return _DETERMINISTIC[0]


class Model(object):
    """Base class of all models (skge/base.py:1140-1192).

    Subclasses set ``model_code`` (SKGE_*), ``rel_id`` ('R' or 'W') and
    implement ``_reg(mode)``: the (rin, rout, fixed_div) gradient combination
    of each table (see skge_table_t)."""
    model_code = None
    rel_id = "R"
    default_posts = {}

    def __init__(self, *args, **kwargs):
        self.params = {}
        self.hyperparams = {}
        self.add_hyperparam("init", kwargs.pop("init", "nunif"))
        self._acc = {}
        self.nviolations = 0
        self.loss = 0.0

    def add_param(self, param_id, shape, post=None, value=None):
        if value is None:
            value = Parameter(shape, self.init, name=param_id, post=post)
        elif not isinstance(value, Parameter):
            value = Parameter(None, name=param_id, post=post, value=value)
        setattr(self, param_id, value)
        self.params[param_id] = value

    def add_hyperparam(self, param_id, value):
        setattr(self, param_id, value)
        self.hyperparams[param_id] = value

    # ---- serialisation: the reference's {'hyperparams', 'params'} layout ----
    def __getstate__(self):
        return {"hyperparams": self.hyperparams,
                "params": {pid: np.asarray(p, dtype=np.float64) for pid, p in self.params.items()},
                "posts": {pid: p.post for pid, p in self.params.items()}}

    def __setstate__(self, st):
        self.params = {}
        self.hyperparams = {}
        self._acc = {}
        posts = st.get("posts", type(self).default_posts)
        for pid, p in st["params"].items():
            self.add_param(pid, None, posts.get(pid), value=p)
        for pid, p in st["hyperparams"].items():
            self.add_hyperparam(pid, p)

    def save_reference(self, fname, updaters=None):
        """Write the reference's model pickle (skge.<module>.<Class>, float64
        params) -- readable by skge's Model.load; see checkpoint.py."""
        from .checkpoint import save_reference
        save_reference(self, fname, updaters=updaters)

    def save(self, fname, protocol=pickle.HIGHEST_PROTOCOL):
        with open(fname, "wb") as fout:
            pickle.dump(self, fout, protocol=protocol)

    @staticmethod
    def load(fname):
        with open(fname, "rb") as fin:
            return pickle.load(fin)

    # ---- device plumbing ----
    @property
    def device(self):
        return self.params["E"].data.device

    @property
    def d(self):
        return int(self.ncomp)

    def accumulator(self, pid):
        """The device accumulator of table pid.  A narrow relation table is
        dense (no slot records; its apply is one wave or workgroup per row):
        each of its few rows is hit by most pairs of a batch, and per-slot
        claims -- or atomics -- on the same rows would serialise."""
        acc = self._acc.get(pid)
        if acc is None:
            p = self.params[pid]
            dense = pid == "R" and p.width <= 1024 and p.rows <= 65536   # not RESCAL W
            # and spread over copies when rows are very few (pair i adds into
            # copy i mod replicas; the apply / collect fold them)
            reps = 16 if p.rows <= 256 else (4 if p.rows <= 4096 else 1)
            mode = L.SKGE_ACC_F32
            if deterministic() and p.width <= 1024 and len(p.shape) == 2:
                # exact fixed-point sums (one copy): bitwise reproducible
                # (RESCAL's W sums are plain stores in a fixed order already)
                mode, reps = L.SKGE_ACC_FX64, 1
            acc = Accumulator(p.rows, p.width, p.data.device, dense=dense,
                              replicas=reps if dense else 1, mode=mode)
            self._acc[pid] = acc
        return acc

    def _af_code(self):
        return L.SKGE_AF_LINEAR

    def _reg(self, mode):
        return {"E": (0.0, 0.0, 0.0), self.rel_id: (0.0, 0.0, 0.0)}

    def _tables(self, mode, updaters=None, gate=None, slots=(0, 0)):
        """skge_table_t for E and R/W, with the accumulator (grown to hold
        `slots` touched slots) and, optionally, the updater fields."""
        out = []
        reg = self._reg(mode)
        for pid, ns in zip(("E", self.rel_id), slots):
            rin, rout, fdiv = reg[pid]
            acc = self.accumulator(pid).ensure_slots(ns)
            if updaters is not None:
                t = updaters[pid].table(acc, rin=rin, rout=rout, fixed_div=fdiv, gate=gate)
            else:
                from .param import table_struct
                t = table_struct(self.params[pid], None, acc, rin=rin, rout=rout, fixed_div=fdiv,
                                 gate=gate)
            out.append(t)
        if mode == "pairwise" and self._kernel_model() in (L.SKGE_TRANSE_L1, L.SKGE_TRANSE_L2):
            out[0].violations = L.ptr(self.params["E"].counter("viol"))   # transe.py:78-83
        return out

    def _collect(self, pid, t):
        """Accumulator -> (gradient rows, sorted unique idx) on the device."""
        p = self.params[pid]
        dev = p.data.device
        lib = L.lib()
        ws = torch.empty(int(lib.skge_collect_workspace_bytes(p.rows)), dtype=torch.uint8, device=dev)
        idx = torch.empty(p.rows, dtype=torch.int32, device=dev)
        g = torch.empty((p.rows,) + tuple(p.shape[1:]), dtype=torch.float32, device=dev)
        U = torch.zeros(1, dtype=torch.int32, device=dev)
        L.check(lib.skge_accum_collect(L.stream_ptr(), t, L.ptr(idx), L.ptr(g), L.ptr(U),
                                       L.ptr(ws), ws.numel()), "collect " + pid)
        u = int(U.item())
        return g[:u], idx[:u].long()

    # ---- the reference protocol ----
    def _scores(self, ss, ps, os):
        """Raw scores of triples (s, p, o) (e.g. skge/transe.py:25-46)."""
        dev = self.device
        trip = torch.stack([torch.as_tensor(np.asarray(x), dtype=torch.int32, device=dev)
                            for x in (ss, os, ps)], dim=1).contiguous()
        n = trip.shape[0]
        out = torch.empty(n, dtype=torch.float32, device=dev)
        te, tr = self._tables("pairwise")
        L.check(L.lib().skge_pair_grad(L.stream_ptr(), self._kernel_model(), self._af_code(), te,
                                       tr, self.d, L.ptr(trip), L.ptr(trip), n, float("-inf"),
                                       L.ptr(out), None, None, None), "scores")
        return out

    def _kernel_model(self):
        return self.model_code

    def _pair_slots(self, P):
        """touched slots per table written by skge_pair_grad (+ wgrad)"""
        return (4 * P, self.params[self.rel_id].rows if self.rel_id == "W" else 2 * P)

    def _triple_slots(self, T):
        return (2 * T, self.params[self.rel_id].rows if self.rel_id == "W" else T)

    def _pairwise_gradients(self, pxs, nxs):
        """Pairwise margin gradients (see the subclass docstring for the
        reference lines).  Returns None when no pair violates the margin,
        else {pid: (grad rows [U, ...] fp32, sorted unique idx [U] int64)}."""
        dev = self.device
        pos = to_device_triples(pxs, dev)
        neg = to_device_triples(nxs, dev)
        P = pos.shape[0]
        nviol = torch.zeros(1, dtype=torch.int32, device=dev)
        self._pscore = torch.empty(P, dtype=torch.float32, device=dev)
        self._nscore = torch.empty(P, dtype=torch.float32, device=dev)
        coef = torch.empty(2 * P, dtype=torch.float32, device=dev) if self.rel_id == "W" else None
        te, tr = self._tables("pairwise", slots=self._pair_slots(P))
        L.check(L.lib().skge_pair_grad(L.stream_ptr(), self._kernel_model(), self._af_code(), te,
                                       tr, self.d, L.ptr(pos), L.ptr(neg), P, float(self.margin),
                                       L.ptr(self._pscore), L.ptr(self._nscore), L.ptr(coef),
                                       L.ptr(nviol)), "pair_grad")
        self.nviolations = int(nviol.item())
        if self.nviolations == 0:
            return None
        if self.rel_id == "W":
            L.check(L.lib().skge_rescal_wgrad(L.stream_ptr(), te, tr, self.d, L.ptr(pos),
                                              L.ptr(coef), P, L.ptr(neg), L.ptr(coef[P:]), P),
                    "rescal_wgrad")
        return {"E": self._collect("E", te), self.rel_id: self._collect(self.rel_id, tr)}

    def _gradients(self, xys):
        """Logistic-loss gradients (HolE, RESCAL).  Sets self.loss."""
        dev = self.device
        trip = to_device_triples(xys, dev)
        ys = torch.as_tensor(labels_array(xys), device=dev)
        T = trip.shape[0]
        loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self._score = torch.empty(T, dtype=torch.float32, device=dev)
        coef = torch.empty(T, dtype=torch.float32, device=dev)
        te, tr = self._tables("logistic", slots=self._triple_slots(T))
        L.check(L.lib().skge_triple_grad(L.stream_ptr(), self._kernel_model(), te, tr, self.d,
                                         L.ptr(trip), L.ptr(ys), T, L.ptr(self._score),
                                         L.ptr(coef), L.ptr(loss)), "triple_grad")
        if self.rel_id == "W":
            L.check(L.lib().skge_rescal_wgrad(L.stream_ptr(), te, tr, self.d, L.ptr(trip),
                                              L.ptr(coef), T, None, None, 0), "rescal_wgrad")
        self.loss = float(loss.item())
        return {"E": self._collect("E", te), self.rel_id: self._collect(self.rel_id, tr)}

    # ---- fused steps used by the trainers ----
    def _pairwise_step(self, pos, neg, updaters, nviol):
        """score + grad + update for explicit pairs in one skge_pair_step.
        `nviol` must be zero on entry; it receives the violation count."""
        P = pos.shape[0]
        lib = L.lib()
        nbytes = lib.skge_pair_step_workspace_bytes(self._kernel_model(), P,
                                                    self.params[self.rel_id].rows, self.d)
        ws = self._workspace(nbytes)
        te, tr = self._tables("pairwise", updaters, gate=nviol, slots=self._pair_slots(P))
        L.check(lib.skge_pair_step(L.stream_ptr(), self._kernel_model(), self._af_code(), te,
                                   tr, self.d, L.ptr(pos), L.ptr(neg), P, float(self.margin),
                                   L.ptr(ws), nbytes, L.ptr(nviol)), "pair_step")

    def _workspace(self, nbytes):
        """Device scratch of at least nbytes (kept and grown across calls)."""
        if nbytes == 0:
            return None
        ws = getattr(self, "_ws", None)
        if ws is None or ws.numel() < nbytes:
            ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            self._ws = ws
        return ws

    def _logistic_step(self, trip, ys, updaters, loss):
        """score + grad + update for labelled triples in one skge_triple_step."""
        T = trip.shape[0]
        lib = L.lib()
        nbytes = lib.skge_triple_step_workspace_bytes(self._kernel_model(), T,
                                                      self.params[self.rel_id].rows, self.d)
        ws = self._workspace(nbytes)
        te, tr = self._tables("logistic", updaters, slots=self._triple_slots(T))
        L.check(lib.skge_triple_step(L.stream_ptr(), self._kernel_model(), te, tr, self.d,
                                     L.ptr(trip), L.ptr(ys), T, L.ptr(ws), nbytes, L.ptr(loss)),
                "triple_step")


class StochasticTrainer(object):
    """Stochastic gradient descent trainer with scalar loss (skge/base.py:1195-1316)."""

    def __init__(self, *args, **kwargs):
        self.model = args[0]
        self.hyperparams = {}
        self.add_hyperparam("max_epochs", kwargs.pop("max_epochs", _DEF_MAX_EPOCHS))
        self.add_hyperparam("nbatches", kwargs.pop("nbatches", _DEF_NBATCHES))
        self.add_hyperparam("learning_rate", kwargs.pop("learning_rate", _DEF_LEARNING_RATE))
        self.post_epoch = kwargs.pop("post_epoch", _DEF_POST_EPOCH)
        self.samplef = kwargs.pop("samplef", _DEF_SAMPLE_FUN)
        self.fused = kwargs.pop("fused", True)
        pu = kwargs.pop("param_update", AdaGrad)
        self._updaters = {key: pu(param, self.learning_rate)
                          for key, param in self.model.params.items()}
        self._fusable = all(type(u).__call__ is ParameterUpdate.__call__
                            for u in self._updaters.values())
        self._loss_dev = None
        self._loss_host = 0.0

    def set_max_epochs(self, epoch):
        self.max_epochs = epoch

    def __getstate__(self):
        return self.hyperparams

    def __setstate__(self, st):
        self.hyperparams = {}
        for pid, p in st.items():   # the reference iterates st['hyperparams'] as pairs (bug)
            self.add_hyperparam(pid, p)

    def add_hyperparam(self, param_id, value):
        setattr(self, param_id, value)
        self.hyperparams[param_id] = value

    def fit(self, xs, ys):
        self._optim(list(zip(xs, ys)))

    def _pre_epoch(self):
        self.loss = 0

    @property
    def loss(self):
        extra = float(self._loss_dev.item()) if self._loss_dev is not None else 0.0
        return self._loss_host + extra

    @loss.setter
    def loss(self, v):
        self._loss_host = float(v)
        if self._loss_dev is not None:
            self._loss_dev.zero_()

    def _optim(self, xys):
        """The reference loop (skge/base.py:1242-1291): numpy-global-RNG
        shuffle, np.split batches (nb full batches + the remainder)."""
        idx = np.arange(len(xys))
        self.batch_size = len(xys) // self.nbatches
        batch_idx = np.arange(self.batch_size, len(xys), self.batch_size)
        for self.epoch in range(1, self.max_epochs + 1):
            self._pre_epoch()
            shuffle(idx)
            self.epoch_start = timeit.default_timer()
            for batch in np.split(idx, batch_idx):
                bxys = [xys[z] for z in batch]
                self._process_batch(bxys)
            if deterministic():   # FX64 sums: range flag of the epoch's applies
                L.check_device_error(L.stream_ptr(), "trainer")
            for f in self.post_epoch:
                if not f(self):
                    break

    def _process_batch(self, xys):
        if self.samplef is not None:
            xys += self.samplef(xys)
        if hasattr(self.model, "_prepare_batch_step"):
            self.model._prepare_batch_step(xys)
        if self.fused and self._fusable:
            dev = self.model.device
            if self._loss_dev is None:
                self._loss_dev = torch.zeros(1, dtype=torch.float32, device=dev)
            trip = to_device_triples(xys, dev)
            ys = torch.as_tensor(labels_array(xys), device=dev)
            self.model._logistic_step(trip, ys, self._updaters, self._loss_dev)
            return
        grads = self.model._gradients(xys)
        self.loss += self.model.loss
        self._batch_step(grads)

    def _batch_step(self, grads):
        for paramID in self._updaters.keys():
            self._updaters[paramID](*grads[paramID])


class PairwiseStochasticTrainer(StochasticTrainer):
    """Stochastic gradient descent trainer with pairwise ranking loss
    (skge/base.py:1320-1427).  Extra kwargs: ``fused`` (default True),
    ``device_loop`` (device-resident epochs, see module doc), ``device_runner``
    ('auto', 'epoch': TransE's fused runners, 'pairs': the any-model pair
    loop), ``seed`` (device sampler / permutation key), ``ntries``."""

    def __init__(self, *args, **kwargs):
        self.device_loop = kwargs.pop("device_loop", False)
        self.device_runner = kwargs.pop("device_runner", "auto")
        self.seed = kwargs.pop("seed", 0)
        self.ntries = kwargs.pop("ntries", 100)
        super(PairwiseStochasticTrainer, self).__init__(*args, **kwargs)
        self.model.add_hyperparam("margin", kwargs.pop("margin", _DEF_MARGIN))
        fg = kwargs.pop("file_grad", _FILE_GRADIENTS)
        fe = kwargs.pop("file_embed", _FILE_EMBEDDINGS)
        self.file_gradients = None
        self.file_embeddings = None
        self.pickle_file_embeddings = None
        if fg is not None:
            self.file_gradients = open(fg, "w")
        if fe is not None:
            self.file_embeddings = open(fe, "w")
            self.pickle_file_embeddings = open(fe + ".pkl", "wb")
        self._nviol_host = 0
        self._nviol_dev = None
        self._nviol_batch = None
        self._runner = None

    @property
    def nviolations(self):
        extra = int(self._nviol_dev.item()) if self._nviol_dev is not None else 0
        return self._nviol_host + extra

    @nviolations.setter
    def nviolations(self, v):
        self._nviol_host = int(v)
        if self._nviol_dev is not None:
            self._nviol_dev.zero_()

    def fit(self, xs, ys):
        use_device = False
        if self.device_loop:
            from .device import device_sampler_args
            use_device, ntries, why = device_sampler_args(self, xs, ys)
            if not use_device:
                # the device loop draws RandomModeSampler(1, [0, 1]) negatives
                # itself; anything else trains on the per-batch path instead
                warnings.warn("device_loop: %s; training on the per-batch path" % why)
        self._on_device = use_device
        if use_device:
            from .device import device_optim
            device_optim(self, xs, ntries=ntries)
        elif self.samplef is None:
            pidx = np.where(np.array(ys) == 1)[0]
            nidx = np.where(np.array(ys) != 1)[0]
            pxs = [xs[i] for i in pidx]
            self.nxs = [xs[i] for i in nidx]
            self.pxs = int(len(self.nxs) / len(pxs)) * pxs
            xys = list(range(min(len(pxs), len(self.nxs))))
            self._optim(xys)
            return   # the labelled-negatives branch writes no files (skge/base.py:1350-1357)
        else:
            self._optim(list(zip(xs, ys)))
        self._write_outputs(xs, use_device)

    def _write_outputs(self, xs, device=False):
        """Post-fit counters and files of the reference's samplef branch
        (skge/base.py:1364-1386): E.neighbours accumulates over fits."""
        n = self.model.E.rows
        if self.model.E.neighbours is None:
            self.model.E.neighbours = np.zeros(n, dtype=np.int64)
        neighbours = self.model.E.neighbours
        x = np.asarray(xs, dtype=np.int64).reshape(-1, 3)
        np.add.at(neighbours, x[:, 0], 1)
        np.add.at(neighbours, x[:, 1], 1)
        if self.file_gradients is not None:
            # E.violations / E.updateCounts: device counters of the per-batch
            # paths and the device pair loop; the TransE epoch runners keep none
            if device and not getattr(self._runner, "counters", True):
                warnings.warn("device_loop (%s) keeps no per-row counters: the #(violations) "
                              "and #(updates) columns of file_grad are zero; use "
                              "device_runner='pairs' to count them" % type(self._runner).__name__)
            viol = self.model.E.violations
            upd = self.model.E.updateCounts
            self.file_gradients.write("Entity,Degree,#(violations),#(updates)\n")
            for index in range(n):
                self.file_gradients.write("%d,%d,%d,%d\n" % (index, neighbours[index],
                                                              viol[index], upd[index]))
            self.file_gradients.flush()
        E = np.asarray(self.model.E, dtype=np.float64)
        if self.file_embeddings is not None:
            for index, e in enumerate(E):
                self.file_embeddings.write("%d,%s\n" % (index, str(e)))
            self.file_embeddings.flush()
        if self.pickle_file_embeddings is not None:
            pickle.dump(list(E), self.pickle_file_embeddings, protocol=2)
            self.pickle_file_embeddings.flush()

    def _pre_epoch(self):
        self.nviolations = 0
        if self.samplef is None and not getattr(self, "_on_device", False):
            shuffle(self.pxs)
            shuffle(self.nxs)

    def _process_batch(self, xys):
        pxs = []
        nxs = []
        for xy in xys:
            if self.samplef is not None:
                for nx in self.samplef([xy]):
                    pxs.append(xy)
                    nxs.append(nx)
            else:
                pxs.append((self.pxs[xy], 1))
                nxs.append((self.nxs[xy], 1))
        if hasattr(self.model, "_prepare_batch_step"):
            self.model._prepare_batch_step(pxs, nxs)
        if len(pxs) == 0:
            return
        if self.fused and self._fusable:
            dev = self.model.device
            if self._nviol_dev is None:
                self._nviol_dev = torch.zeros(1, dtype=torch.int32, device=dev)
                self._nviol_batch = torch.zeros(1, dtype=torch.int32, device=dev)
            pos = to_device_triples(pxs, dev)
            neg = to_device_triples(nxs, dev)
            self._nviol_batch.zero_()
            self.model._pairwise_step(pos, neg, self._updaters, self._nviol_batch)
            self._nviol_dev += self._nviol_batch
            return
        grads = self.model._pairwise_gradients(pxs, nxs)
        if grads is not None:
            self._nviol_host += self.model.nviolations
            self._batch_step(grads)
