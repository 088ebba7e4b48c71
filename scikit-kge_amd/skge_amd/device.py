"""Device-resident training data and the native epoch runners.

DeviceKG holds the training triples on the GPU ([T, 3] int32, (s, o, p)) and
the open-addressing triple set the device sampler rejects against.
EpochRunner wraps the TransE runners (skge_pipe_runner_* / skge_runner_*,
csrc/skge_pipeline.hip, skge_epoch.hip) and PairLoopRunner the any-model pair
loop (skge_pair_runner_*, csrc/skge_pairloop.hip): one epoch of
PairwiseStochasticTrainer batches (nbatches full batches + the remainder,
skge/base.py:1246-1268), captured once into a hipGraph and replayed."""
import math
import timeit
import warnings

import numpy as np
import torch

from . import _lib as L
from .util import to_device_triples


def _next_pow2(n):
    c = 1
    while c < n:
        c <<= 1
    return c


class DeviceKG(object):
    def __init__(self, xs, device=None, stream=None):
        L.require_gpu()
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.trip = to_device_triples(xs, dev)
        self.T = int(self.trip.shape[0])
        self.capacity = _next_pow2(max(2 * self.T, 4))
        nbytes = int(L.lib().skge_triple_set_bytes(self.capacity))
        self.slots = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        L.check(L.lib().skge_triple_set_build(L.stream_ptr(stream), L.ptr(self.trip), self.T,
                                              L.ptr(self.slots), self.capacity), "triple set build")


PACKED_MAX = 32767   # a 16-bit packed field's bound (csrc/skge_pipeline.hip PACKED_MAX)
import os as _os


def _bincount_max(col, n):
    return torch.bincount(col.long(), minlength=n)


def packed_count_bound(kg, n_ent, batch, tail=None):
    """Upper bound on an ENTITY row's per-batch occurrence count in the
    TransE-L1 device loops (the count bounds every 16-bit field of its packed
    sums, csrc/skge_pipeline.hip).  A positive adds at most 3 to each of its s
    and o (skge/transe.py:103-136: s is sp of both pairs and sn of the
    tail-corrupted one) and 1 to each accepted corruption.  The first part
    comes from the training triples: a row that is the subject of c_s of the
    T triples is the subject of at most min(c_s, B) positives of a batch, and
    -- the batch being a uniform sample of the triples (the epoch permutation)
    -- of fewer than the binomial tail mu + 12 sqrt(mu) + 40, mu = c_s B / T,
    as relation_replicas() bounds the relation rows (round 4: the whole-KG
    count alone sent skewed KGs to fp32 sums at every batch past ~3k);
    likewise as object.  The corruptions are uniform draws over the entities
    (skge/sample.py:41-46), bounded by their Poisson tail (lambda + 12
    sqrt(lambda) + 40, lambda = 2 batch / n_ent).  The applies still check
    every row's count at run time (ERR_PACKED), and device_optim reads that
    flag after every epoch."""
    T = float(max(int(kg.trip.shape[0]), 1))
    B = float(min(int(batch), int(kg.trip.shape[0])))

    def per_batch(col):
        c = _bincount_max(col, n_ent).double()
        mu = c * (B / T)
        return torch.minimum(torch.minimum(c, torch.full_like(c, B)), (tail or _tail)(mu))
    occ = per_batch(kg.trip[:, 0]) + per_batch(kg.trip[:, 1])
    det = 3 * min(int(math.ceil(float(occ.max().item()))), 2 * int(batch))
    lam = 2.0 * batch / max(n_ent, 1)
    corr = min(2 * int(batch), int(math.ceil((tail or _tail)(lam))))
    return det + corr


def _tail8(mu):
    """A tighter tail for the int8x4 entity sums' choice (mu + 8 sqrt(mu) +
    20: a Poisson count passes it with probability < 1e-15): the choice only
    trades atomic bytes, and a count past 127 is still caught by the apply
    (the runner raises, use SKGE_PIPE_E8=0)."""
    return mu + 8.0 * mu ** 0.5 + 20.0


def _tail(mu):
    """Poisson/binomial upper tail used for the random parts of the count
    bounds: mu + 12 sqrt(mu) + 40 (never reached in practice; the applies
    still check every count at run time)."""
    return mu + 12.0 * mu ** 0.5 + 40.0


def relation_replicas(kg, n_rel, batch, max_reps=32, ranks=1):
    """Accumulator copies the packed relation sums need (the two-launch
    runner; the pipelined runner switches to int32x2 sums when this is not 1).
    Positive j adds into copy j mod reps, so a copy of a (union, over `ranks`)
    batch holds per = ranks * ceil(batch / reps) positives; relation p's count
    among them is at most min(per, count_p) and, the batch being a uniform
    sample of the triples, below the binomial tail of mu = per * count_p / T.
    Each positive adds <= 4 to its relation's count.  Returns 0 when even
    max_reps copies cannot keep 4 * bound <= PACKED_MAX."""
    cnt = _bincount_max(kg.trip[:, 2], n_rel).double()
    T = float(max(int(kg.trip.shape[0]), 1))
    reps = 1
    while True:
        per = float(int(ranks) * -(-int(batch) // reps))
        mu = cnt * (per / T)
        tail = mu + 12.0 * torch.sqrt(mu) + 40.0
        bound = torch.minimum(torch.minimum(cnt, torch.full_like(cnt, per)), tail)
        if 4.0 * float(bound.max().item()) <= PACKED_MAX:
            return reps
        reps *= 2
        if reps > max_reps:
            return 0


def padded_width(d):
    """Row width the quad-layout runners use for a d % 4 != 0 table: the next
    multiple of 32 floats (whole 128-B lines: config 1's d = 50 -> 64, 256-B
    rows; same box, WN18 SGD: 128.4 M vs 122.1 M triples/s at 52) when that
    costs at most 30% more row bytes, else the next multiple of 4.
    SKGE_PIPE_PAD_TO (A/B) forces the rounding (4: the round-3 width)."""
    force = _os.environ.get("SKGE_PIPE_PAD_TO")
    if force:
        k = max(4, int(force) // 4 * 4)
        return (d + k - 1) // k * k
    d32 = (d + 31) // 32 * 32
    return d32 if d32 <= 1.3 * d else (d + 3) // 4 * 4


class EpochRunner(object):
    """Native hipGraph epoch of the TransE device batch loop (keeps no per-row
    counters).

    pipelined: None (auto) uses the one-launch-per-batch pipelined runner
    (skge_pipe_runner_*) whenever it applies (TransE-L1, packed accumulators,
    single-copy relation accumulator) and the two-launch runner otherwise;
    True demands it, False forces the two-launch runner.  Both give identical
    parameters.

    Packed (exact int16x4) entity sums are used for TransE-L1 unless
    force_f32, or unless packed_count_bound() says a row's per-batch count
    could pass 32767 (then fp32 sums: packed=None decides, packed=True
    insists).  The pipelined runner keeps relation sums as int32x2; the
    two-launch runner spreads them over relation_replicas() copies.
    """

    counters = False

    def __init__(self, model, updaters, kg, nbatches, seed=0, ntries=100, stream=None,
                 nviol_total=None, force_f32=False, replicas=1, pipelined=None, packed=None):
        from .transe import TransE
        if not isinstance(model, TransE):
            raise NotImplementedError("device_loop supports TransE (the north-star path) only")
        dev = model.device
        self.stream = stream if stream is not None else torch.cuda.Stream(device=dev)
        self.kg = kg
        self.model = model
        self.seed, self.ntries = int(seed) & (2 ** 64 - 1), int(ntries)
        self.epoch_key = torch.zeros(1, dtype=torch.int64, device=dev)
        self.nviol_total = nviol_total if nviol_total is not None else \
            torch.zeros(1, dtype=torch.int32, device=dev)
        bs = kg.T // nbatches
        self.nbatches = nbatches
        self._auto = pipelined is None
        self.hot_rows = 0   # pipelined TransE: entity rows with replicated sums (skewed KGs)
        # d % 4 != 0 (e.g. the reference's d = 50): the packed / pipelined
        # runners work on quads, so they run on zero-padded copies of the
        # tables (width rounded up to 4), copied in and out around every run().
        # A zero column stays zero (TransE-L1: sign(0) = 0 contributions, AdaGrad
        # and the projection leave 0 at 0) and adds nothing to a score or norm,
        # so the padded step is the d-wide step.
        self.d_pad = padded_width(model.d)
        self._pad = (bool(model.l1) and model.d % 4 != 0 and not force_f32 and replicas <= 1
                     and pipelined is not False and packed is not False
                     and _os.environ.get("SKGE_PIPE_PAD", "1") != "0")
        # TransE-L1 sign contributions are small integers: exact packed int16x4
        # sums while every row's per-batch count stays <= 32767 (the applies
        # flag a larger count, checked by synchronize())
        can_pack = bool(model.l1) and (model.d % 4 == 0 or self._pad) and not force_f32
        self.count_bound = packed_count_bound(kg, model.E.rows, bs) if can_pack else 0
        auto_packed = packed is None
        if packed is None:
            packed = can_pack and self.count_bound <= PACKED_MAX
        elif packed and not can_pack:
            raise ValueError("packed sums need TransE-L1, d % 4 == 0 and no force_f32")
        packed = bool(packed)
        # the two-launch runner's packed relation sums: hot relations spread
        # over accumulator copies (0: not even 32 copies suffice)
        rel_reps = relation_replicas(kg, model.R.rows, bs) if packed else 1
        E, R = model.params["E"], model.params["R"]
        can_pipe = packed and replicas <= 1 and pipelined is not False
        if pipelined and not can_pipe:
            raise ValueError("pipelined runner needs TransE-L1, d % 4 == 0, packed sums "
                             "and replicas == 1")
        if can_pipe and pipelined is None:
            # the pipelined runner's scratch (auto mode: only if it fits): the
            # epoch's records and, per entity row, k_pipe_fused (rows of <= 64
            # floats, batches of <= 16k slot records; skge_pipeline.hip) three
            # accumulator copies, a second copy of E and its AdaGrad state and a
            # meta word -- k_pipe_batch two accumulator copies (the table's and
            # one more, packed 16- or 8-bit fields) and five words (done word,
            # pending marks and owner marks of both copies)
            torch.cuda.synchronize(dev)
            torch.cuda.empty_cache()
            wd = self.d_pad if self._pad else model.d
            if wd <= 64 and 4 * bs <= 4 * 4096:
                acc = E.rows * (E.width * 2 + 4) + 4 * 4 * bs
                extra = 3 * acc + kg.T * 20 + (64 << 20) + E.rows * (16 + 8 * E.width)
            else:
                e8_est = (packed_count_bound(kg, model.E.rows, bs, _tail8) <= 127 and
                          _os.environ.get("SKGE_PIPE_E8", "1") != "0")
                acc = E.rows * ((wd // 4) * (4 if e8_est else 8) + 4) + 2 * 4 * 4 * bs
                extra = 2 * acc + E.rows * 5 * 4 + kg.T * 20 + (256 << 20)
            can_pipe = extra < torch.cuda.mem_get_info(dev)[0] * 0.9
        torch.cuda.current_stream().synchronize()
        lib = L.lib()
        if can_pipe:
            # relation sums in 16-bit fields while a relation's per-batch count
            # fits them (faster: half the atomics), else int32x2; entity sums in
            # 8-bit fields while every entity's per-batch count is <= 127 (half
            # the atomic bytes again; the apply checks every count)
            e8 = (packed_count_bound(kg, model.E.rows, bs, _tail8) <= 127 and
                  _os.environ.get("SKGE_PIPE_E8", "1") != "0")
            self._tables(model, updaters, packed, 1, rel_w32=rel_reps != 1, ent_i8=e8,
                         pad=self._pad)
            # the tables' zero-filled accumulators were made on the current
            # stream; the runner works on its own (a reused allocation could
            # otherwise hold a freed runner's counts when the first launch runs)
            torch.cuda.current_stream().synchronize()
            self.ent_i8 = e8
            h = lib.skge_pipe_runner_create(
                L.stream_ptr(self.stream), self.te, self.tr,
                self.d_pad if self._pad else model.d, L.ptr(kg.trip), kg.T,
                L.ptr(kg.slots), kg.capacity, int(nbatches), int(seed) & (2 ** 64 - 1),
                L.ptr(self.epoch_key), float(model.margin), int(ntries), L.ptr(self.nviol_total))
            if h:
                self.pipelined = True
                self.handle = h
                self.nlaunches = lib.skge_pipe_runner_nlaunches(h)
                self.hot_rows = lib.skge_pipe_runner_hot_rows(h)
                self.kernel = ("k_pipe_batch", "k_pipe_fused")[lib.skge_pipe_runner_kernel(h)]
                return
            err = lib.skge_last_error().decode()
            if not (self._auto and "allocation" in err):
                raise L.SkgeError("skge_pipe_runner_create: %s" % err)
            # auto mode: out of device memory -> two-launch runner
            self.accE = self.accR = self.te = self.tr = None
            torch.cuda.empty_cache()
        self.pipelined = False
        self.kernel = "k_transe_sample_grad"
        if self._pad:   # the two-launch runner takes any d: no padded copies
            self._pad = False
            packed = packed and model.d % 4 == 0
            rel_reps = relation_replicas(kg, model.R.rows, bs) if packed else 1
        if packed and rel_reps == 0:
            if not auto_packed:
                raise ValueError("packed sums: a relation's per-batch count exceeds what 32 "
                                 "accumulator copies hold; use packed=None or force_f32=True")
            packed = False
        self._tables(model, updaters, packed, max(int(replicas), rel_reps) if packed else replicas)
        torch.cuda.current_stream().synchronize()   # (as above)
        h = lib.skge_runner_create(L.stream_ptr(self.stream), int(bool(model.l1)),
                                   self.te, self.tr,
                                   model.d, L.ptr(kg.trip), kg.T, L.ptr(kg.slots), kg.capacity,
                                   int(nbatches), int(seed) & (2 ** 64 - 1), L.ptr(self.epoch_key),
                                   float(model.margin), int(ntries), None, L.ptr(self.nviol_total))
        if not h:
            raise L.SkgeError("skge_runner_create: %s" % lib.skge_last_error().decode())
        self.handle = h
        self.nlaunches = lib.skge_runner_nlaunches(h)

    def _tables(self, model, updaters, packed, rel_replicas, rel_w32=False, ent_i8=False,
                pad=False):
        """The runner's own accumulators (captured by its graph) and tables
        (pad: over zero-padded copies of the parameters and AdaGrad states)."""
        from .param import Accumulator, table_struct, post_code
        from .base import deterministic
        dev = model.device
        E, R = model.params["E"], model.params["R"]
        if pad:
            class _Padded(object):   # what table_struct reads of a Parameter
                def __init__(self, rows, width):
                    self.rows, self.width = rows, width
                    self.data = torch.zeros((rows, width), dtype=torch.float32, device=dev)
            self._padded = []
            tabs = {}
            for pid, P in (("E", E), ("R", R)):
                u = updaters[pid]
                pp = _Padded(P.rows, self.d_pad)
                st = u.state()
                sp = None if st is None else torch.zeros_like(pp.data)
                self._padded.append((P, pp.data, st, sp))
                tabs[pid] = (u, pp, sp)
            E = tabs["E"][1]
            R = tabs["R"][1]
        mode = L.SKGE_ACC_I16X4 if packed else L.SKGE_ACC_F32
        if not packed and deterministic():   # exact fixed-point sums, one copy
            mode, rel_replicas = L.SKGE_ACC_FX64, 1
        bs = self.kg.T // self.nbatches
        self.accE = Accumulator(E.rows, E.width, dev, slots=4 * bs,
                                mode=L.SKGE_ACC_I8X4 if ent_i8 else mode)
        # relation rows are hot (every positive adds to one of |R| rows): the
        # two-launch runner spreads the adds over `rel_replicas` copies, the
        # pipelined one keeps 32-bit fields (rel_w32)
        self.accR = Accumulator(R.rows, R.width, dev, mode=L.SKGE_ACC_I32X2 if rel_w32 else mode,
                                dense=True, replicas=rel_replicas)
        self.rel_w32 = rel_w32
        self.packed = packed
        if pad:
            def tab(pid, acc):
                u, pp, sp = tabs[pid]
                return table_struct(pp, sp, acc, opt=u.opt, post=post_code(u.param.post),
                                    lr=float(u.learning_rate))
            self.te = tab("E", self.accE)
            self.tr = tab("R", self.accR)
            return
        self.te = updaters["E"].table(self.accE, counters=False)
        self.tr = updaters["R"].table(self.accR, counters=False)

    def _pad_in(self):
        """Padded tables: the model's parameters / states into the copies
        (ordered after the caller's stream)."""
        if not getattr(self, "_pad", False):
            return
        d = self.model.d
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            for P, Pp, st, sp in self._padded:
                Pp[:, :d].copy_(P.data)
                if st is not None:
                    sp[:, :d].copy_(st)

    def _pad_out(self):
        if not getattr(self, "_pad", False):
            return
        d = self.model.d
        with torch.cuda.stream(self.stream):
            for P, Pp, st, sp in self._padded:
                P.data.copy_(Pp[:, :d])
                if st is not None:
                    st.copy_(sp[:, :d])
        torch.cuda.current_stream().wait_stream(self.stream)

    def run(self, nepochs=1):
        """nepochs epochs on the runner's stream, ordered after the caller's
        stream (parameters it wrote) and before its later work."""
        lib = L.lib()
        fn = lib.skge_pipe_runner_run if self.pipelined else lib.skge_runner_run
        self.stream.wait_stream(torch.cuda.current_stream())
        self._pad_in()
        L.check(fn(self.handle, L.stream_ptr(self.stream), int(nepochs)), "runner run")
        self._pad_out()
        torch.cuda.current_stream().wait_stream(self.stream)

    def profile(self, trace_launch=None):
        """Pipelined runner only: one eager epoch with HIP events around every
        launch (trains like run(1)).  Returns (us, stats): per-launch durations
        and [entity rows applied, relation rows applied, violating pairs];
        with trace_launch (1..nb1+1) also the per-wave timestamp trace of that
        launch (include/skge_hip.h, skge_pipe_runner_profile)."""
        if not self.pipelined:
            raise ValueError("profile() needs the pipelined runner")
        import numpy as np
        n = self.nlaunches
        us = np.zeros(n, dtype=np.float32)
        stats = np.zeros((n, 3), dtype=np.int32)
        tr = np.zeros(2 + 6 * self.kg.T + 8 * self.kg.T + 64, dtype=np.uint64) \
            if trace_launch else None
        self.stream.wait_stream(torch.cuda.current_stream())
        EpochRunner._pad_in(self)   # (also HolePipeRunner.profile: no padded tables there)
        L.check(L.lib().skge_pipe_runner_profile(
            self.handle, L.stream_ptr(self.stream), us.ctypes.data, stats.ctypes.data, n,
            int(trace_launch or 0), None if tr is None else tr.ctypes.data,
            0 if tr is None else len(tr)), "runner profile")
        EpochRunner._pad_out(self)
        if trace_launch:
            return us, stats, tr
        return us, stats

    def synchronize(self):
        self.stream.synchronize()
        if not self.pipelined:
            L.check_device_error(L.stream_ptr(self.stream), "epoch runner")
        if self.pipelined:
            rc = L.lib().skge_pipe_runner_error(self.handle, L.stream_ptr(self.stream))
            if rc < 0:
                raise L.SkgeError("pipelined runner: %s" % L.lib().skge_last_error().decode())
            # (the runner is now invalid: later epochs of this run changed
            # nothing and every later run() is refused)
            if rc & 1:
                raise L.SkgeError("pipelined runner: a cross-workgroup wait timed out; the "
                                  "tables hold that epoch's partial updates and the runner "
                                  "refuses further runs")
            if rc & 2:
                raise L.SkgeError("pipelined runner: a row's per-batch count exceeded 32767 "
                                  "(packed sums may have wrapped); the tables hold that "
                                  "epoch's partial updates and the runner refuses further "
                                  "runs; use force_f32=True")

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                self.stream.synchronize()
                lib = L.lib()
                (lib.skge_pipe_runner_destroy if self.pipelined else lib.skge_runner_destroy)(h)
            except Exception:
                pass
            self.handle = None


class HolePipeRunner(object):
    """Pipelined HolE device loop (skge_hole_pipe_runner_create,
    csrc/skge_pipeline.hip k_hole_pipe): the TransE pipelined runner's launch
    structure -- launch g scores batch b (both pairs of a positive per wave,
    k_hole_pos's arithmetic) while batch b-1's rows are applied beside it --
    with fp32 sums.  Same pairs as PairLoopRunner's HolE path (the same
    device draws); parameters equal to fp32 rounding (float atomics add in
    any order).  Needs d % 4 == 0, 4 <= d <= 256.  Keeps no per-row
    counters."""

    pipelined = True
    counters = False   # keeps no per-row counters (updateCounts)

    def __init__(self, model, updaters, kg, nbatches, seed=0, ntries=100, stream=None,
                 nviol_total=None):
        from .hole import HolE
        from .param import Accumulator
        if not isinstance(model, HolE):
            raise TypeError("HolePipeRunner trains HolE")
        dev = model.device
        self.stream = stream if stream is not None else torch.cuda.Stream(device=dev)
        self.kg = kg
        self.model = model
        self.nbatches = nbatches
        self.epoch_key = torch.zeros(1, dtype=torch.int64, device=dev)
        self.nviol_total = nviol_total if nviol_total is not None else \
            torch.zeros(1, dtype=torch.int32, device=dev)
        E, R = model.params["E"], model.params["R"]
        bs = kg.T // nbatches
        self.accE = Accumulator(E.rows, E.width, dev, slots=4 * bs)
        self.accR = Accumulator(R.rows, R.width, dev, dense=True)
        reg = model._reg("pairwise")
        self.te = updaters["E"].table(self.accE, counters=False, rin=reg["E"][0],
                                      rout=reg["E"][1], fixed_div=reg["E"][2])
        self.tr = updaters["R"].table(self.accR, counters=False, rin=reg["R"][0],
                                      rout=reg["R"][1], fixed_div=reg["R"][2])
        torch.cuda.current_stream().synchronize()
        lib = L.lib()
        h = lib.skge_hole_pipe_runner_create(
            L.stream_ptr(self.stream), model._af_code(), self.te, self.tr, model.d,
            L.ptr(kg.trip), kg.T, L.ptr(kg.slots), kg.capacity, int(nbatches),
            int(seed) & (2 ** 64 - 1), L.ptr(self.epoch_key), float(model.margin), int(ntries),
            L.ptr(self.nviol_total))
        if not h:
            raise L.SkgeError("skge_hole_pipe_runner_create: %s" % lib.skge_last_error().decode())
        self.handle = h
        self.nlaunches = lib.skge_pipe_runner_nlaunches(h)
        self.hot_rows = lib.skge_pipe_runner_hot_rows(h)   # hub rows (pair form, skewed KGs)

    @staticmethod
    def eligible(model):
        from .hole import HolE
        d = model.d
        return isinstance(model, HolE) and d % 4 == 0 and 4 <= d <= 256

    def run(self, nepochs=1):
        self.stream.wait_stream(torch.cuda.current_stream())
        L.check(L.lib().skge_pipe_runner_run(self.handle, L.stream_ptr(self.stream),
                                             int(nepochs)), "hole runner run")
        torch.cuda.current_stream().wait_stream(self.stream)

    profile = EpochRunner.profile

    def synchronize(self):
        self.stream.synchronize()
        rc = L.lib().skge_pipe_runner_error(self.handle, L.stream_ptr(self.stream))
        if rc < 0:
            raise L.SkgeError("pipelined HolE runner: %s" % L.lib().skge_last_error().decode())
        if rc & 1:
            raise L.SkgeError("pipelined HolE runner: a cross-workgroup wait timed out; the "
                              "runner refuses further runs")

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                self.stream.synchronize()
                L.lib().skge_pipe_runner_destroy(h)
            except Exception:
                pass
            self.handle = None


def batch_sizes(T, nbatches):
    """Batch sizes of StochasticTrainer._optim's np.split (skge/base.py:1246-1268)."""
    bs = T // nbatches
    return [min(bs, T - s0) for s0 in range(0, T, bs)]


class PairLoopRunner(object):
    """Native hipGraph epoch of the device pair loop for any model
    (skge_pair_runner_*, csrc/skge_pairloop.hip): the epoch's permutation and
    negatives drawn on the device (the same keyed draws as EpochRunner), every
    batch's explicit pairs built once per epoch, then per batch one
    skge_pair_step -- the kernels of the explicit-pair path, so a device epoch
    trains like feeding those pairs to model._pairwise_step.  HolE and RESCAL
    (MFMA) run both pairs of a positive together instead (k_hole_pos,
    k_rescal_pos_scatter: the same pairs, contributions and counts; the env
    switches SKGE_HOLE_PAIRS=1 / SKGE_RESCAL_PAIRS=1 select the explicit
    pairs).  The per-row counters (updateCounts, TransE violations) are kept
    as on that path."""

    pipelined = False
    counters = True    # updateCounts / TransE violations, as on the per-batch path

    def __init__(self, model, updaters, kg, nbatches, seed=0, ntries=100, stream=None,
                 nviol_total=None):
        dev = model.device
        self.stream = stream if stream is not None else torch.cuda.Stream(device=dev)
        self.kg = kg
        self.model = model
        self.nbatches = nbatches
        self.epoch_key = torch.zeros(1, dtype=torch.int64, device=dev)
        self.nviol_total = nviol_total if nviol_total is not None else \
            torch.zeros(1, dtype=torch.int32, device=dev)
        P = 2 * max(batch_sizes(kg.T, nbatches))
        self.te, self.tr = model._tables("pairwise", updaters, slots=model._pair_slots(P))
        # the graph captures raw pointers to the model's accumulators and
        # counters: hold the tensors, so a later per-batch call that grows the
        # model's slot arrays cannot free what this runner still writes
        self._captured = [(a.sum, a.cnt, a.touched) for a in model._acc.values()] + \
            [p._counters.copy() for p in model.params.values()]
        torch.cuda.current_stream().synchronize()
        lib = L.lib()
        h = lib.skge_pair_runner_create(
            L.stream_ptr(self.stream), model._kernel_model(), model._af_code(), self.te, self.tr,
            model.d, L.ptr(kg.trip), kg.T, L.ptr(kg.slots), kg.capacity, int(nbatches),
            int(seed) & (2 ** 64 - 1), L.ptr(self.epoch_key), float(model.margin), int(ntries),
            L.ptr(self.nviol_total))
        if not h:
            raise L.SkgeError("skge_pair_runner_create: %s" % lib.skge_last_error().decode())
        self.handle = h
        self.nlaunches = lib.skge_pair_runner_nlaunches(h)

    def run(self, nepochs=1):
        self.stream.wait_stream(torch.cuda.current_stream())
        L.check(L.lib().skge_pair_runner_run(self.handle, L.stream_ptr(self.stream),
                                             int(nepochs)), "pair runner run")
        torch.cuda.current_stream().wait_stream(self.stream)

    def synchronize(self):
        self.stream.synchronize()
        L.check_device_error(L.stream_ptr(self.stream), "pair-loop runner")

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                self.stream.synchronize()
                L.lib().skge_pair_runner_destroy(h)
            except Exception:
                pass
            self.handle = None


def epoch_records(kg, n_ent, seed, epoch_key, ntries=100, stream=None):
    """The epoch's positives and draws as the device loops make them:
    (rec [T, 4] = (s, o, p, s' or -1), rec_n1 [T] = o' or -1) on the device."""
    dev = kg.trip.device
    rec = torch.empty((kg.T, 4), dtype=torch.int32, device=dev)
    rec_n1 = torch.empty(kg.T, dtype=torch.int32, device=dev)
    ek = torch.tensor([int(epoch_key)], dtype=torch.int64, device=dev)
    L.check(L.lib().skge_epoch_sample(L.stream_ptr(stream), L.ptr(kg.trip), kg.T, L.ptr(kg.slots),
                                      kg.capacity, int(n_ent), int(seed) & (2 ** 64 - 1),
                                      L.ptr(ek), int(ntries), L.ptr(rec), L.ptr(rec_n1)),
            "epoch sample")
    return rec, rec_n1


def make_runner(model, updaters, kg, nbatches, seed=0, ntries=100, nviol_total=None,
                runner="auto"):
    """runner: 'auto' (TransE -> EpochRunner, the fused sampler/score runners;
    HolE -> HolePipeRunner where it applies, RESCAL -> PairLoopRunner),
    'epoch', 'hole_pipe' or 'pairs'."""
    from .transe import TransE
    from .base import deterministic
    if runner == "auto":
        runner = "epoch" if isinstance(model, TransE) else \
            ("hole_pipe" if HolePipeRunner.eligible(model) and not deterministic() else "pairs")
    if runner == "hole_pipe":
        return HolePipeRunner(model, updaters, kg, nbatches, seed=seed, ntries=ntries,
                              nviol_total=nviol_total)
    if runner == "epoch":
        return EpochRunner(model, updaters, kg, nbatches, seed=seed, ntries=ntries,
                           nviol_total=nviol_total)
    if runner == "pairs":
        return PairLoopRunner(model, updaters, kg, nbatches, seed=seed, ntries=ntries,
                              nviol_total=nviol_total)
    raise ValueError("unknown device runner %r" % (runner,))


def device_sampler_args(trainer, xs, ys):
    """(eligible, ntries, reason): whether PairwiseStochasticTrainer.fit with
    device_loop=True may run the device loop, whose sampler draws what
    RandomModeSampler(1, [0, 1], xs, sz).sample would (skge/sample.py:28-46,
    skge/base.py:426).  Needed: every y is +1, samplef is such a sampler's
    sample, and the sampler rejects against the same training triples the
    device loop does (its xs == the fit's xs).  samplef None is the
    reference's labelled-negatives branch (skge/base.py:1350-1357: positives
    paired with the given y != 1 rows; with none it builds no pairs), which
    the device loop does not mirror."""
    if ys is not None and not np.all(np.asarray(ys) == 1):
        return False, trainer.ntries, "labelled negatives (y != 1)"
    f = trainer.samplef
    if f is None:
        return False, trainer.ntries, ("samplef is None (the labelled-negatives branch, "
                                       "skge/base.py:1350-1357); pass samplef="
                                       "RandomModeSampler(1, [0, 1], xs, sz).sample")
    from .sample import RandomModeSampler
    smp = getattr(f, "__self__", None)
    if not isinstance(smp, RandomModeSampler) or getattr(f, "__func__", None) is not \
            RandomModeSampler.sample:
        return False, trainer.ntries, "samplef is not RandomModeSampler.sample"
    if smp.n != 1 or list(smp.modes) != [0, 1]:
        return False, trainer.ntries, "RandomModeSampler(n=%r, modes=%r) is not (1, [0, 1])" % (
            smp.n, smp.modes)
    n_ent = trainer.model.E.rows
    if tuple(smp.sz[:2]) != (n_ent, n_ent):
        return False, trainer.ntries, "sampler sizes %r differ from the model's" % (smp.sz,)
    fit_set = set(tuple(int(v) for v in x) for x in
                  np.asarray(xs, dtype=np.int64).reshape(-1, 3).tolist())
    if fit_set != smp.xs:
        return False, trainer.ntries, ("the sampler's rejection set differs from the fit's "
                                       "triples (the device sampler rejects against xs)")
    return True, smp.ntries, ""


def device_optim(trainer, xs, ntries=None):
    """PairwiseStochasticTrainer.fit with device_loop=True.  The runner's
    error word (packed-sum overflow, cross-workgroup wait timeout) is read
    after every epoch, before the post_epoch callbacks, so no callback ever
    sees parameters from a failed epoch."""
    model = trainer.model
    dev = model.device
    if trainer._nviol_dev is None:
        trainer._nviol_dev = torch.zeros(1, dtype=torch.int32, device=dev)
    kg = DeviceKG(xs, dev)
    which = trainer.device_runner
    if which == "auto" and trainer.file_gradients is not None:
        # file_grad's #(violations) / #(updates) columns need the per-row
        # counters, which only the pair loop keeps (file_grad=None: the
        # fused / pipelined runners)
        which = "pairs"
    runner = make_runner(model, trainer._updaters, kg, trainer.nbatches, seed=trainer.seed,
                         ntries=trainer.ntries if ntries is None else ntries,
                         nviol_total=trainer._nviol_dev, runner=which)
    trainer._runner = runner
    with torch.cuda.stream(runner.stream):
        for trainer.epoch in range(1, trainer.max_epochs + 1):
            trainer._pre_epoch()
            trainer.epoch_start = timeit.default_timer()
            runner.run(1)
            runner.synchronize()   # raises on the epoch's error bits
            for f in trainer.post_epoch:
                if not f(trainer):
                    break
