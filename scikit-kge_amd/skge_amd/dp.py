"""Data-parallel TransE-L1: ONE model trained over the G GPUs of a node
(the WN18 tables are small, so every rank holds
the whole model).

The reference trains one process on one table: every mini-batch is scored,
its gradients segment-meaned and applied before the next batch starts
(PairwiseStochasticTrainer._process_batch + _batch_step, skge/base.py:1394-1427
and 1306-1316).  Here every rank draws the SAME epoch order and negatives
(the keyed device sampler, one seed), and each union batch [start, start +
count) is split into G slices:

    score     rank g scores its slice: sampler, L1 scores, strict margin
              test, sign sub-gradients -> one record per positive        [HIP]
    gather    the G slices' records, all-gathered                        [RCCL]
    scatter   every rank adds the whole batch's records into its exact
              packed row sums, counts and touched slots                  [HIP]
    apply     segment mean + AdaGrad + normalize of every touched row    [HIP]

A record is the positive's (s, o, p, s', o'), its violation flags and, if it
violates, its three sign vectors as 2-bit codes (240 B at d = 200).  The
scatter runs the one-GPU kernel's own commit code over the union batch, and
TransE-L1's sums are exact integers, so every replica ends each batch with
the parameters ONE GPU computes for that union batch -- bit for bit (tests).

The protocol (`dp_step`) is written against two small interfaces -- the
rank's compute (`DPOps`) and the collective (`DPExchange`) -- so a CPU test
drives the same protocol over gloo with a NumPy compute stand-in
(tests/dp_numpy.py).  Under the "nccl" backend (RCCL) the whole epoch --
kernels and all-gathers -- is captured in one hipGraph per rank.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L


def slice_of(count, G, rank):
    """Rank `rank`'s slice [lo, hi) of a union batch of `count` positives:
    contiguous slices of ceil(count / G), so after the all-gather the record of
    batch position w sits at index w (slots past `count` are never read)."""
    share = -(-int(count) // int(G)) if count else 0
    lo = min(rank * share, count)
    hi = min((rank + 1) * share, count)
    return share, lo, hi


class DPExchange(object):
    """The one collective of a data-parallel step: all-gather of equal-size
    byte slices over a torch.distributed group (RCCL under "nccl"; gloo
    stages device tensors through host memory).  G == 1: the identity."""

    def __init__(self, group=None):
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.G = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
            self.backend = dist.get_backend(group)
        else:
            self.G, self.rank, self.backend = 1, 0, None

    def all_gather(self, out, inp):
        """out [G * n] <- every rank's inp [n], rank-major (a real collective
        whenever a process group exists, also at G == 1)."""
        if self.backend is None:
            if out.data_ptr() != inp.data_ptr():
                out[:inp.numel()].copy_(inp)
            return out
        if self.backend == "gloo" and inp.is_cuda:
            h = torch.empty(out.shape, dtype=out.dtype)
            dist.all_gather_into_tensor(h, inp.cpu(), group=self.group)
            out.copy_(h)
        else:
            dist.all_gather_into_tensor(out, inp, group=self.group)
        return out

    def sum_int(self, x):
        """Sum of a host int over the ranks (violation totals)."""
        if self.G == 1:
            return int(x)
        dev = "cpu" if self.backend == "gloo" else torch.device("cuda", torch.cuda.current_device())
        t = torch.tensor([int(x)], dtype=torch.int64, device=dev)
        dist.all_reduce(t, group=self.group)
        return int(t.item())


def dp_step(ops, ex, start, count):
    """One union batch of the data-parallel job (positions start .. start +
    count of the common epoch order); see the module docstring."""
    share, lo, hi = slice_of(count, ex.G, ex.rank)
    send = ops.score(start, count, lo, hi, share)     # [share] records of this rank
    recs = ops.gathered(ex, send, share)              # [G * share] records, rank-major
    ops.scatter(start, count, recs)
    ops.apply(count)


class DPOps(object):
    """The HIP compute of one rank (skge_dp_score / skge_dp_scatter /
    skge_accum_apply, csrc/skge_epoch.hip, skge_update.hip)."""

    def __init__(self, runner):
        self.r = runner

    def score(self, start, count, lo, hi, share):
        r = self.r
        rb = r.rec_bytes
        send = r.send[:share * rb]
        L.check(L.lib().skge_dp_score(r.sp, r.te, r.tr, r.d, L.ptr(r.kg.trip), r.kg.T,
                                      L.ptr(r.kg.slots), r.kg.capacity, start, count, lo, hi,
                                      r.seed, L.ptr(r.epoch_key), r.margin, r.ntries,
                                      L.ptr(r.vshards), L.ptr(send)), "dp score")
        return send

    def gathered(self, ex, send, share):
        r = self.r
        if ex.backend is None:       # one process: the slice is the batch
            return send
        out = r.recv[:ex.G * share * r.rec_bytes]
        return ex.all_gather(out, send)

    def scatter(self, start, count, recs):
        r = self.r
        L.check(L.lib().skge_dp_scatter(r.sp, r.te, r.tr, r.d, start, count, L.ptr(recs)),
                "dp scatter")

    def apply(self, count):
        r = self.r
        L.check(L.lib().skge_accum_apply(r.sp, (L.SkgeTable * 2)(r.te, r.tr), 2,
                                         L.int_array(4 * count, count)), "dp apply")


class _PaddedParam(object):
    """What table_struct reads of a Parameter: a zero-padded fp32 copy."""

    def __init__(self, rows, width, dev):
        self.rows, self.width = rows, width
        self.data = torch.zeros((rows, width), dtype=torch.float32, device=dev)


class DataParallelRunner(object):
    """TransE-L1 PairwiseStochasticTrainer epochs (margin, strict >,
    RandomModeSampler(1, [0, 1]) negatives drawn on the device) of ONE model
    replicated over the ranks of a process group.

    Every rank passes the same initial model, updaters' learning rate, KG,
    nbatches and seed; the union batches follow np.split's geometry over the
    KG (skge/base.py:1246-1268).  capture: None (auto) captures each rank's
    epoch -- kernels and RCCL all-gathers -- into one CUDA graph under the
    "nccl" backend (or with no process group), and runs eagerly under gloo.
    """

    def __init__(self, model, updaters, kg, nbatches, seed=0, ntries=100, group=None, stream=None,
                 capture=None):
        from .transe import TransE
        from .param import Accumulator, table_struct, post_code
        from .device import packed_count_bound, relation_replicas, PACKED_MAX
        if not isinstance(model, TransE) or not model.l1 or model.d > 1024:
            raise ValueError("data-parallel runner: TransE-L1 with d <= 1024")
        self.ex = DPExchange(group)
        self.G, self.rank = self.ex.G, self.ex.rank
        self.model, self.kg = model, kg
        dev = model.device
        self.device = dev
        self.stream = stream if stream is not None else torch.cuda.Stream(device=dev)
        self.sp = L.stream_ptr(self.stream)
        # d % 4 != 0 (the reference's d = 50): the kernels work on quads, so
        # they run on zero-padded copies of the tables and AdaGrad states (as
        # device.EpochRunner does), copied in and out around every run().  A
        # zero column stays zero (sign(0) = 0 contributions, AdaGrad and the
        # projection keep 0 at 0) and adds nothing to a score or a norm.
        from .device import padded_width
        self.d = int(model.d) if model.d % 4 == 0 else padded_width(int(model.d))
        self._pad = self.d != int(model.d)
        self.margin = float(model.margin)
        self.seed = int(seed) & (2 ** 64 - 1)
        self.ntries = int(ntries)
        T = kg.T
        if not 1 <= nbatches <= T:
            raise ValueError("nbatches must be in [1, T]")
        bs = T // nbatches
        self.batches = [(s0, min(bs, T - s0)) for s0 in range(0, T, bs)]
        if packed_count_bound(kg, model.E.rows, bs) > PACKED_MAX:
            raise ValueError("data-parallel runner: an entity's per-batch count could pass 32767 "
                             "(exact packed sums); use more batches")
        reps = relation_replicas(kg, model.R.rows, bs)
        if reps == 0:
            raise ValueError("data-parallel runner: a relation's per-batch count exceeds what 32 "
                             "packed accumulator copies hold; use more batches")
        E, R = model.params["E"], model.params["R"]
        self.accE = Accumulator(E.rows, self.d, dev, slots=4 * bs, mode=L.SKGE_ACC_I16X4)
        self.accR = Accumulator(R.rows, self.d, dev, mode=L.SKGE_ACC_I16X4, dense=True,
                                replicas=reps)
        if self._pad:
            self._padded = []
            tabs = []
            for pid, acc in (("E", self.accE), ("R", self.accR)):
                u, P = updaters[pid], model.params[pid]
                pp = _PaddedParam(P.rows, self.d, dev)
                st = u.state()
                sp = None if st is None else torch.zeros_like(pp.data)
                self._padded.append((P, pp.data, st, sp))
                tabs.append(table_struct(pp, sp, acc, opt=u.opt, post=post_code(u.param.post),
                                         lr=float(u.learning_rate)))
            self.te, self.tr = tabs
        else:
            self.te = updaters["E"].table(self.accE, counters=False)
            self.tr = updaters["R"].table(self.accR, counters=False)
        self.rec_bytes = int(L.lib().skge_dp_record_bytes(self.d))
        share_max = -(-bs // self.G)
        self.send = torch.zeros(max(share_max, 1) * self.rec_bytes, dtype=torch.uint8, device=dev)
        self.recv = torch.zeros(self.G * max(share_max, 1) * self.rec_bytes, dtype=torch.uint8,
                                device=dev)
        self.vshards = torch.zeros(64 * 32, dtype=torch.int32, device=dev)
        self.nviol_total = torch.zeros(1, dtype=torch.int32, device=dev)   # this rank's slices
        self.epoch_key = torch.zeros(1, dtype=torch.int64, device=dev)
        self.ops = DPOps(self)
        if capture is None:
            capture = self.ex.backend in (None, "nccl")
        self.capture = bool(capture)
        self.graph = None
        self.nlaunches = 3 * len(self.batches) + 2
        self.ncollectives = len(self.batches) if self.ex.backend is not None else 0
        torch.cuda.current_stream(dev).synchronize()

    # ---- one epoch ----
    def _epoch(self):
        for start, count in self.batches:
            dp_step(self.ops, self.ex, start, count)
        L.check(L.lib().skge_shard_fold_violations(self.sp, L.ptr(self.vshards),
                                                   L.ptr(self.nviol_total)), "dp fold")
        L.check(L.lib().skge_epoch_advance(self.sp, L.ptr(self.epoch_key)), "dp advance")

    def _pad_in(self):
        if not self._pad:
            return
        d = self.model.d
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            for P, Pp, st, sp in self._padded:
                Pp[:, :d].copy_(P.data)
                if st is not None:
                    sp[:, :d].copy_(st)

    def _pad_out(self):
        if not self._pad:
            return
        d = self.model.d
        with torch.cuda.stream(self.stream):
            for P, Pp, st, sp in self._padded:
                P.data.copy_(Pp[:, :d])
                if st is not None:
                    st.copy_(sp[:, :d])
        torch.cuda.current_stream().wait_stream(self.stream)

    def run(self, nepochs=1):
        # ordered after the caller's stream (parameters it wrote), and its later
        # work after the epochs
        self.stream.wait_stream(torch.cuda.current_stream())
        self._pad_in()
        self._run(nepochs)
        self._pad_out()
        torch.cuda.current_stream().wait_stream(self.stream)

    def _run(self, nepochs):
        with torch.cuda.stream(self.stream):
            for _ in range(int(nepochs)):
                if not self.capture:
                    self._epoch()
                    continue
                if self.graph is None:
                    # first epoch eagerly (communicator / allocator warm-up), then capture
                    self._epoch()
                    self.stream.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=self.stream):
                        self._epoch()
                    # capture recorded the epoch without running it
                    self.graph = g
                    continue
                self.graph.replay()

    def synchronize(self):
        self.stream.synchronize()
        rc = L.lib().skge_device_error(self.sp, 1)
        if rc & 2:
            raise L.SkgeError("data-parallel runner: a row's per-batch count exceeded 32767 "
                              "(packed sums may have wrapped)")

    def total_violations(self):
        """Violating pairs of all ranks (every pair is scored by one rank)."""
        return self.ex.sum_int(int(self.nviol_total.item()))
