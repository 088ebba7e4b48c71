"""Data-parallel TransE-L1: ONE model trained over the G GPUs of a node
(the WN18 tables are small, so every rank holds
the whole model).

The reference trains one process on one table: every mini-batch is scored,
its gradients segment-meaned and applied before the next batch starts
(PairwiseStochasticTrainer._process_batch + _batch_step, skge/base.py:1394-1427
and 1306-1316).  Here every rank draws the SAME epoch order and negatives
(the keyed device sampler, one seed), and each union batch [start, start +
count) is split into G slices.  Per union batch b, on every rank:

    launch    ONE launch of the one-GPU pipelined runner (k_pipe_batch in
              its data-parallel form): apply union batch b-1's rows while
              scoring the rank's slice of batch b -- its contributions added
              locally, one record per positive written for the others  [HIP]
    gather    the G slices' records, all-gathered                        [RCCL]
    scatter   the OTHER ranks' positives added into the same exact packed
              sums, counts, slot records and pending marks (none at G = 1) [HIP]

and the epoch ends with the flush (applies the last batch).  A record is the
positive's violation flags and, if it violates, its three sign vectors as
2-bit codes (208 B at d = 200); the header (s, o, p, s', o') every rank has
from the common epoch draws.  The scatter runs the scoring wave's own commit
code, and TransE-L1's sums are exact integers, so every replica ends each
batch with the parameters ONE GPU computes for that union batch -- bit for
bit (tests).  Round 5's form (score, all-gather, scatter, apply: four serial
phases, three launches) took ~60 us of kernels per union batch against 8.6
us for the one-GPU launch; this one is that launch plus the exchange.

The protocol (`dp_epoch`) is written against two small interfaces -- the
rank's compute (`DPOps`) and the collective (`DPExchange`) -- so a CPU test
drives the same protocol over gloo with a NumPy compute stand-in
(tests/dp_numpy.py).  Under the "nccl" backend (RCCL) the whole epoch --
kernels and all-gathers -- is captured in one hipGraph per rank.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L

SKGE_PIPE_DP = 1   # skge_pipe_runner_create_ex flag (include/skge_hip.h)


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
        whenever a process group exists, also at G == 1).  inp may be this
        rank's slice of out (in place)."""
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


def dp_epoch(ops, ex, batches):
    """One epoch of the data-parallel job over the union batches (start,
    count) of the common epoch order; see the module docstring.  Launch b
    applies union batch b-1 and scores this rank's slice of batch b (its own
    contributions added locally); the slices' records are all-gathered (a
    real collective whenever a process group exists, also at G == 1) and the
    other ranks' positives added; the flush applies the last batch."""
    ops.begin()
    grouped = ex.backend is not None
    for b, (start, count) in enumerate(batches):
        share, lo, hi = slice_of(count, ex.G, ex.rank)
        remote = grouped and ex.G > 1
        send = ops.batch(b, start, count, lo, hi, share, fold=not remote)
        if grouped:
            recs = ops.gathered(ex, send, share)
            if remote:
                ops.scatter(b, start, count, recs, lo, hi)
    ops.flush(len(batches))
    ops.end()


class DPOps(object):
    """The HIP compute of one rank: the pipelined runner's data-parallel form
    (skge_pipe_runner_dp_*, csrc/skge_pipeline.hip: k_pipe_batch over the
    rank's slice with record output, k_pipe_dp_scatter for the other ranks'
    records)."""

    def __init__(self, runner):
        self.r = runner

    def begin(self):
        r = self.r
        L.check(L.lib().skge_pipe_runner_dp_begin(r.handle, r.sp), "dp begin")

    def batch(self, b, start, count, lo, hi, share, fold):
        # the records go straight into this rank's slot of the gather buffer
        # (an in-place all-gather: no copy of the own slice; at G = 1 none)
        r = self.r
        rb = r.rec_bytes
        off = r.rank * share * rb
        L.check(L.lib().skge_pipe_runner_dp_batch(r.handle, r.sp, b, lo, hi,
                                                  L.ptr(r.recv[off:off + max(share, 1) * rb]),
                                                  int(bool(fold))), "dp batch")
        return r.recv[off:off + share * rb]

    def gathered(self, ex, send, share):
        r = self.r
        out = r.recv[:ex.G * share * r.rec_bytes]
        return ex.all_gather(out, send)

    def scatter(self, b, start, count, recs, lo, hi):
        r = self.r
        L.check(L.lib().skge_pipe_runner_dp_scatter(r.handle, r.sp, b, L.ptr(recs), lo, hi),
                "dp scatter")

    def flush(self, nb):
        r = self.r
        L.check(L.lib().skge_pipe_runner_dp_batch(r.handle, r.sp, nb, 0, 0, None, 0), "dp flush")

    def end(self):
        r = self.r
        L.check(L.lib().skge_pipe_runner_dp_end(r.handle, r.sp), "dp end")


class DataParallelRunner(object):
    """TransE-L1 PairwiseStochasticTrainer epochs (margin, strict >,
    RandomModeSampler(1, [0, 1]) negatives drawn on the device) of ONE model
    replicated over the ranks of a process group.

    Every rank passes the same initial model, updaters' learning rate, KG,
    nbatches and seed; the union batches follow np.split's geometry over the
    KG (skge/base.py:1246-1268).  The rank's compute is the one-GPU pipelined
    runner in its data-parallel form (one launch per union batch: apply of
    the previous batch + scoring of the rank's slice; then the all-gather of
    the slices' records and the other ranks' positives added).  capture:
    None (auto) captures each rank's epoch -- kernels and RCCL all-gathers --
    into one CUDA graph under the "nccl" backend (or with no process group),
    and runs eagerly under gloo.
    """

    def __init__(self, model, updaters, kg, nbatches, seed=0, ntries=100, group=None, stream=None,
                 capture=None):
        from .transe import TransE
        from .device import (EpochRunner, packed_count_bound, relation_replicas, padded_width,
                             _tail8, PACKED_MAX)
        import os
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
        self.d_pad = padded_width(int(model.d))
        self._pad = model.d % 4 != 0
        self.d = self.d_pad if self._pad else int(model.d)
        self.margin = float(model.margin)
        self.seed = int(seed) & (2 ** 64 - 1)
        self.ntries = int(ntries)
        T = kg.T
        if not 1 <= nbatches <= T:
            raise ValueError("nbatches must be in [1, T]")
        self.nbatches = nbatches
        bs = T // nbatches
        self.batches = [(s0, min(bs, T - s0)) for s0 in range(0, T, bs)]
        if packed_count_bound(kg, model.E.rows, bs) > PACKED_MAX:
            raise ValueError("data-parallel runner: an entity's per-batch count could pass 32767 "
                             "(exact packed sums); use more batches")
        rel_reps = relation_replicas(kg, model.R.rows, bs)
        if rel_reps == 0:
            raise ValueError("data-parallel runner: a relation's per-batch count exceeds what 32 "
                             "packed accumulator copies hold; use more batches")
        e8 = (packed_count_bound(kg, model.E.rows, bs, _tail8) <= 127 and
              os.environ.get("SKGE_PIPE_E8", "1") != "0")
        # the one-GPU pipelined runner's tables (same encodings: the same sums)
        EpochRunner._tables(self, model, updaters, True, 1, rel_w32=rel_reps != 1, ent_i8=e8,
                            pad=self._pad)
        self.rec_bytes = int(L.lib().skge_pipe_dp_record_bytes(self.d))
        share_max = -(-bs // self.G)
        self.recv = torch.zeros((self.G * max(share_max, 1) + 1) * self.rec_bytes,
                                dtype=torch.uint8, device=dev)
        self.nviol_total = torch.zeros(1, dtype=torch.int32, device=dev)   # this rank's slices
        self.epoch_key = torch.zeros(1, dtype=torch.int64, device=dev)
        torch.cuda.current_stream(dev).synchronize()   # the zero fills, before the runner's stream
        h = L.lib().skge_pipe_runner_create_ex(
            self.sp, self.te, self.tr, self.d, L.ptr(kg.trip), kg.T, L.ptr(kg.slots), kg.capacity,
            int(nbatches), self.seed, L.ptr(self.epoch_key), self.margin, self.ntries,
            L.ptr(self.nviol_total), SKGE_PIPE_DP)
        if not h:
            raise L.SkgeError("data-parallel runner: %s" % L.lib().skge_last_error().decode())
        self.handle = h
        self.ops = DPOps(self)
        if capture is None:
            capture = self.ex.backend in (None, "nccl")
        self.capture = bool(capture)
        self.graph = None
        # launches per epoch: the draw, nb1 batch launches (+ nb1 remote
        # scatters when G > 1), the flush, the key advance
        nb1 = len(self.batches)
        self.nlaunches = nb1 * (2 if self.G > 1 else 1) + 3
        self.ncollectives = nb1 if self.ex.backend is not None else 0

    # ---- one epoch ----
    def _epoch(self):
        dp_epoch(self.ops, self.ex, self.batches)

    def _pad_in(self):
        from .device import EpochRunner
        EpochRunner._pad_in(self)

    def _pad_out(self):
        from .device import EpochRunner
        EpochRunner._pad_out(self)

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
        rc = L.lib().skge_pipe_runner_error(self.handle, self.sp)
        if rc < 0:
            raise L.SkgeError("data-parallel runner: %s" % L.lib().skge_last_error().decode())
        if rc & 1:
            raise L.SkgeError("data-parallel runner: a cross-workgroup wait timed out; the "
                              "runner refuses further runs")
        if rc & 2:
            raise L.SkgeError("data-parallel runner: a row's per-batch count exceeded 32767 "
                              "(packed sums may have wrapped); the runner refuses further runs")

    def total_violations(self):
        """Violating pairs of all ranks (every pair is scored by one rank)."""
        return self.ex.sum_int(int(self.nviol_total.item()))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                self.graph = None
                self.stream.synchronize()
                L.lib().skge_pipe_runner_destroy(h)
            except Exception:
                pass
            self.handle = None
