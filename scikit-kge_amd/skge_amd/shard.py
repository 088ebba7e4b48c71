"""Row-sharded TransE-L1 training over the GPUs of one node (SURVEY.md 8(e),
BASELINE.json configs[4]: the entity table sharded over 8 MI355X, gradients
reduce-scattered over RCCL/xGMI).

The reference trains one process on one table (skge/base.py:1242-1291,
1394-1427).  Here the entity table E and its AdaGrad state are split by row
over the ranks of a process group -- rank g owns the rows r with
r % G == g, at local index r // G -- and the relation table R (|R| x d,
20 MB at config 5) is replicated.  Every rank holds its own share of the
training triples; mini-batch b of the job is the union of every rank's
batch b, and one step of it is

    route     requests (s, o, s', o') of the rank's positives into G
              fixed-capacity owner buckets                               [HIP]
    a2a       request ids -> owners                                      [RCCL]
    gather    owners copy the requested rows out of their shard          [HIP]
    a2a       rows -> requesters                                         [RCCL]
    score     scores, margin test, exact int8 contributions, local R sums [HIP]
    a2a       contributions -> owners (the sparse reduce-scatter)        [RCCL]
    accum     owners add them into their exact packed row sums           [HIP]
    allreduce R sums and counts                                          [RCCL]
    apply     segment mean + AdaGrad + normalize, E shard and R          [HIP]

TransE-L1's contributions are small integers, so every sum is exact: the
parameters after a step are, bit for bit, those one GPU computes for the union
batch (the segment mean of skge/util.py:53-101 over all ranks' pairs), and
the R replicas stay identical.  The exchange protocol (`sharded_step`) is
written against two small interfaces -- the rank's compute (`ShardOps`) and
the collectives (`Exchange`) -- so the CPU tests drive the same protocol over
gloo with a NumPy compute stand-in.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L


def owned_rows(n_ent, G, rank):
    """Number of entity rows rank `rank` owns (rows r with r % G == rank)."""
    return (n_ent - rank + G - 1) // G if rank < n_ent else 0


class Exchange(object):
    """The collectives of one sharded step over a torch.distributed group
    (RCCL under the "nccl" backend; gloo stages device tensors through host
    memory).  Every all-to-all moves G EQUAL slices (the fixed-capacity
    layout), so no split sizes travel to the host and the step is
    graph-capturable.  G == 1 needs no process group: every exchange is the
    identity."""

    def __init__(self, group=None):
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.G = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
            self.backend = dist.get_backend(group)
        else:
            self.G, self.rank, self.backend = 1, 0, None

    def all_to_all(self, inp, out=None):
        """Slice g of inp (G equal slices along dim 0) goes to rank g; returns
        the G slices received, rank-major (into `out` if given)."""
        if self.backend is None:
            return inp
        if out is None:
            out = torch.empty_like(inp)
        if self.backend == "gloo" and inp.is_cuda:
            h = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(h, inp.cpu(), group=self.group)
            out.copy_(h)
        else:
            dist.all_to_all_single(out, inp, group=self.group)
        return out

    def all_reduce_(self, t):
        if self.backend is not None:
            if self.backend == "gloo" and t.is_cuda:
                h = t.cpu()
                dist.all_reduce(h, group=self.group)
                t.copy_(h)
            else:
                dist.all_reduce(t, group=self.group)
        return t


def sharded_step(ops, ex, start, count):
    """One mini-batch of the sharded job (positives start .. start+count of
    this rank's epoch order); see the module docstring.  `ops` is the
    rank's compute, `ex` the collectives.  Fixed-capacity buckets of C
    request slots per owner: no host read anywhere in the step."""
    send_ids, req_pos = ops.route(start, count)         # [G * C] ids (-1: unused slot)
    recv_ids = ex.all_to_all(send_ids, ops.buf("recv_ids"))   # owner side: who wants which row
    rows = ops.gather(recv_ids)
    fetched = ex.all_to_all(rows, ops.buf("fetched"))    # requester side, bucket order
    contrib = ops.score(start, count, fetched, req_pos)  # + this rank's R sums
    recv_contrib = ex.all_to_all(contrib, ops.buf("recv_contrib"))   # sparse reduce-scatter
    ops.accum(recv_ids, recv_contrib)
    for t in ops.rel_sums():
        ex.all_reduce_(t)
    ops.apply()


class ShardOps(object):
    """The HIP compute of one rank (csrc/skge_shard.hip + skge_accum_apply),
    on buffers allocated once for the fixed capacity C."""

    def __init__(self, runner):
        self.r = runner

    def buf(self, name):
        return self.r.bufs[name]

    def route(self, start, count):
        r = self.r
        b = r.bufs
        L.check(L.lib().skge_shard_route_cap(r.sp, L.ptr(r.rec), L.ptr(r.rec_n1), start, count,
                                             r.G, r.C, L.ptr(b["send_ids"]), L.ptr(b["req_pos"]),
                                             L.ptr(b["route_ws"]), b["route_ws"].numel(),
                                             L.ptr(r.err)), "shard route")
        return b["send_ids"], b["req_pos"]

    def gather(self, ids):
        r = self.r
        rows = r.bufs["rows"]
        L.check(L.lib().skge_shard_gather(r.sp, L.ptr(r.E.data), r.d, r.G, L.ptr(ids),
                                          ids.shape[0], L.ptr(rows)), "shard gather")
        return rows

    def score(self, start, count, fetched, req_pos):
        r = self.r
        C = r.bufs["contrib"]
        L.check(L.lib().skge_shard_score(r.sp, r.tr, r.d, L.ptr(r.rec), L.ptr(r.rec_n1), start,
                                         count, L.ptr(fetched), L.ptr(req_pos), float(r.margin),
                                         L.ptr(C), L.ptr(r.vshards)), "shard score")
        return C

    def accum(self, ids, contrib):
        r = self.r
        L.check(L.lib().skge_shard_accum(r.sp, r.te, r.G, L.ptr(ids), L.ptr(contrib),
                                         ids.shape[0]), "shard accum")

    def rel_sums(self):
        acc = self.r.accR
        return acc.sum.view(torch.int64), acc.cnt   # packed sums add as int64

    def apply(self):
        r = self.r
        L.check(L.lib().skge_accum_apply(r.sp, (L.SkgeTable * 2)(r.te, r.tr), 2,
                                         L.int_array(r.G * r.C, r.R.rows)), "shard apply")


def bucket_capacity(trip_local, n_ent, G, batch, sigmas=8.0):
    """Request slots per owner bucket (the fixed-capacity layout): a batch of
    `batch` of this rank's positives sends 4 requests each (s, o, s', o');
    s and o go to owner (id % G) with this rank's exact frequencies f_g, the
    corruptions uniformly (skge/sample.py:41-46).  mu = batch (2 max_g f_g +
    2 / G), plus `sigmas` standard deviations and 64; never above 4 batch.
    The route kernel flags any bucket that still overflows (checked after
    every epoch)."""
    batch = int(batch)
    if G == 1 or batch == 0:
        return max(4 * batch, 1)
    so = torch.cat([trip_local[:, 0], trip_local[:, 1]]).long() % G
    f = torch.bincount(so, minlength=G).double() / max(int(so.numel()), 1)
    mu = batch * (2.0 * float(f.max().item()) + 2.0 / G)
    return int(min(4 * batch, np.ceil(mu + sigmas * np.sqrt(mu) + 64)))


class ShardedRunner(object):
    """Row-sharded TransE-L1 + AdaGrad pairwise training (margin, strict >,
    RandomModeSampler(1, [0, 1]) negatives drawn on the device against the
    set of ALL ranks' triples).

    E_local: this rank's rows of E (rows rank, rank + G, ...), R: the full
    relation table (identical on every rank), trip_local: this rank's training
    triples [T_r, 3] (s, o, p) int32 on the device.  Every rank runs the same
    number of batches per epoch (the largest rank's; ranks with fewer
    positives take empty batches, which still join the exchanges)."""

    def __init__(self, n_ent, E_local, R, trip_local, nbatches, lr=0.1, margin=2.0, seed=0,
                 ntries=100, group=None, stream=None, capacity=None, capture=None):
        from .param import AdaGrad, Accumulator, Parameter, normalize
        from .device import DeviceKG
        self.ex = Exchange(group)
        self.G, self.rank = self.ex.G, self.ex.rank
        dev = E_local.device
        self.device = dev
        self.stream = stream if stream is not None else torch.cuda.Stream(device=dev)
        self.sp = L.stream_ptr(self.stream)
        self.n_ent, self.d = int(n_ent), int(E_local.shape[1])
        if self.d % 4 or self.d > 1024:
            raise ValueError("sharded TransE-L1 needs d % 4 == 0 and d <= 1024")
        if E_local.shape[0] != owned_rows(self.n_ent, self.G, self.rank):
            raise ValueError("E_local must hold rows rank, rank + G, ... (%d rows)"
                             % owned_rows(self.n_ent, self.G, self.rank))
        self.margin, self.ntries = float(margin), int(ntries)
        self.seed = int(seed) & (2 ** 64 - 1)
        self.E = Parameter(None, name="E", post=normalize, value=E_local)
        self.R = Parameter(None, name="R", value=R)
        self.updE, self.updR = AdaGrad(self.E, lr), AdaGrad(self.R, lr)
        self.updaters = {"E": self.updE, "R": self.updR}
        self.trip = trip_local
        self.T = int(trip_local.shape[0])
        # the sampler rejects against every rank's triples
        self.kg = DeviceKG(self._all_triples(trip_local), dev)
        # np.split geometry of the largest rank (skge/base.py:1246-1268)
        T_max = self._max_over_ranks(self.T)
        bs = max(T_max // nbatches, 1)
        self.batches = [(s0, max(0, min(bs, self.T - s0))) for s0 in range(0, T_max, bs)]
        # fixed-capacity buckets: C request slots per owner (every rank uses the
        # largest rank's C, so the all-to-all slices are equal)
        self.C = self._max_over_ranks(bucket_capacity(trip_local, self.n_ent, self.G, bs)
                                      if capacity is None else int(capacity))
        n_slots = self.G * self.C
        self.accE = Accumulator(self.E.rows, self.d, dev, slots=n_slots, mode=L.SKGE_ACC_I16X4)
        # packed relation sums all-reduced over the ranks' batches: positive j
        # adds into copy j mod reps, enough copies that no 16-bit field of the
        # union batch can wrap (the apply folds them, device.relation_replicas)
        from .device import relation_replicas
        reps = relation_replicas(self.kg, self.R.rows, bs, ranks=self.G)
        if reps == 0:
            raise ValueError("sharded runner: a relation's count in the union batch exceeds "
                             "what 32 packed accumulator copies hold; use more batches")
        self.accR = Accumulator(self.R.rows, self.d, dev, mode=L.SKGE_ACC_I16X4, dense=True,
                                replicas=reps)
        self.te = self.updE.table(self.accE, counters=False)
        self.tr = self.updR.table(self.accR, counters=False)
        self.cstride = int(L.lib().skge_shard_contrib_stride(self.d))
        u8, i32 = torch.uint8, torch.int32
        ws = int(L.lib().skge_shard_route_workspace_bytes(bs, self.G))
        self.bufs = {"send_ids": torch.full((n_slots,), -1, dtype=i32, device=dev),
                     "recv_ids": torch.full((n_slots,), -1, dtype=i32, device=dev),
                     "req_pos": torch.full((4 * bs,), -1, dtype=i32, device=dev),
                     "route_ws": torch.zeros(ws, dtype=u8, device=dev),
                     "rows": torch.zeros((n_slots, self.d), dtype=torch.float32, device=dev),
                     "fetched": torch.zeros((n_slots, self.d), dtype=torch.float32, device=dev),
                     "contrib": torch.zeros((n_slots, self.cstride), dtype=u8, device=dev),
                     "recv_contrib": torch.zeros((n_slots, self.cstride), dtype=u8, device=dev)}
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)   # bucket overflow flag
        self.vshards = torch.zeros(64 * 32, dtype=torch.int32, device=dev)
        self.nviol_total = torch.zeros(1, dtype=torch.int32, device=dev)
        self.epoch_key = torch.zeros(1, dtype=torch.int64, device=dev)
        self.rec = torch.empty((max(self.T, 1), 4), dtype=torch.int32, device=dev)
        self.rec_n1 = torch.empty(max(self.T, 1), dtype=torch.int32, device=dev)
        self.ops = ShardOps(self)
        if capture is None:
            capture = self.ex.backend in (None, "nccl")
        self.capture = bool(capture)
        self.graph = None
        torch.cuda.current_stream(dev).synchronize()

    # ---- helpers ----
    def _max_over_ranks(self, x):
        if self.G == 1:
            return int(x)
        t = torch.tensor([int(x)], dtype=torch.int64, device=self._coll_device())
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.ex.group)
        return int(t.item())

    def _coll_device(self):
        return "cpu" if self.ex.backend == "gloo" else self.device

    def _all_triples(self, trip):
        if self.G == 1:
            return trip
        cd = self._coll_device()
        n = torch.tensor([trip.shape[0]], dtype=torch.int64, device=cd)
        ns = [torch.zeros_like(n) for _ in range(self.G)]
        dist.all_gather(ns, n, group=self.ex.group)
        ns = [int(x.item()) for x in ns]
        m = max(ns)
        pad = torch.full((m, 3), -1, dtype=torch.int32, device=cd)
        pad[:trip.shape[0]] = trip.to(cd)
        parts = [torch.empty_like(pad) for _ in range(self.G)]
        dist.all_gather(parts, pad, group=self.ex.group)
        return torch.cat([p[:k] for p, k in zip(parts, ns)]).to(self.device)

    # ---- training ----
    def sample_epoch(self):
        """The epoch's order and negatives (skge_epoch_sample, keyed by
        epoch_key) for this rank's triples."""
        if self.T:
            L.check(L.lib().skge_epoch_sample(self.sp, L.ptr(self.trip), self.T,
                                              L.ptr(self.kg.slots), self.kg.capacity, self.n_ent,
                                              self.seed, L.ptr(self.epoch_key), self.ntries,
                                              L.ptr(self.rec), L.ptr(self.rec_n1)),
                    "epoch sample")

    def step(self, start, count):
        with torch.cuda.stream(self.stream):
            sharded_step(self.ops, self.ex, start, count)

    def fold_violations(self):
        """Add the violation shards into nviol_total (this rank's pairs)."""
        L.check(L.lib().skge_shard_fold_violations(self.sp, L.ptr(self.vshards),
                                                   L.ptr(self.nviol_total)), "fold")

    def _epoch(self):
        self.sample_epoch()
        for start, count in self.batches:
            sharded_step(self.ops, self.ex, start, count)
        self.fold_violations()
        L.check(L.lib().skge_epoch_advance(self.sp, L.ptr(self.epoch_key)), "advance")

    def run(self, nepochs=1):
        """nepochs epochs.  With capture (the "nccl" backend, or one process)
        the first epoch runs eagerly and is then captured -- kernels and RCCL
        collectives -- into one CUDA graph that later epochs replay: no host
        read or host-side size anywhere in an epoch.  Ordered after the
        caller's stream, and its later work after the epochs."""
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            for _ in range(int(nepochs)):
                if not self.capture:
                    self._epoch()
                elif self.graph is None:
                    self._epoch()
                    self.stream.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=self.stream):
                        self._epoch()
                    self.graph = g
                else:
                    self.graph.replay()
        torch.cuda.current_stream().wait_stream(self.stream)

    def synchronize(self):
        self.stream.synchronize()
        if int(self.err.item()):
            raise L.SkgeError("sharded runner: an owner bucket overflowed its %d request slots "
                              "(skewed rows); pass a larger capacity" % self.C)
        rc = L.lib().skge_device_error(self.sp, 1)
        if rc & 2:
            raise L.SkgeError("sharded runner: a row's per-batch count exceeded 32767 "
                              "(packed sums may have wrapped)")

    def gather_full_E(self):
        """The whole entity table assembled on every rank (tests, checkpoints)."""
        E = self.E.data
        if self.G == 1:
            return E.clone()
        cd = self._coll_device()
        m = owned_rows(self.n_ent, self.G, 0)
        pad = torch.zeros((m, self.d), dtype=torch.float32, device=cd)
        pad[:E.shape[0]] = E.to(cd)
        parts = [torch.empty_like(pad) for _ in range(self.G)]
        dist.all_gather(parts, pad, group=self.ex.group)
        full = torch.empty((self.n_ent, self.d), dtype=torch.float32, device=cd)
        for g, p in enumerate(parts):
            full[g::self.G] = p[:owned_rows(self.n_ent, self.G, g)]
        return full.to(self.device)
