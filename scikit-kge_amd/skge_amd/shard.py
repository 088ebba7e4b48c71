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

    route     requests (s, o, s', o') of the rank's positives, by owner  [HIP]
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
    memory).  G == 1 needs no process group: every exchange is the identity."""

    def __init__(self, group=None):
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.G = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
            self.backend = dist.get_backend(group)
        else:
            self.G, self.rank, self.backend = 1, 0, None

    def split_sizes(self, send_counts):
        """Bucket sizes this rank sends (device int64 [G]) -> (send list,
        receive list): one tiny all-to-all and ONE host copy per step."""
        if self.G == 1:
            c = send_counts.cpu().tolist()
            return c, c
        recv = torch.empty_like(send_counts)
        self._a2a(recv, send_counts, None, None)
        both = torch.stack([send_counts, recv]).cpu()
        return both[0].tolist(), both[1].tolist()

    def all_to_all(self, inp, send, recv):
        """Rows inp[sum(send[:g]) : ...] go to rank g; returns the rows
        received, grouped by source rank."""
        if self.G == 1:
            return inp[:send[0]]
        out = torch.empty((int(sum(recv)),) + tuple(inp.shape[1:]), dtype=inp.dtype,
                          device=inp.device)
        self._a2a(out, inp[:int(sum(send))], recv, send)
        return out

    def all_reduce_(self, t):
        if self.G > 1:
            if self.backend == "gloo" and t.is_cuda:
                h = t.cpu()
                dist.all_reduce(h, group=self.group)
                t.copy_(h)
            else:
                dist.all_reduce(t, group=self.group)
        return t

    def _a2a(self, out, inp, out_splits, in_splits):
        if self.backend == "gloo" and inp.is_cuda:
            h = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(h, inp.cpu(), out_splits, in_splits, group=self.group)
            out.copy_(h)
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)


def sharded_step(ops, ex, start, count):
    """One mini-batch of the sharded job (positives start .. start+count of
    this rank's epoch order); see the module docstring.  `ops` is the
    rank's compute, `ex` the collectives."""
    send_ids, req_pos, send_counts = ops.route(start, count, ex.G)
    send, recv = ex.split_sizes(send_counts)
    recv_ids = ex.all_to_all(send_ids, send, recv)       # owner side: who wants which row
    rows = ops.gather(recv_ids)
    fetched = ex.all_to_all(rows, recv, send)            # requester side, send order
    contrib = ops.score(start, count, fetched, req_pos)  # + this rank's R sums
    recv_contrib = ex.all_to_all(contrib, send, recv)    # sparse reduce-scatter
    ops.accum(recv_ids, recv_contrib)
    for t in ops.rel_sums():
        ex.all_reduce_(t)
    ops.apply(int(sum(recv)))


class ShardOps(object):
    """The HIP compute of one rank (csrc/skge_shard.hip + skge_accum_apply)."""

    def __init__(self, runner):
        self.r = runner

    def route(self, start, count, G):
        r = self.r
        n = 4 * count
        r._grow("send_ids", n, torch.int32)
        r._grow("req_pos", n, torch.int32)
        ws_bytes = int(L.lib().skge_shard_route_workspace_bytes(count, G))
        ws = r._grow("route_ws", ws_bytes, torch.uint8)
        L.check(L.lib().skge_shard_route(r.sp, L.ptr(r.rec), L.ptr(r.rec_n1), start, count, G,
                                         L.ptr(r.bufs["send_ids"]), L.ptr(r.bufs["req_pos"]),
                                         L.ptr(r.send_counts), L.ptr(ws), ws_bytes), "shard route")
        return r.bufs["send_ids"], r.bufs["req_pos"], r.send_counts

    def gather(self, ids):
        r = self.r
        n = ids.shape[0]
        rows = r._grow("rows", n * r.d, torch.float32)[:n * r.d].view(n, r.d)
        L.check(L.lib().skge_shard_gather(r.sp, L.ptr(r.E.data), r.d, r.G, L.ptr(ids), n,
                                          L.ptr(rows)), "shard gather")
        return rows

    def score(self, start, count, fetched, req_pos):
        r = self.r
        n = fetched.shape[0]
        cs = r.cstride
        C = r._grow("contrib", n * cs, torch.uint8)[:n * cs].view(n, cs)
        L.check(L.lib().skge_shard_score(r.sp, r.tr, r.d, L.ptr(r.rec), L.ptr(r.rec_n1), start,
                                         count, L.ptr(fetched), L.ptr(req_pos), float(r.margin),
                                         L.ptr(C), L.ptr(r.vshards)), "shard score")
        return C

    def accum(self, ids, contrib):
        r = self.r
        n = ids.shape[0]
        r.accE.ensure_slots(n)
        r.te = r.updE.table(r.accE, counters=False)
        L.check(L.lib().skge_shard_accum(r.sp, r.te, r.G, L.ptr(ids), L.ptr(contrib), n),
                "shard accum")

    def rel_sums(self):
        acc = self.r.accR
        return acc.sum.view(torch.int64), acc.cnt   # packed sums add as int64

    def apply(self, n_recv):
        r = self.r
        L.check(L.lib().skge_accum_apply(r.sp, (L.SkgeTable * 2)(r.te, r.tr), 2,
                                         L.int_array(n_recv, r.R.rows)), "shard apply")


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
                 ntries=100, group=None, stream=None):
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
        self.accE = Accumulator(self.E.rows, self.d, dev, slots=4 * bs * self.G,
                                mode=L.SKGE_ACC_I16X4)
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
        self.bufs = {}
        self.send_counts = torch.zeros(self.G, dtype=torch.int64, device=dev)
        self.vshards = torch.zeros(64 * 32, dtype=torch.int32, device=dev)
        self.nviol_total = torch.zeros(1, dtype=torch.int32, device=dev)
        self.epoch_key = torch.zeros(1, dtype=torch.int64, device=dev)
        self.rec = torch.empty((max(self.T, 1), 4), dtype=torch.int32, device=dev)
        self.rec_n1 = torch.empty(max(self.T, 1), dtype=torch.int32, device=dev)
        self.ops = ShardOps(self)
        torch.cuda.current_stream(dev).synchronize()

    # ---- helpers ----
    def _grow(self, name, n, dtype):
        b = self.bufs.get(name)
        if b is None or b.numel() < n:
            b = torch.empty(max(int(n * 1.25), 16), dtype=dtype, device=self.device)
            self.bufs[name] = b
        return b

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

    def run(self, nepochs=1):
        with torch.cuda.stream(self.stream):
            for _ in range(nepochs):
                self.sample_epoch()
                for start, count in self.batches:
                    sharded_step(self.ops, self.ex, start, count)
                self.fold_violations()
                L.check(L.lib().skge_epoch_advance(self.sp, L.ptr(self.epoch_key)), "advance")

    def synchronize(self):
        self.stream.synchronize()
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
