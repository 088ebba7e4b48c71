"""Device-resident training data and the native epoch runners.

DeviceKG holds the training triples on the GPU ([T, 3] int32, (s, o, p)) and
the open-addressing triple set the device sampler rejects against.
EpochRunner wraps the TransE runners (skge_pipe_runner_* / skge_runner_*,
csrc/skge_pipeline.hip, skge_epoch.hip) and PairLoopRunner the any-model pair
loop (skge_pair_runner_*, csrc/skge_pairloop.hip): one epoch of
PairwiseStochasticTrainer batches (nbatches full batches + the remainder,
skge/base.py:1246-1268), captured once into a hipGraph and replayed."""
import timeit

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


class EpochRunner(object):
    """Native hipGraph epoch of the TransE device batch loop.

    pipelined: None (auto) uses the one-launch-per-batch pipelined runner
    (skge_pipe_runner_*) whenever it applies (TransE-L1, packed accumulators,
    single-copy relation accumulator) and the two-launch runner otherwise;
    True demands it, False forces the two-launch runner.  Both give identical
    parameters.
    """

    def __init__(self, model, updaters, kg, nbatches, seed=0, ntries=100, stream=None,
                 nviol_total=None, force_f32=False, replicas=1, pipelined=None):
        from .transe import TransE
        if not isinstance(model, TransE):
            raise NotImplementedError("device_loop supports TransE (the north-star path) only")
        dev = model.device
        self.stream = stream if stream is not None else torch.cuda.Stream(device=dev)
        self.kg = kg
        self.model = model
        self.epoch_key = torch.zeros(1, dtype=torch.int64, device=dev)
        self.nviol_total = nviol_total if nviol_total is not None else \
            torch.zeros(1, dtype=torch.int32, device=dev)
        bs = kg.T // nbatches
        # TransE-L1 sign contributions are small integers: exact packed int16x4
        # sums at any batch size (the applies flag a row whose count could have
        # wrapped a 16-bit field, checked by synchronize())
        can_pack = bool(model.l1) and model.d % 4 == 0 and not force_f32
        can_pipe = can_pack and replicas <= 1 and pipelined is not False
        self._auto = pipelined is None
        packed = can_pack
        mode = L.SKGE_ACC_I16X4 if packed else L.SKGE_ACC_F32
        from .param import Accumulator
        E, R = model.params["E"], model.params["R"]
        self.accE = Accumulator(E.rows, E.width, dev, slots=4 * bs, mode=mode)
        # relation rows are hot (every positive adds to one of |R| rows):
        # `replicas` > 1 spreads the adds over accumulator copies (dense apply sums them)
        self.accR = Accumulator(R.rows, R.width, dev, mode=mode, dense=True,
                                replicas=replicas)
        self.packed = packed
        if can_pipe and pipelined is None:
            # the pipelined runner's scratch: a second entity accumulator copy,
            # per-row marks and the epoch's records (auto mode: only if it fits)
            torch.cuda.synchronize(dev)
            torch.cuda.empty_cache()
            extra = E.rows * E.width * 2 + E.rows * 12 + kg.T * 20 + (64 << 20)
            can_pipe = extra < torch.cuda.mem_get_info(dev)[0] * 0.9
        self.te = updaters["E"].table(self.accE, counters=False)
        self.tr = updaters["R"].table(self.accR, counters=False)
        self.nbatches = nbatches
        torch.cuda.current_stream().synchronize()
        lib = L.lib()
        if pipelined and not can_pipe:
            raise ValueError("pipelined runner needs TransE-L1, d % 4 == 0, "
                             "no forced f32 and replicas == 1")
        self.pipelined = can_pipe if pipelined is None else bool(pipelined)
        if self.pipelined:
            h = lib.skge_pipe_runner_create(
                L.stream_ptr(self.stream), self.te, self.tr, model.d, L.ptr(kg.trip), kg.T,
                L.ptr(kg.slots), kg.capacity, int(nbatches), int(seed) & (2 ** 64 - 1),
                L.ptr(self.epoch_key), float(model.margin), int(ntries), L.ptr(self.nviol_total))
            if h:
                self.handle = h
                self.nlaunches = lib.skge_pipe_runner_nlaunches(h)
                return
            err = lib.skge_last_error().decode()
            if not (self._auto and "allocation" in err):
                raise L.SkgeError("skge_pipe_runner_create: %s" % err)
            self.pipelined = False   # auto mode: out of device memory -> two-launch runner
        h = lib.skge_runner_create(L.stream_ptr(self.stream), int(bool(model.l1)),
                                   self.te, self.tr,
                                   model.d, L.ptr(kg.trip), kg.T, L.ptr(kg.slots), kg.capacity,
                                   int(nbatches), int(seed) & (2 ** 64 - 1), L.ptr(self.epoch_key),
                                   float(model.margin), int(ntries), None, L.ptr(self.nviol_total))
        if not h:
            raise L.SkgeError("skge_runner_create: %s" % lib.skge_last_error().decode())
        self.handle = h
        self.nlaunches = lib.skge_runner_nlaunches(h)

    def run(self, nepochs=1):
        lib = L.lib()
        fn = lib.skge_pipe_runner_run if self.pipelined else lib.skge_runner_run
        L.check(fn(self.handle, L.stream_ptr(self.stream), int(nepochs)), "runner run")

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
        L.check(L.lib().skge_pipe_runner_profile(
            self.handle, L.stream_ptr(self.stream), us.ctypes.data, stats.ctypes.data, n,
            int(trace_launch or 0), None if tr is None else tr.ctypes.data,
            0 if tr is None else len(tr)), "runner profile")
        if trace_launch:
            return us, stats, tr
        return us, stats

    def synchronize(self):
        self.stream.synchronize()
        if not self.pipelined and self.packed:
            rc = L.lib().skge_device_error(L.stream_ptr(self.stream), 1)
            if rc & 2:
                raise L.SkgeError("epoch runner: a row's per-batch count exceeded 32767 "
                                  "(packed sums may have wrapped); use force_f32=True")
        if self.pipelined:
            rc = L.lib().skge_pipe_runner_error(self.handle, L.stream_ptr(self.stream))
            if rc < 0:
                raise L.SkgeError("pipelined runner: %s" % L.lib().skge_last_error().decode())
            if rc & 1:
                raise L.SkgeError("pipelined runner: a cross-workgroup wait timed out")
            if rc & 2:
                raise L.SkgeError("pipelined runner: a row's per-batch count exceeded 32767 "
                                  "(packed sums may have wrapped); use force_f32=True")

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
        L.check(L.lib().skge_pair_runner_run(self.handle, L.stream_ptr(self.stream),
                                             int(nepochs)), "pair runner run")

    def synchronize(self):
        self.stream.synchronize()

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
    HolE / RESCAL -> PairLoopRunner), 'epoch' or 'pairs'."""
    from .transe import TransE
    if runner == "auto":
        runner = "epoch" if isinstance(model, TransE) else "pairs"
    if runner == "epoch":
        return EpochRunner(model, updaters, kg, nbatches, seed=seed, ntries=ntries,
                           nviol_total=nviol_total)
    if runner == "pairs":
        return PairLoopRunner(model, updaters, kg, nbatches, seed=seed, ntries=ntries,
                              nviol_total=nviol_total)
    raise ValueError("unknown device runner %r" % (runner,))


def device_optim(trainer, xs):
    """PairwiseStochasticTrainer.fit with device_loop=True."""
    model = trainer.model
    dev = model.device
    if trainer._nviol_dev is None:
        trainer._nviol_dev = torch.zeros(1, dtype=torch.int32, device=dev)
    kg = DeviceKG(xs, dev)
    runner = make_runner(model, trainer._updaters, kg, trainer.nbatches, seed=trainer.seed,
                         ntries=trainer.ntries, nviol_total=trainer._nviol_dev,
                         runner=trainer.device_runner)
    trainer._runner = runner
    with torch.cuda.stream(runner.stream):
        for trainer.epoch in range(1, trainer.max_epochs + 1):
            trainer._pre_epoch()
            trainer.epoch_start = timeit.default_timer()
            runner.run(1)
            for f in trainer.post_epoch:
                if not f(trainer):
                    break
    runner.synchronize()
