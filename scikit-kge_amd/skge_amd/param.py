"""Parameters, initialisers, updaters and projections (mirrors skge/param.py).

Parameters live on the GPU as fp32 torch tensors; the updaters and the
projections run as HIP kernels (skge_update_rows / skge_accum_apply).
Initialisation draws from numpy's global RNG exactly like the reference
(skge/param.py:11-54, 57-86), in float64, applies the post projection, then
rounds to fp32 -- so `np.random.seed(42); TransE(...)` gives the reference's
initial embeddings rounded to fp32.
"""
import sys

import numpy as np
import torch

from . import _lib as L


def _device():
    L.require_gpu()
    return torch.device("cuda", torch.cuda.current_device())


# --------------------------------------------------------------------------
# initialisers (host, float64, numpy global RNG) -- skge/param.py:11-54
# --------------------------------------------------------------------------

def init_unif(sz):
    """Uniform U(+-1/sqrt(rows))  (skge/param.py:11-19)."""
    bnd = 1 / np.sqrt(sz[0])
    return np.squeeze(np.random.uniform(low=-bnd, high=bnd, size=sz))


def init_nunif(sz):
    """Normalised uniform U(+-sqrt(6)/sqrt(rows+cols))  (skge/param.py:23-51)."""
    bnd = np.sqrt(6) / np.sqrt(sz[0] + sz[1])
    p = np.random.uniform(low=-bnd, high=bnd, size=sz)
    init_nunif.counter += 1
    return np.squeeze(p)


init_nunif.counter = 0


def init_randn(sz):
    """Standard normal (skge/param.py:53-54)."""
    return np.squeeze(np.random.randn(*sz))


def _init_array(shape, method):
    mod = sys.modules[__name__]
    fn = getattr(mod, "init_%s" % method, None)
    if fn is None:
        raise ValueError("Unknown initialization (%s)" % method)   # param.py:100-101
    if len(shape) != 2:
        raise ValueError("Shape must be of size 2")                 # param.py:102-103
    return fn(shape)


# --------------------------------------------------------------------------
# projections  (skge/param.py:161-174)
# --------------------------------------------------------------------------

def normalize(M, idx=None):
    """Unit-L2 rows.  On a host array (model init) all rows when idx is None;
    on a device Parameter the rows idx are projected by the HIP kernel."""
    if isinstance(M, Parameter):
        return _project_device(M, idx, L.SKGE_POST_NORMALIZE)
    if idx is None:
        return M / np.sqrt(np.sum(M ** 2, axis=1))[:, np.newaxis]
    nrm = np.sqrt(np.sum(M[idx, :] ** 2, axis=1))[:, np.newaxis]
    M[idx, :] = M[idx, :] / nrm
    return M


def normless1(M, idx=None):
    """Divide by the SQUARED norm when it is >= 1.  idx None reproduces the
    reference's column-wise quirk (``M[None]`` sums over rows, skge/hole.py:16)."""
    if isinstance(M, Parameter):
        return _project_device(M, idx, L.SKGE_POST_NORMLESS1)
    if idx is None:
        nrm = np.sum(M ** 2, axis=0)[np.newaxis, :]
        nrm = np.where(nrm < 1, 1.0, nrm)
        return M / nrm
    nrm = np.sum(M[idx] ** 2, axis=1)[:, np.newaxis]
    nrm[nrm < 1] = 1
    M[idx] = M[idx] / nrm
    return M


POST_CODES = {None: L.SKGE_POST_NONE, normalize: L.SKGE_POST_NORMALIZE,
              normless1: L.SKGE_POST_NORMLESS1}


def post_code(post):
    try:
        return POST_CODES[post]
    except KeyError:
        raise ValueError("unsupported post projection %r (device path supports "
                         "normalize / normless1)" % (post,))


def _device_init(shape, method, dev):
    """init_nunif / init_unif / init_randn (skge/param.py:23-54) drawn on the
    device, fp32, in place."""
    t = torch.empty(shape, dtype=torch.float32, device=dev)
    rows, cols = shape[-2], shape[-1]
    if method == "nunif":
        bnd = float(np.sqrt(6) / np.sqrt(rows + cols))
        t.uniform_(-bnd, bnd)
    elif method == "unif":
        bnd = float(np.sqrt(1.0 / rows))
        t.uniform_(-bnd, bnd)
    elif method == "randn":
        t.normal_()
    else:
        raise ValueError("Unknown initialization (device_%s)" % method)
    return t


def _device_post_init(t, post, chunk=1 << 20):
    """The model-construction projection (idx=None) on a device table, in
    row chunks so no full-size temporary is made."""
    if post is normalize:
        for r0 in range(0, t.shape[0], chunk):
            blk = t[r0:r0 + chunk]
            blk.div_(blk.norm(dim=1, keepdim=True))
    elif post is normless1:   # the column-wise quirk of normless1(M, None)
        col = torch.zeros(t.shape[1], dtype=torch.float64, device=t.device)
        for r0 in range(0, t.shape[0], chunk):
            col += (t[r0:r0 + chunk].double() ** 2).sum(dim=0)
        col = torch.where(col < 1, torch.ones_like(col), col).float()
        for r0 in range(0, t.shape[0], chunk):
            t[r0:r0 + chunk].div_(col)
    else:
        raise ValueError("unsupported post projection %r" % (post,))


# --------------------------------------------------------------------------
# Parameter
# --------------------------------------------------------------------------

class Parameter(object):
    """A model parameter table on the GPU (mirrors skge/param.py:57-105).

    ``.data`` is the fp32 torch tensor ([rows, d] or [M, d, d]); ``.name``,
    ``.post`` as in the reference.  ``np.asarray(param)`` copies to the host.
    The reference's per-row counters (param.py:84-86) are device int32 arrays,
    read as host copies: ``updateCounts`` (AdaGrad applies, param.py:149-150)
    and ``violations`` (TransE violating pairs, transe.py:78-83) are counted
    by the kernels of the per-batch paths (not by the device-loop runners);
    ``neighbours`` (entity degree) is filled by PairwiseStochasticTrainer.fit.
    """

    def __init__(self, shape, method="nunif", name=None, post=None, value=None, device=None):
        self.name = name
        self.post = post
        self._counters = {}
        self.neighbours = None
        dev = device if device is not None else _device()
        if value is None and method.startswith("device_"):
            # tables too large for a host NumPy draw (e.g. 50M x 512): the same
            # distribution drawn on the device with torch's generator -- not the
            # reference's RNG stream
            self.data = _device_init(tuple(shape), method[len("device_"):], dev)
            if post is not None:
                _device_post_init(self.data, post)
            return
        if value is None:
            shape = tuple(shape)
            if len(shape) == 3:   # param.py:62-64: each d x d slice drawn independently
                arr = np.array([_init_array((shape[1], shape[2]), method) for _ in range(shape[0])])
            else:
                arr = _init_array(shape, method)
            if post is not None:
                arr = post(arr)
            value = arr
        if isinstance(value, Parameter):
            value = value.data
        self.data = torch.as_tensor(np.asarray(value) if not torch.is_tensor(value) else value,
                                    dtype=torch.float32, device=dev).contiguous()

    def counter(self, name):
        """Device int32 [rows] counter `name` ('upd' or 'viol'), allocated zeroed
        on first use."""
        c = self._counters.get(name)
        if c is None:
            c = torch.zeros(self.rows, dtype=torch.int32, device=self.data.device)
            self._counters[name] = c
        return c

    def _counts(self, name):
        c = self._counters.get(name)
        if c is None:
            return np.zeros(self.rows, dtype=np.int64)
        return c.cpu().numpy().astype(np.int64)

    @property
    def updateCounts(self):
        return self._counts("upd")

    @property
    def violations(self):
        return self._counts("viol")

    # array-ish conveniences
    @property
    def shape(self):
        return tuple(self.data.shape)

    @property
    def rows(self):
        return self.data.shape[0]

    @property
    def width(self):
        return int(np.prod(self.data.shape[1:]))

    def __len__(self):
        return self.data.shape[0]

    def __getitem__(self, idx):
        return self.data[idx]

    def __setitem__(self, idx, v):
        self.data[idx] = torch.as_tensor(v, dtype=torch.float32, device=self.data.device)

    def numpy(self):
        return self.data.detach().cpu().numpy()

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a.astype(dtype) if dtype is not None else a

    def __repr__(self):
        return "Parameter(name=%r, shape=%r)" % (self.name, self.shape)


def as_index(idx, device):
    if torch.is_tensor(idx):
        return idx.to(device=device, dtype=torch.int32).contiguous()
    return torch.as_tensor(np.asarray(idx, dtype=np.int64), dtype=torch.int32, device=device)


def as_rows(g, device):
    if torch.is_tensor(g):
        return g.to(device=device, dtype=torch.float32).contiguous()
    return torch.as_tensor(np.asarray(g), dtype=torch.float32, device=device).contiguous()


def table_struct(param, state=None, acc=None, opt=L.SKGE_SGD, post=L.SKGE_POST_NONE, lr=0.0,
                 rin=0.0, rout=0.0, fixed_div=0.0, gate=None, upd_count=None, violations=None):
    t = L.SkgeTable()
    t.param = L.ptr(param.data)
    t.state = L.ptr(state)
    if acc is not None:
        t.acc_sum, t.acc_cnt = L.ptr(acc.sum), L.ptr(acc.cnt)
        t.acc_touched = L.ptr(acc.touched)          # None -> dense table
        t.touched_cap = acc.touched.numel() if acc.touched is not None else 0
        t.acc_mode = acc.mode
        t.acc_replicas = acc.replicas
    t.rows = param.rows
    t.width = param.width
    t.opt, t.post, t.lr = opt, post, lr
    t.rin, t.rout, t.fixed_div = rin, rout, fixed_div
    t.gate = L.ptr(gate)
    t.upd_count = L.ptr(upd_count)
    t.violations = L.ptr(violations)
    return t


def _project_device(M, idx, code):
    dev = M.data.device
    if idx is None:
        idx = torch.arange(M.rows, device=dev)
    ii = as_index(idx, dev)
    g = torch.zeros((ii.numel(), M.width), dtype=torch.float32, device=dev)
    t = table_struct(M, opt=L.SKGE_SGD, post=code, lr=0.0)
    L.check(L.lib().skge_update_rows(L.stream_ptr(), t, L.ptr(g), L.ptr(ii), ii.numel()),
            "projection")
    return M


class Accumulator(object):
    """Device segment-sum accumulator of one table (see skge_table_t): dense
    fp32 sums, occurrence counts and the fixed-slot touched records."""

    def __init__(self, rows, width, device, slots=1024, mode=L.SKGE_ACC_F32, dense=False,
                 replicas=1):
        self.rows, self.width, self.mode = rows, width, mode
        self.replicas = replicas if dense else 1
        # int16x4 mode packs four elements per 8 bytes: width / 2 dwords per row;
        # the deterministic fixed-point mode keeps one int64 per element
        dw = width // 2 if mode == L.SKGE_ACC_I16X4 else \
            (2 * width if mode == L.SKGE_ACC_FX64 else
             (width // 4 if mode == L.SKGE_ACC_I8X4 else width))
        self.sum = torch.zeros(self.replicas * rows * dw, dtype=torch.float32, device=device)
        self.cnt = torch.zeros(self.replicas * rows, dtype=torch.int32, device=device)
        self.touched = None if dense else \
            torch.full((max(slots, 1),), -1, dtype=torch.int32, device=device)

    def ensure_slots(self, n):
        """Grow the touched-slot array to hold n slots (before building tables)."""
        if self.touched is not None and n > self.touched.numel():
            self.touched = torch.full((max(n, 2 * self.touched.numel()),), -1, dtype=torch.int32,
                                      device=self.sum.device)
        return self


# --------------------------------------------------------------------------
# updaters  (skge/param.py:108-158)
# --------------------------------------------------------------------------

class ParameterUpdate(object):
    """``updater(gradient, idx)`` updates ``param`` in place, then applies
    ``param.post`` to the rows idx -- one fused HIP kernel."""
    opt = None

    def __init__(self, param, learning_rate):
        self.param = param
        self.learning_rate = learning_rate

    def state(self):
        return None

    def table(self, acc=None, counters=True, **kw):
        """skge_table_t of this updater; counters=True lets the apply kernels
        count AdaGrad row updates into param.updateCounts."""
        if counters and self.opt == L.SKGE_ADAGRAD:
            kw.setdefault("upd_count", self.param.counter("upd"))
        return table_struct(self.param, self.state(), acc, opt=self.opt,
                            post=post_code(self.param.post), lr=float(self.learning_rate), **kw)

    def __call__(self, gradient, idx=None):
        dev = self.param.data.device
        if idx is None:
            idx = torch.arange(self.param.rows, device=dev)
        ii = as_index(idx, dev)
        g = as_rows(gradient, dev).reshape(ii.numel(), self.param.width)
        L.check(L.lib().skge_update_rows(L.stream_ptr(), self.table(), L.ptr(g), L.ptr(ii),
                                         ii.numel()), type(self).__name__)

    def reset(self):
        pass


class SGD(ParameterUpdate):
    """param[idx] -= lr * g   (skge/param.py:124-130)."""
    opt = L.SKGE_SGD


class AdaGrad(ParameterUpdate):
    """p2[idx] += g^2; param[idx] -= lr * g / max(sqrt(p2[idx]), 1e-7)
    (skge/param.py:134-158)."""
    opt = L.SKGE_ADAGRAD

    def __init__(self, param, learning_rate):
        super(AdaGrad, self).__init__(param, learning_rate)
        self.p2 = torch.zeros_like(param.data)

    def state(self):
        return self.p2

    def reset(self):
        self.p2.zero_()
