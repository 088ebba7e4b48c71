"""Parity checks against the fp64 oracle / golden vectors, with headroom.

The bar (BASELINE.json north_star): the fp32 HIP path matches the fp64
reference within 1e-5 on identical batches.  Per element

    tol = ATOL + RTOL * |want|                                  (scores, state, SGD)
    tol = ATOL + RTOL * |want| + lr * grad_rounding / H         (AdaGrad parameters)

where H = max(sqrt(p2), 1e-7) is the AdaGrad divisor: the step lr*g/H turns an
absolute fp32 rounding e of a gradient element into lr*e/H of parameter error,
up to 1e6 * lr * e where the reference's own accumulator is ~0 (see
test_gpu_parity.close_adagrad).  Every check records its HEADROOM = tol /
max|err| over the array (inf when exact; >= 1 passes, >= 2 means the error
uses at most half the budget); conftest.py writes the records of a session to
gpurun_out/parity_headroom.json so the margin to the bar is on record, not
just pass/fail.
"""
import numpy as np
import torch

ATOL = 1e-5
RTOL = 1e-5
GRAD_ROUNDING = 1e-8

RECORDS = []   # (what, headroom, max_abs_err, n_elements)
FLIPS = []     # (what, rows past the plain bar, rows checked, allowed)

# check_step's sign-flip allowance (lr eps / H, up to 2 lr) admits an
# isolated near-zero gradient whose sign the fp32 and fp64 paths decide
# differently.  A real bug that flips signs would do so in many rows, so the
# rows that need the allowance -- any element past the plain ATOL + RTOL
# |want| bar -- may be at most FLIP_ROWS_FRAC of the checked rows (at least
# FLIP_ROWS_MIN).  Measured on the full GPU suite: at most 2.6% (RESCAL's W
# after a runner epoch, every element updated every batch), 1.3% (HolE E);
# a sign error in the path would put about half of the rows past the bar.
FLIP_ROWS_FRAC = 0.05
FLIP_ROWS_MIN = 3


def _np(t):
    return t.detach().cpu().numpy() if torch.is_tensor(t) else np.asarray(t)


def headroom(got, want, tol):
    err = np.abs(np.asarray(got, dtype=np.float64) - np.asarray(want, dtype=np.float64))
    if err.size == 0:
        return float("inf"), 0.0
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.where(err > 0, tol / np.where(err > 0, err, 1.0), np.inf)
    return float(np.min(r)), float(np.max(err))


def check(got, want, what, lr=None, p2=None, grad_rounding=GRAD_ROUNDING, atol=ATOL, rtol=RTOL,
          min_headroom=1.0):
    """Assert |got - want| <= tol elementwise (AdaGrad form when p2 is given)
    and record the headroom; min_headroom > 1 demands more margin."""
    got = _np(got).astype(np.float64)
    want = np.asarray(want, dtype=np.float64)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    tol = atol + rtol * np.abs(want)
    if p2 is not None:
        H = np.maximum(np.sqrt(np.asarray(_np(p2), dtype=np.float64)), 1e-7)
        tol = tol + lr * grad_rounding / H
    h, emax = headroom(got, want, tol)
    RECORDS.append((what, h, emax, int(got.size)))
    if not h >= min_headroom:
        bad = np.abs(got - want) > tol / min_headroom
        raise AssertionError("%s: %d of %d elements past tol/%g, headroom %.3g, max |err| %.3g"
                             % (what, int(bad.sum()), got.size, min_headroom, h, emax))
    return h


ROW_ULPS = 2.0 ** -22   # 4 fp32 ulps (u = 2^-24) of a gradient row's 2-norm


def grad_rounding(shape, grads):
    """Per-element absolute rounding bound of the fp32 gradient: GRAD_ROUNDING
    plus 4 ulps of the element's ROW norm (the oracle's own gradient rows,
    (g, idx)).  A row of d-term dot products (RESCAL's W E_o / E_s W) or of
    FFT correlations (HolE) carries absolute error of a few ulps of the row's
    magnitude, not of the element's -- an element near zero inherits it."""
    eps = np.full(shape, GRAD_ROUNDING)
    if grads is not None:
        g, idx = grads
        g = np.asarray(g, dtype=np.float64).reshape(len(idx), -1)
        rown = np.sqrt((g ** 2).sum(axis=1))
        eps.reshape(shape[0], -1)[np.asarray(idx)] += ROW_ULPS * rown[:, None]
    return eps


def check_step(got, want, before, grads, p2_after, lr, what, post=None, opt="adagrad",
               min_headroom=1.0):
    """Parameters after one updater step (+ projection) from `before`, against
    the oracle's `want`.  Per element

      a   = lr * eps / H              (AdaGrad: the gradient rounding eps,
                                       grad_rounding(), through the divisor
                                       H = max(sqrt(p2), 1e-7); at most 2 lr,
                                       a sign flip of a near-zero gradient)
      tol = ATOL + RTOL |want| + a

    and, for a projected row (post 'normalize' / 'normless1', skge/param.py:
    161-174), the projection's scale moves every element of the row when any
    element moves: + |want| * dss / ss (normless1, ss >= 1) or |want| * dss /
    (2 ss) (normalize), dss = sum over the row of 2 |pre| a + a^2, pre the
    oracle's row before the projection."""
    want = np.asarray(want, dtype=np.float64)
    eps = grad_rounding(want.shape, grads)
    if opt == "adagrad":
        H = np.maximum(np.sqrt(np.asarray(_np(p2_after), dtype=np.float64)), 1e-7)
        a = np.minimum(lr * eps / H, 2.0 * lr)
    else:
        a = lr * eps
    tol = ATOL + RTOL * np.abs(want) + a
    if post is not None and grads is not None:
        g, idx = grads
        idx = np.asarray(idx)
        g = np.asarray(g, dtype=np.float64).reshape(want[idx].shape)
        b = np.asarray(before, dtype=np.float64)[idx]
        if opt == "adagrad":
            step = lr * g / np.maximum(np.sqrt(np.asarray(_np(p2_after), dtype=np.float64)[idx]),
                                       1e-7)
        else:
            step = lr * g
        pre = b - step
        flat = lambda x: x.reshape(len(idx), -1)
        ss = (flat(pre) ** 2).sum(axis=1)
        ar = flat(a[idx])
        dss = (2.0 * np.abs(flat(pre)) * ar + ar ** 2).sum(axis=1)
        if post == "normless1":
            rel = np.where(ss >= 1.0, dss / np.maximum(ss, 1.0), 0.0)
        else:
            rel = dss / (2.0 * np.maximum(ss, 1e-30))
        extra = np.abs(flat(want[idx])) * rel[:, None]
        tol.reshape(want.shape[0], -1)[idx] += extra
    got = _np(got).astype(np.float64)
    h, emax = headroom(got, want, tol)
    RECORDS.append((what, h, emax, int(got.size)))
    if not h >= min_headroom:
        bad = np.abs(got - want) > tol / min_headroom
        raise AssertionError("%s: %d of %d elements past tol/%g, headroom %.3g, max |err| %.3g"
                             % (what, int(bad.sum()), got.size, min_headroom, h, emax))
    # rows along the last axis: E / R rows, or the d rows of each of RESCAL's
    # W_p matrices (an element's flip touches its row; a projection moves it)
    plain = np.abs(got - want) > ATOL + RTOL * np.abs(want)
    flat = plain.reshape(-1, want.shape[-1])
    nflip = int(flat.any(axis=1).sum())
    per = flat.shape[0] // want.shape[0]      # last-axis rows per first-axis index
    nrows = (len(np.unique(np.asarray(grads[1]))) * per if grads is not None
             else flat.shape[0])
    allowed = max(FLIP_ROWS_MIN, int(np.ceil(FLIP_ROWS_FRAC * nrows)))
    FLIPS.append((what, nflip, nrows, allowed))
    if nflip > allowed:
        raise AssertionError("%s: %d of %d rows need the sign-flip allowance (at most %d)"
                             % (what, nflip, nrows, allowed))
    return h


POSTS = {"transe": {"E": "normalize"}, "hole": {"E": "normless1"}, "rescal": {}}
