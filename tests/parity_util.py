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
