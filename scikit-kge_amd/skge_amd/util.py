"""Host-side helpers (mirrors the non-kernel parts of skge/util.py)."""
import numpy as np
import torch


def unzip_triples(xys, with_ys=False):
    """skge/util.py:104-110: list of ((s, o, p), y) -> ss, ps, os[, ys]."""
    xs, ys = list(zip(*xys))
    ss, os, ps = list(zip(*xs))
    if with_ys:
        return np.array(ss), np.array(ps), np.array(os), np.array(ys)
    return np.array(ss), np.array(ps), np.array(os)


def triples_array(xs):
    """Pairs/triples in any accepted form -> int32 numpy [n, 3] (s, o, p).

    Accepts the reference's list of ((s, o, p), y) tuples, a list of
    (s, o, p) tuples, or an int array [n, 3]."""
    if torch.is_tensor(xs):
        return xs
    if isinstance(xs, np.ndarray):
        a = xs
    else:
        xs = list(xs)
        if len(xs) == 0:
            return np.zeros((0, 3), dtype=np.int32)
        first = xs[0]
        if len(first) == 2 and not np.isscalar(first[0]):
            a = np.array([x for x, _ in xs], dtype=np.int64)
        else:
            a = np.array(xs, dtype=np.int64)
    a = np.asarray(a).reshape(-1, 3)
    return a.astype(np.int32)


def labels_array(xys):
    return np.array([y for _, y in xys], dtype=np.float32)


def to_device_triples(xs, device):
    a = triples_array(xs)
    if torch.is_tensor(a):
        return a.to(device=device, dtype=torch.int32).reshape(-1, 3).contiguous()
    return torch.as_tensor(a, device=device)
