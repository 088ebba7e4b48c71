"""CPU oracle for the scikit-kge mini-batch training hot path.

TEST INFRASTRUCTURE ONLY.  This module is the checker: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``skge_amd``) never calls into it and fails loudly when
its HIP library is missing.

It restates, in float64 NumPy, the reference's algorithm for every function on
the path (file:line citations are into /root/reference).  Parity is PINNED:
``tests/test_oracle_golden.py`` checks this module against the golden vectors in
``tests/golden/`` that ``tools/gen_golden.py`` produced by importing and
running the reference library layer itself.

Conventions (as in the reference): a triple is (s, o, p)
(skge/base.py:511, skge/util.py:104-110); index arrays here are int arrays of
shape (P, 3) holding columns s, o, p.
"""
import numpy as np

# ----------------------------------------------------------------------------
# activation functions  (skge/actfun.py)
# ----------------------------------------------------------------------------


class Linear:
    """skge/actfun.py:13-24: f(x) = x, g_given_f = ones."""
    name = "linear"

    @staticmethod
    def f(x):
        return x

    @staticmethod
    def g_given_f(fx):
        return np.ones(fx.shape[0])


class Sigmoid:
    """skge/actfun.py:27-35: f = 1/(1+exp(-x)), g_given_f = f(1-f)."""
    name = "sigmoid"

    @staticmethod
    def f(x):
        return 1.0 / (1 + np.exp(-x))

    @staticmethod
    def g_given_f(fx):
        return fx * (1.0 - fx)


class Tanh:
    """skge/actfun.py:38-46."""
    name = "tanh"

    @staticmethod
    def f(x):
        return np.tanh(x)

    @staticmethod
    def g_given_f(fx):
        return 1 - fx ** 2


class ReLU:
    """skge/actfun.py:49-57."""
    name = "relu"

    @staticmethod
    def f(x):
        return np.maximum(0, x)

    @staticmethod
    def g_given_f(fx):
        return (fx > 0).astype(np.int64)


AFUNS = {c.name: c for c in (Linear, Sigmoid, Tanh, ReLU)}

# ----------------------------------------------------------------------------
# numeric utilities  (skge/util.py)
# ----------------------------------------------------------------------------


def ccorr(a, b):
    """Circular correlation along the last axis, skge/util.py:30-50:
    c_k = sum_j a_j b_{(j+k) mod d} = ifft(conj(fft a) * fft b).real"""
    return np.fft.ifft(np.conj(np.fft.fft(a)) * np.fft.fft(b)).real


def cconv(a, b):
    """Circular convolution along the last axis, skge/util.py:8-27:
    c_k = sum_j a_j b_{(k-j) mod d} = ifft(fft a * fft b).real"""
    return np.fft.ifft(np.fft.fft(a) * np.fft.fft(b)).real


def ccorr_direct(a, b):
    """O(d^2) definition of ccorr (used to cross-check the FFT form)."""
    d = a.shape[-1]
    k = np.arange(d)
    return np.stack([np.sum(a * np.roll(b, -kk, axis=-1), axis=-1) for kk in k], axis=-1)


def cconv_direct(a, b):
    d = a.shape[-1]
    out = np.zeros(np.broadcast(a, b).shape)
    for kk in range(d):
        idx = (kk - np.arange(d)) % d
        out[..., kk] = np.sum(a * b[..., idx], axis=-1)
    return out


def segment_mean(idx, rows):
    """grad_sum_matrix + ``Sm.dot(G) / n`` (skge/util.py:53-101 and its callers,
    e.g. skge/transe.py:128-136): the MEAN over occurrences of the contribution
    rows per unique (sorted) index.  Returns (uidx, sums, counts)."""
    idx = np.asarray(idx, dtype=np.int64)
    uidx, inv = np.unique(idx, return_inverse=True)
    sums = np.zeros((len(uidx),) + rows.shape[1:])
    np.add.at(sums, inv, rows)
    n = np.bincount(inv, minlength=len(uidx)).astype(np.float64)
    return uidx, sums, n


def _bcast(n, ndim):
    return n.reshape((-1,) + (1,) * (ndim - 1))


def _split(trip):
    trip = np.asarray(trip, dtype=np.int64)
    return trip[:, 0], trip[:, 2], trip[:, 1]   # ss, ps, os  (skge/util.py:104-110)

# ----------------------------------------------------------------------------
# TransE  (skge/transe.py)
# ----------------------------------------------------------------------------


def transe_scores(E, R, trip, l1=True):
    """skge/transe.py:25-46: -||E[s]+R[p]-E[o]||_1 or -||.||_2^2 (no sqrt)."""
    s, p, o = _split(trip)
    v = E[s] + R[p] - E[o]
    return -np.sum(np.abs(v), axis=1) if l1 else -np.sum(v ** 2, axis=1)


def transe_pairwise_gradients(E, R, pos, neg, margin, l1=True):
    """skge/transe.py:48-165.  Returns (pscore, nscore, nviol, grads|None)."""
    sp, pp, op = _split(pos)
    sn, pn, on = _split(neg)
    ps = transe_scores(E, R, pos, l1)
    ns = transe_scores(E, R, neg, l1)
    ind = np.where(ns + margin > ps)[0]            # strict >  (transe.py:73)
    nviol = len(ind)
    if nviol == 0:
        return ps, ns, 0, None
    sp, sn, pp, pn, op, on = sp[ind], sn[ind], pp[ind], pn[ind], op[ind], on[ind]
    pg = E[op] - R[pp] - E[sp]                      # transe.py:103-104
    ng = E[on] - R[pn] - E[sn]
    if l1:
        pg, ng = np.sign(-pg), np.sign(ng)          # transe.py:115-117
    else:
        pg = -pg                                    # transe.py:120-121
    eidx, es, en = segment_mean(np.concatenate([sp, op, sn, on]),
                                np.vstack([pg, -pg, ng, -ng]))   # transe.py:128-136
    ridx, rs, rn = segment_mean(np.concatenate([pp, pn]), np.vstack([pg, ng]))  # 158-160
    return ps, ns, nviol, {"E": (es / en[:, None], eidx), "R": (rs / rn[:, None], ridx)}

def transe_violation_counts(violations, pos, neg, ind):
    """E.violations bookkeeping of skge/transe.py:78-83: for every violating
    pair i in ind, +1 for each distinct entity of {sn, on, sp, op}."""
    sp, _, op = _split(pos)
    sn, _, on = _split(neg)
    for i in ind:
        for u in set([sn[i], on[i], sp[i], op[i]]):
            violations[u] += 1
    return violations


def adagrad_update_counts(counts, idx):
    """Parameter.updateCounts of skge/param.py:149-150: +1 per row of an
    AdaGrad update's idx."""
    for i in idx:
        counts[i] += 1
    return counts


# ----------------------------------------------------------------------------
# HolE  (skge/hole.py)
# ----------------------------------------------------------------------------


def hole_scores(E, R, trip):
    """skge/hole.py:19-20: sum_k R[p]_k * ccorr(E[s], E[o])_k."""
    s, p, o = _split(trip)
    return np.sum(R[p] * ccorr(E[s], E[o]), axis=1)


def hole_gradients(E, R, trip, ys, rparam=0.0):
    """Logistic loss, skge/hole.py:22-42.  Returns (score, loss, grads)."""
    ss, ps, os_ = _split(trip)
    ys = np.asarray(ys, dtype=np.float64)
    score = hole_scores(E, R, trip)
    ysc = ys * score
    loss = np.sum(np.logaddexp(0, -ysc))
    fs = -(ys * Sigmoid.f(-ysc))[:, None]
    ridx, rsum, rn = segment_mean(ps, fs * ccorr(E[ss], E[os_]))
    gr = rsum / rn[:, None] + rparam * R[ridx]
    eidx, esum, en = segment_mean(np.concatenate([ss, os_]),
                                  np.vstack([fs * ccorr(R[ps], E[os_]), fs * cconv(E[ss], R[ps])]))
    ge = esum / en[:, None] + rparam * E[eidx]
    return score, loss, {"E": (ge, eidx), "R": (gr, ridx)}


def hole_pairwise_gradients(E, R, pos, neg, margin, rparam=0.0, af=Sigmoid):
    """skge/hole.py:44-100.  Returns (pscore_raw, nscore_raw, nviol, grads|None)."""
    sp, pp, op = _split(pos)
    sn, pn, on = _split(neg)
    praw = hole_scores(E, R, pos)
    nraw = hole_scores(E, R, neg)
    pf, nf = af.f(praw), af.f(nraw)
    ind = np.where(nf + margin > pf)[0]
    nviol = len(ind)
    if nviol == 0:
        return praw, nraw, 0, None
    sp, sn, op, on, pp, pn = sp[ind], sn[ind], op[ind], on[ind], pp[ind], pn[ind]
    gp = -af.g_given_f(pf[ind])[:, None]
    gn = af.g_given_f(nf[ind])[:, None]
    ridx, rsum, rn = segment_mean(np.concatenate([pp, pn]),
                                  np.vstack([gp * ccorr(E[sp], E[op]), gn * ccorr(E[sn], E[on])]))
    gr = rsum / rn[:, None] + rparam * R[ridx]                  # hole.py:82-83
    eidx, esum, en = segment_mean(
        np.concatenate([sp, sn, op, on]),
        np.vstack([gp * ccorr(R[pp], E[op]), gn * ccorr(R[pn], E[on]),
                   gp * cconv(E[sp], R[pp]), gn * cconv(E[sn], R[pn])]))
    ge = esum / en[:, None]                                     # no rparam (hole.py:98)
    return praw, nraw, nviol, {"E": (ge, eidx), "R": (gr, ridx)}

# ----------------------------------------------------------------------------
# RESCAL  (skge/rescal.py)
# ----------------------------------------------------------------------------


def rescal_scores(E, W, trip):
    """skge/rescal.py:31-35: E[s] . (W[p] E[o])."""
    s, p, o = _split(trip)
    return np.einsum("nd,nd->n", E[s], np.einsum("nij,nj->ni", W[p], E[o]))


def rescal_gradients(E, W, trip, ys, rparam=0.0):
    """Logistic loss, skge/rescal.py:37-76.  Returns (score, loss, grads)."""
    ss, ps, os_ = _split(trip)
    ys = np.asarray(ys, dtype=np.float64)
    WE = np.einsum("nij,nj->ni", W[ps], E[os_])
    EW = np.einsum("ni,nij->nj", E[ss], W[ps])
    score = np.sum(E[ss] * WE, axis=1)
    ysc = ys * score
    loss = np.sum(np.logaddexp(0, -ysc))
    fs = -(ys * Sigmoid.f(-ysc))[:, None]
    pidx = np.unique(ps)
    gw = np.zeros((len(pidx),) + W.shape[1:])
    for i, p in enumerate(pidx):                                # rescal.py:61-70
        ind = np.where(ps == p)[0]
        gw[i] = np.dot(E[ss[ind]].T, fs[ind] * E[os_[ind]]) / len(ind)
        gw[i] += rparam * W[p]
    eidx, esum, en = segment_mean(np.concatenate([ss, os_]), np.vstack([fs * WE, fs * EW]))
    ge = esum / en[:, None] + rparam * E[eidx]                 # rparam outside the mean
    return score, loss, {"E": (ge, eidx), "W": (gw, pidx)}


def rescal_pairwise_gradients(E, W, pos, neg, margin, rparam=0.0, af=Linear):
    """skge/rescal.py:78-139, quirks kept: the dW divisor is always 2 and dW
    uses ALL pairs; rparam sits inside the entity mean."""
    sp, pp, op = _split(pos)
    sn, pn, on = _split(neg)
    WEp = np.einsum("nij,nj->ni", W[pp], E[op])
    WEn = np.einsum("nij,nj->ni", W[pn], E[on])
    praw = np.sum(E[sp] * WEp, axis=1)
    nraw = np.sum(E[sn] * WEn, axis=1)
    pf, nf = af.f(praw), af.f(nraw)
    ind = np.where(nf + margin > pf)[0]
    nviol = len(ind)
    if nviol == 0:
        return praw, nraw, 0, None
    gp = -np.asarray(af.g_given_f(pf), dtype=np.float64)[:, None]
    gn = np.asarray(af.g_given_f(nf), dtype=np.float64)[:, None]
    pidx = np.unique(np.concatenate([pp, pn]))
    gw = np.zeros((len(pidx),) + W.shape[1:])
    for i, p in enumerate(pidx):                                # rescal.py:113-125
        a = pp == p
        b = pn == p
        gw[i] += np.dot(E[sp[a]].T, gp[a] * E[op[a]])
        gw[i] += np.dot(E[sn[b]].T, gn[b] * E[on[b]])
        gw[i] += rparam * W[p]
        gw[i] /= 2.0
    EWp = np.einsum("ni,nij->nj", E[sp[ind]], W[pp[ind]])
    EWn = np.einsum("ni,nij->nj", E[sn[ind]], W[pn[ind]])
    gpi, gni = gp[ind], gn[ind]
    eidx, esum, en = segment_mean(
        np.concatenate([sp[ind], sn[ind], op[ind], on[ind]]),
        np.vstack([gpi * WEp[ind], gni * WEn[ind], gpi * EWp, gni * EWn]))
    ge = (esum + rparam * E[eidx]) / en[:, None]               # rparam inside
    return praw, nraw, nviol, {"E": (ge, eidx), "W": (gw, pidx)}

# ----------------------------------------------------------------------------
# parameters, updaters and projections  (skge/param.py)
# ----------------------------------------------------------------------------


def init_nunif(shape):
    """skge/param.py:23-51: U(+-sqrt(6)/sqrt(rows+cols)) from numpy's global RNG."""
    bnd = np.sqrt(6) / np.sqrt(shape[0] + shape[1])
    return np.squeeze(np.random.uniform(low=-bnd, high=bnd, size=shape))


def init_unif(shape):
    """skge/param.py:11-19."""
    bnd = 1 / np.sqrt(shape[0])
    return np.squeeze(np.random.uniform(low=-bnd, high=bnd, size=shape))


def init_randn(shape):
    """skge/param.py:53-54."""
    return np.squeeze(np.random.randn(*shape))


def normalize(M, idx=None):
    """skge/param.py:161-167: unit L2 rows (all rows when idx is None)."""
    if idx is None:
        return M / np.sqrt(np.sum(M ** 2, axis=1))[:, None]
    nrm = np.sqrt(np.sum(M[idx, :] ** 2, axis=1))[:, None]
    M[idx, :] = M[idx, :] / nrm
    return M


def normless1(M, idx=None):
    """skge/param.py:170-174: divide by the SQUARED norm when it is >= 1.
    With idx None, ``M[None]`` makes the sum run over rows, i.e. each COLUMN
    is divided by max(column sum of squares, 1) (the HolE init quirk)."""
    if idx is None:
        nrm = np.sum(M ** 2, axis=0)[None, :]
        nrm = np.where(nrm < 1, 1.0, nrm)
        return M / nrm
    nrm = np.sum(M[idx] ** 2, axis=1)[:, None]
    nrm[nrm < 1] = 1
    M[idx] = M[idx] / nrm
    return M


def sgd_update(P, g, idx, lr):
    """skge/param.py:129-130."""
    P[idx] -= lr * g


def adagrad_update(P, A, g, idx, lr):
    """skge/param.py:140-155 (the per-row updateCounts loop is instrumentation)."""
    A[idx] += g * g
    H = np.maximum(np.sqrt(A[idx]), 1e-7)
    P[idx] -= lr * g / H


POSTS = {"transe": {"E": normalize}, "hole": {"E": normless1}, "rescal": {}}


def apply_grads(model, params, state, grads, lr, opt):
    """StochasticTrainer._batch_step (skge/base.py:1306-1316): one updater per
    parameter in insertion order (E first), then the post projection
    (skge/param.py:115-118)."""
    for pid in params:
        g, idx = grads[pid]
        if opt == "sgd":
            sgd_update(params[pid], g, idx, lr)
        else:
            adagrad_update(params[pid], state[pid], g, idx, lr)
        post = POSTS[model].get(pid)
        if post is not None:
            params[pid] = post(params[pid], idx)

# ----------------------------------------------------------------------------
# batch loop  (skge/base.py, skge/sample.py)
# ----------------------------------------------------------------------------


def batch_bounds(n_triples, nbatches):
    """StochasticTrainer._optim batch split (skge/base.py:1246-1268):
    bs = T // nb; np.split(idx, arange(bs, T, bs)) -> nb batches (+1 remainder)."""
    bs = n_triples // nbatches
    cuts = list(range(bs, n_triples, bs))
    starts = [0] + cuts
    ends = cuts + [n_triples]
    return list(zip(starts, ends))


def random_mode_sample(trip, triple_set, sz, modes=(0, 1), n=1, ntries=100, rng=np.random):
    """Sampler.sample + RandomModeSampler._sample (skge/sample.py:17-46):
    per positive, per repetition, per mode, up to ``ntries`` draws of
    randint(sz[mode]) until the corrupted tuple is not a training triple."""
    out = []
    for x in trip:
        for _ in range(n):
            for mode in modes:
                nex = list(int(v) for v in x)
                res = None
                for _t in range(ntries):
                    nex[mode] = int(rng.randint(sz[mode]))
                    if tuple(nex) not in triple_set:
                        res = tuple(nex)
                        break
                if res is not None:
                    out.append((tuple(int(v) for v in x), res))
    return out


def pairwise_step(model, params, state, pos, neg, lr, margin, opt="adagrad", **kw):
    """One PairwiseStochasticTrainer._process_batch (skge/base.py:1394-1427)
    given explicit pairs.  Returns (pscore, nscore, nviol, grads)."""
    if model == "transe":
        ps, ns, nv, g = transe_pairwise_gradients(params["E"], params["R"], pos, neg, margin,
                                                  l1=kw.get("l1", True))
    elif model == "hole":
        ps, ns, nv, g = hole_pairwise_gradients(params["E"], params["R"], pos, neg, margin,
                                                rparam=kw.get("rparam", 0.0),
                                                af=kw.get("af", Sigmoid))
    else:
        ps, ns, nv, g = rescal_pairwise_gradients(params["E"], params["W"], pos, neg, margin,
                                                  rparam=kw.get("rparam", 0.0),
                                                  af=kw.get("af", Linear))
    if g is not None:
        apply_grads(model, params, state, g, lr, opt)
    return ps, ns, nv, g


def logistic_step(model, params, state, trip, ys, lr, opt="adagrad", rparam=0.0):
    """One StochasticTrainer._process_batch (skge/base.py:1293-1304)."""
    if model == "hole":
        sc, loss, g = hole_gradients(params["E"], params["R"], trip, ys, rparam)
    else:
        sc, loss, g = rescal_gradients(params["E"], params["W"], trip, ys, rparam)
    apply_grads(model, params, state, g, lr, opt)
    return sc, loss, g


# ----------------------------------------------------------------------------
# filtered ranking evaluation  (skge/base.py:913-1031, skge/run_transe.py:15-29,
# skge/run_hole.py:12-19)
# ----------------------------------------------------------------------------

def entity_scores(model, E, R, s, o, p, direction):
    """Scores of every entity as the tail (direction 'tail': (s, p, ?)) or the
    head ('head': (?, p, o)), as the reference's evaluators compute them:
    TransEEval  scores_o = -sum|E[s] + R[p] - E|, scores_s = -sum|E + R[p] - E[o]|
                (run_transe.py:24-29; the L1 form whatever the training norm)
    HolEEval    ER = ccorr(R[p], E); scores_o = ER . E[s], scores_s = E . ER[o]
                (run_hole.py:14-19)
    RESCAL      (no reference evaluator) E[s] W[p] E^T / E W[p] E[o]."""
    if model == "transe":
        if direction == "tail":
            return -np.sum(np.abs(E[s] + R[p] - E), axis=1)
        return -np.sum(np.abs(E + R[p] - E[o]), axis=1)
    if model == "hole":
        ER = ccorr(R[p], E)
        return ER.dot(E[s]) if direction == "tail" else E.dot(ER[o])
    W = R[p]
    return E.dot(E[s].dot(W)) if direction == "tail" else E.dot(W.dot(E[o]))


def filtered_ranks(model, E, R, queries, known):
    """FilteredRankingEval.positions for explicit queries (s, o, p): per query
    (tail raw, tail filtered, head raw, head filtered) positions.  A position
    is 1 + #entities scoring strictly higher than the true one -- the
    reference's descending-argsort position whenever no other entity ties the
    true score exactly; the filtered count skips known triples other than the
    query itself (the reference's -inf masking, base.py:970-977, 1011-1017)."""
    known = set(map(tuple, np.asarray(known).tolist()))
    out = np.zeros((len(queries), 4), dtype=np.int64)
    n = E.shape[0]
    for i, (s, o, p) in enumerate(np.asarray(queries).tolist()):
        for col, direction, target in ((0, "tail", o), (2, "head", s)):
            sc = entity_scores(model, E, R, s, o, p, direction)
            higher = sc > sc[target]
            out[i, col] = 1 + int(higher.sum())
            if direction == "tail":
                mask = np.array([(s, j, p) in known and j != o for j in range(n)])
            else:
                mask = np.array([(j, o, p) in known and j != s for j in range(n)])
            out[i, col + 1] = 1 + int((higher & ~mask).sum())
    return out


def compute_scores(pos, hits=10):
    """(MRR, mean position, hits@k in percent) of a position array
    (skge/base.py:1099-1103)."""
    pos = np.asarray(pos, dtype=np.float64)
    return float(np.mean(1.0 / pos)), float(np.mean(pos)), float(np.mean(pos <= hits) * 100)
