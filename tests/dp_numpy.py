"""Test infrastructure: a float64 NumPy stand-in for the rank compute of the
data-parallel TransE-L1 epoch (skge_amd.dp.DPOps), so the protocol
(skge_amd.dp.dp_epoch: per union batch one launch that applies the previous
batch and scores this rank's slice, the all-gather of the slices' records,
the other ranks' positives added; the flush) runs over gloo on CPU.
Arithmetic follows the oracle (oracle/skge_oracle.py:
transe_pairwise_gradients, adagrad_update, normalize; skge/transe.py:48-165,
skge/param.py:140-167).  A record is one row of a float64 array:
[v0 | v1 << 1, gp (d), g0 (d), g1 (d)] (the header s, o, p, s', o' comes from
the common epoch draws, as on the GPU)."""
import numpy as np
import torch


class NumpyDPOps(object):
    def __init__(self, rec, rec_n1, E, R, margin, lr):
        self.rec, self.rec_n1 = rec, rec_n1
        self.E, self.R = E.astype(np.float64).copy(), R.astype(np.float64).copy()
        self.AE, self.AR = np.zeros_like(self.E), np.zeros_like(self.R)
        self.margin, self.lr = margin, lr
        self.d = self.E.shape[1]
        self.nviol = 0
        self.sumE, self.cntE = np.zeros_like(self.E), np.zeros(len(self.E), np.int64)
        self.sumR, self.cntR = np.zeros_like(self.R), np.zeros(len(self.R), np.int64)
        self.snaps = []   # (E, R, AE) after every batch's apply

    def begin(self):
        pass

    def _header(self, j):
        s, o, p, s1 = (int(x) for x in self.rec[j])
        return s, o, p, s1, int(self.rec_n1[j])

    def _add(self, j, fl, gp, g0, g1):
        """One positive's contributions (transe.py:128-160 before the mean)."""
        s, o, p, s1, o1 = self._header(j)
        v0, v1 = fl & 1, (fl >> 1) & 1
        if not (v0 + v1):
            return
        # pair 0 rows (sp,op,sn,on) = (s,o,s',o): (+gp,-gp,+g0,-g0); pair 1 = (s,o,s,o')
        for row, c, vec in ((s, v0 + 2 * v1, v0 * gp + v1 * (gp + g1)),
                            (o, 2 * v0 + v1, -(v0 * (gp + g0) + v1 * gp)),
                            (s1, v0, g0), (o1, v1, -g1)):
            if c:
                self.sumE[row] += vec
                self.cntE[row] += c
        self.sumR[p] += v0 * (gp + g0) + v1 * (gp + g1)
        self.cntR[p] += 2 * (v0 + v1)

    def _apply(self):
        self._adagrad(self.E, self.AE, self.sumE, self.cntE, self.lr, True)
        self._adagrad(self.R, self.AR, self.sumR, self.cntR, self.lr, False)
        self.snaps.append((self.E.copy(), self.R.copy(), self.AE.copy()))

    def batch(self, b, start, count, lo, hi, share, fold):
        if b > 0:
            self._apply()                  # union batch b-1 (complete after its scatter)
        d = self.d
        out = np.zeros((max(share, 1), 1 + 3 * d))
        for w in range(lo, hi):
            j = start + w
            s, o, p, s1, o1 = self._header(j)
            es, eo, r = self.E[s], self.E[o], self.R[p]
            ps = -np.abs(es + r - eo).sum()                       # transe.py:25-46
            gp = np.sign(-(eo - r - es))                          # transe.py:103, 115
            v, g = [0, 0], [np.zeros(d), np.zeros(d)]
            for k, c in enumerate((s1, o1)):
                if c < 0:
                    continue
                f = self.E[c]
                ns = -np.abs((f + r - eo) if k == 0 else (es + r - f)).sum()
                v[k] = int(ns + self.margin > ps)                 # strict >, transe.py:73
                g[k] = np.sign((eo - r - f) if k == 0 else (f - r - es))   # transe.py:104, 117
            self.nviol += v[0] + v[1]
            fl = v[0] | (v[1] << 1)
            row = out[w - lo]
            row[0] = fl
            if v[0] + v[1]:
                row[1:1 + d], row[1 + d:1 + 2 * d], row[1 + 2 * d:] = gp, g[0], g[1]
            self._add(j, fl, gp, g[0], g[1])                      # own slice: added locally
        return torch.from_numpy(out[:share] if share else out[:0])

    def gathered(self, ex, send, share):
        out = torch.empty((ex.G * share,) + tuple(send.shape[1:]), dtype=send.dtype)
        return ex.all_gather(out, send)

    def scatter(self, b, start, count, recs, lo, hi):
        R = recs.numpy()
        d = self.d
        for w in range(count):
            if lo <= w < hi:
                continue
            fl = int(R[w, 0])
            self._add(start + w, fl, R[w, 1:1 + d], R[w, 1 + d:1 + 2 * d], R[w, 1 + 2 * d:])

    def flush(self, nb):
        self._apply()

    def end(self):
        pass

    @staticmethod
    def _adagrad(P, A, S, cnt, lr, post):
        rows = np.nonzero(cnt)[0]
        g = S[rows] / cnt[rows, None]                             # Sm.dot(G) / n
        A[rows] += g * g                                          # param.py:147
        P[rows] -= lr * g / np.maximum(np.sqrt(A[rows]), 1e-7)    # param.py:152-155
        if post:
            P[rows] /= np.sqrt((P[rows] ** 2).sum(axis=1))[:, None]   # param.py:161-167
        S[rows] = 0.0
        cnt[rows] = 0
