"""Test infrastructure: a float64 NumPy stand-in for the rank compute of the
sharded TransE-L1 step (skge_amd.shard.ShardOps), so the exchange protocol
(skge_amd.shard.sharded_step) can run over gloo on CPU, and the HIP kernels'
routing can be checked against it.  Arithmetic follows the oracle
(oracle/skge_oracle.py: transe_pairwise_gradients, adagrad_update, normalize;
skge/transe.py:48-165, skge/param.py:140-167)."""
import numpy as np
import torch


def route(rec, rec_n1, start, count, G):
    """The owner-major request layout of skge_shard_route: request 4j+k
    (k: s, o, s', o'), bucket = id % G, request order inside a bucket."""
    req = np.stack([rec[start:start + count, 0], rec[start:start + count, 1],
                    rec[start:start + count, 3], rec_n1[start:start + count]], axis=1).reshape(-1)
    req_pos = np.full(req.shape, -1, dtype=np.int64)
    send_ids, counts, off = [], [], 0
    for g in range(G):
        sel = np.nonzero((req >= 0) & (req % G == g))[0]
        req_pos[sel] = off + np.arange(len(sel))
        send_ids.append(req[sel])
        counts.append(len(sel))
        off += len(sel)
    send_ids = np.concatenate(send_ids) if send_ids else np.zeros(0, np.int64)
    return send_ids.astype(np.int32), req_pos.astype(np.int32), np.array(counts, dtype=np.int64)


def route_cap(rec, rec_n1, start, count, G, C):
    """The fixed-capacity layout of skge_shard_route_cap: bucket g = slots
    [g C, (g + 1) C) holds the requests owned by rank g in request order,
    unused slots -1; req_pos = bucket slot of each request (-1: skipped)."""
    ids, pos, counts = route(rec, rec_n1, start, count, G)
    send = np.full(G * C, -1, dtype=np.int32)
    base = np.concatenate([[0], np.cumsum(counts)])[:-1]
    out_pos = np.full(pos.shape, -1, dtype=np.int32)
    for g in range(G):
        assert counts[g] <= C, "bucket overflow"
        send[g * C:g * C + counts[g]] = ids[base[g]:base[g] + counts[g]]
    for i, p in enumerate(pos):
        if p >= 0:
            g = int(np.searchsorted(base, p, side="right") - 1)
            out_pos[i] = g * C + (p - base[g])
    return send, out_pos


class NumpyShardOps(object):
    """Rank compute of one sharded step in float64 (d columns; the
    contribution record is [count, c_0 .. c_{d-1}] as float64), in the
    fixed-capacity layout (C slots per owner bucket)."""

    def __init__(self, rec, rec_n1, E_local, R, G, margin, lr, C):
        self.C = C
        self.rec, self.rec_n1 = rec, rec_n1
        self.E, self.R = E_local.astype(np.float64).copy(), R.astype(np.float64).copy()
        self.AE, self.AR = np.zeros_like(self.E), np.zeros_like(self.R)
        self.G, self.margin, self.lr = G, margin, lr
        self.d = self.E.shape[1]
        self.sumE, self.cntE = np.zeros_like(self.E), np.zeros(len(self.E), np.int64)
        self.sumR = torch.zeros(self.R.shape, dtype=torch.float64)
        self.cntR = torch.zeros(len(self.R), dtype=torch.int64)
        self.nviol = 0

    def buf(self, name):
        return None

    def route(self, start, count):
        s, p = route_cap(self.rec, self.rec_n1, start, count, self.G, self.C)
        return torch.from_numpy(s), torch.from_numpy(p)

    def gather(self, ids):
        i = ids.numpy().astype(np.int64)
        out = np.zeros((len(i), self.d))
        ok = i >= 0
        out[ok] = self.E[i[ok] // self.G]
        return torch.from_numpy(out)

    def score(self, start, count, fetched, req_pos):
        F = fetched.numpy()
        rp = req_pos.numpy().reshape(-1, 4)
        C = np.zeros((len(F), 1 + self.d))
        sumR, cntR = self.sumR.numpy(), self.cntR.numpy()
        for w in range(count):
            j = start + w
            p = self.rec[j, 2]
            es, eo = F[rp[w, 0]], F[rp[w, 1]]
            r = self.R[p]
            ps = -np.abs(es + r - eo).sum()                 # transe.py:25-46
            gp = np.sign(-(eo - r - es))                    # transe.py:103, 115
            v, g = [0, 0], [None, None]
            for k, (pos, ent) in enumerate(((rp[w, 2], 0), (rp[w, 3], 1))):
                if pos < 0:
                    continue
                f = F[pos]
                ns = -np.abs((f + r - eo) if ent == 0 else (es + r - f)).sum()
                v[k] = int(ns + self.margin > ps)           # strict >, transe.py:73
                g[k] = np.sign((eo - r - f) if ent == 0 else (f - r - es))   # transe.py:104, 117
            self.nviol += v[0] + v[1]
            z = np.zeros(self.d)
            g0 = g[0] if g[0] is not None else z
            g1 = g[1] if g[1] is not None else z
            # pair 0 rows (sp,op,sn,on) = (s,o,s',o): (+gp,-gp,+g0,-g0); pair 1 = (s,o,s,o')
            rows = [(rp[w, 0], v[0] + 2 * v[1], v[0] * gp + v[1] * (gp + g1)),
                    (rp[w, 1], 2 * v[0] + v[1], -(v[0] * (gp + g0) + v[1] * gp)),
                    (rp[w, 2], v[0], g0), (rp[w, 3], v[1], -g1)]
            for pos, c, vec in rows:
                if pos >= 0:
                    C[pos, 0] = c
                    C[pos, 1:] = vec if c else 0.0
            if v[0] + v[1]:
                sumR[p] += v[0] * (gp + g0) + v[1] * (gp + g1)
                cntR[p] += 2 * (v[0] + v[1])
        return torch.from_numpy(C)

    def accum(self, ids, contrib):
        C = contrib.numpy()
        for i, gid in enumerate(ids.numpy()):
            if gid >= 0 and C[i, 0]:
                row = int(gid) // self.G
                self.sumE[row] += C[i, 1:]
                self.cntE[row] += int(C[i, 0])

    def rel_sums(self):
        return self.sumR, self.cntR

    @staticmethod
    def _adagrad_normalize(P, A, S, cnt, lr, post):
        rows = np.nonzero(cnt)[0]
        g = S[rows] / cnt[rows, None]                      # Sm.dot(G) / n
        A[rows] += g * g                                   # param.py:147
        P[rows] -= lr * g / np.maximum(np.sqrt(A[rows]), 1e-7)   # param.py:152-155
        if post:
            P[rows] /= np.sqrt((P[rows] ** 2).sum(axis=1))[:, None]   # param.py:161-167
        S[rows] = 0.0
        cnt[rows] = 0

    def apply(self):
        self._adagrad_normalize(self.E, self.AE, self.sumE, self.cntE, self.lr, True)
        self._adagrad_normalize(self.R, self.AR, self.sumR.numpy(), self.cntR.numpy(), self.lr,
                                False)


def union_pairs(recs):
    """Explicit (pos, neg) pairs of every rank's batch, in the reference's
    pair layout ((s, o, p) rows): pair 0 corrupts s, pair 1 corrupts o."""
    pos, neg = [], []
    for rec, rec_n1, start, count in recs:
        for j in range(start, start + count):
            s, o, p, s1 = (int(x) for x in rec[j])
            o1 = int(rec_n1[j])
            if s1 >= 0:
                pos.append((s, o, p))
                neg.append((s1, o, p))
            if o1 >= 0:
                pos.append((s, o, p))
                neg.append((s, o1, p))
    return np.array(pos, dtype=np.int64).reshape(-1, 3), np.array(neg, dtype=np.int64).reshape(-1, 3)


def random_records(rs, T, n_ent, n_rel, skip=0.1):
    """Synthetic epoch records (s, o, p, s'|-1) and o'|-1 (negatives differ
    from the corrupted entity, as the sampler's set rejection guarantees)."""
    s = rs.randint(n_ent, size=T)
    o = rs.randint(n_ent, size=T)
    p = rs.randint(n_rel, size=T)
    s1 = (s + 1 + rs.randint(n_ent - 1, size=T)) % n_ent
    o1 = (o + 1 + rs.randint(n_ent - 1, size=T)) % n_ent
    s1[rs.rand(T) < skip] = -1
    o1[rs.rand(T) < skip] = -1
    return (np.stack([s, o, p, s1], axis=1).astype(np.int32), o1.astype(np.int32))
