#!/usr/bin/env python3
"""LDS bank-conflict model of the HolE wave FFT (csrc/skge_hole_fft.h) at
M = d/2 = 100 (d = 200): every ds instruction's lane addresses, grouped the
way the LDS serves them (64 banks x 4 B; a b64 access serves 32 lanes per
cycle, b128 16), and the cycles each takes = the most distinct dwords any
bank is asked for in a group.  Reports cycles per transform phase against
the conflict-free count, for a layout function (float2 index of element j of
signal t in buffer `buf` at stage s).  Host-only analysis, no GPU."""
import argparse

BANKS = 64


def cycles(addrs, width):
    """addrs: byte address per active lane (None: inactive); width 8 or 16."""
    per = 256 // width                     # lanes served per cycle
    tot = 0
    for g0 in range(0, 64, per):
        banks = {}
        for a in addrs[g0:g0 + per]:
            if a is None:
                continue
            for w in range(width // 4):
                dw = a // 4 + w
                banks.setdefault(dw % BANKS, set()).add(dw)
        tot += max((len(v) for v in banks.values()), default=0)
    return tot


def ideal(addrs, width):
    per = 256 // width
    return sum(1 for g0 in range(0, 64, per) if any(a is not None for a in addrs[g0:g0 + per]))


def radices(M):
    out, m = [], M
    for R in (4, 2, 3, 5):
        while m % R == 0 and not (R == 2 and m % 4 == 0 and 4 in out and False):
            if R == 4 or (R == 2 and m % 4 != 0) or R in (3, 5):
                out.append(R)
                m //= R
            else:
                break
    return out


def stage_accesses(M, NT, R, P, lay_in, lay_out, s):
    """fft_stage_c<R, INV, M, NT, P>: per pass j, per q one read, per t one write."""
    T = M // R
    n = NT * T
    insts = []
    for j in range((n + 63) // 64):
        lanes = [(l + 64 * j) for l in range(64)]
        def bti(b):
            tr, i = b // T, b % T
            return tr, i, i // P, i % P
        for q in range(R):
            insts.append(("r", [8 * lay_in(bti(b)[0], bti(b)[1] + q * T, s) if b < n else None
                                for b in lanes], 8))
        for t in range(R):
            insts.append(("w", [8 * lay_out(bti(b)[0], bti(b)[2] * P * R + bti(b)[3] + t * P, s + 1)
                                if b < n else None for b in lanes], 8))
    return insts


def natural(S):
    return lambda t, j, s: t * S + j


def report(M, NT, layout, name):
    rs = []
    m = M
    for R in (4, 2, 3, 5):
        while m % R == 0:
            rs.append(R)
            m //= R
    tot = idl = 0
    P = 1
    for s, R in enumerate(rs):
        insts = stage_accesses(M, NT, R, P, layout, layout, s)
        c = sum(cycles(a, w) for _, a, w in insts)
        i = sum(ideal(a, w) for _, a, w in insts)
        print("  stage %d R=%d P=%-3d cycles %4d ideal %4d" % (s, R, P, c, i))
        tot += c
        idl += i
        P *= R
    print("%-28s NT=%d: %d cycles, ideal %d (conflict share %.2f)" % (name, NT, tot, idl,
                                                                       1 - idl / tot))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=100)
    args = ap.parse_args()
    for nt in (5, 4):
        report(args.M, nt, natural(args.M), "natural (stride M)")


if __name__ == "__main__":
    main()


def padded(S, sh, pw):
    """float2 index t*S + j + (j >> sh) * pw (sh 0: no padding)"""
    return lambda t, j: t * S + j + ((j >> sh) * pw if sh else 0)


def total_cycles(M, NT, lays):
    """lays[k]: the layout of the buffer stage k reads (k = number of stages: the output)"""
    rs = []
    m = M
    for R in (4, 2, 3, 5):
        while m % R == 0:
            rs.append(R)
            m //= R
    tot, P = 0, 1
    for s, R in enumerate(rs):
        insts = stage_accesses(M, NT, R, P, lambda t, j, s_: lays[s](t, j),
                               lambda t, j, s_: lays[s + 1](t, j), s)
        tot += sum(cycles(a, w) for _, a, w in insts)
        P *= R
    return tot, len(rs)
