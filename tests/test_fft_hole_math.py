"""The frequency-domain HolE step (csrc/skge_hole_fft.h) restated in NumPy:
the wave FFT's exact index math (Stockham autosort, radix 4 then 2, 3, 5,
butterfly i of a stage reading x[i + q M/R], twiddling by W_{pR}^{q k},
k = i mod p, writing y[(i / p) p R + k + t p]), the real-row packing
z_m = x_{2m} + i x_{2m+1} with its (k, M - k) post- / pre-processing, and the
HolE scores and contribution rows as spectral products -- checked against
numpy.fft and against the direct definitions of skge/util.py:8-50 (ccorr,
cconv) and skge/hole.py:44-100 (scores, rows), which the oracle restates.
CPU only: this pins the algorithm the device kernels implement; the GPU tests
check the kernels against the direct sums (test_hole_fft_matches_direct)."""
import numpy as np
import pytest


def plan(M):
    rs = []
    while M % 4 == 0:
        rs.append(4)
        M //= 4
    for r in (2, 3, 5):
        while M % r == 0:
            rs.append(r)
            M //= r
    return rs if M == 1 else None


def fft_ok(d):   # hole_fft_ok
    return d % 4 == 0 and d >= 4 and d // 4 + 1 <= 64 and plan(d // 2) is not None


def stockham(x, inv=False):
    N = len(x)
    sign = 1.0 if inv else -1.0
    p = 1
    x = np.asarray(x, complex).copy()
    for R in plan(N):
        T = N // R
        y = np.zeros(N, complex)
        for i in range(T):
            k = i % p
            u = np.array([x[i + q * T] for q in range(R)])
            u = u * np.exp(sign * 2j * np.pi * np.arange(R) * k / (p * R))
            v = np.array([np.sum(u * np.exp(sign * 2j * np.pi * np.arange(R) * t / R))
                          for t in range(R)])
            j = (i // p) * p * R + k
            y[j + np.arange(R) * p] = v
        x = y
        p *= R
    return x


def real_spectrum(x):
    """X_k, k = 0..M, from the complex transform of z_m = x_{2m} + i x_{2m+1}"""
    d = len(x)
    M = d // 2
    Z = stockham(x[0::2] + 1j * x[1::2])
    out = np.empty(M + 1, complex)
    for k in range(M // 2 + 1):   # one lane per pair (k, M - k)
        a, b = Z[k], Z[(M - k) % M]
        e, f = a + np.conj(b), a - np.conj(b)
        out[k] = 0.5 * e - 0.5j * np.exp(-2j * np.pi * k / d) * f
        e, f = b + np.conj(a), b - np.conj(a)
        out[M - k] = 0.5 * e - 0.5j * np.exp(-2j * np.pi * (M - k) / d) * f
    return out


def real_row(H, d):
    """the real row of Hermitian half-spectrum H (k = 0..M), via the complex
    inverse transform of length M"""
    M = d // 2
    Z = np.empty(M, complex)
    for k in range(M // 2 + 1):
        hk, hm = H[k], H[M - k]
        Z[k] = 0.5 * ((hk + np.conj(hm)) + 1j * np.exp(2j * np.pi * k / d) * (hk - np.conj(hm)))
        if 0 < k and M - k != k:
            Z[M - k] = 0.5 * ((hm + np.conj(hk)) +
                              1j * np.exp(2j * np.pi * (M - k) / d) * (hm - np.conj(hk)))
    z = stockham(Z, inv=True) / M
    x = np.empty(d)
    x[0::2], x[1::2] = z.real, z.imag
    return x


def ccorr(a, b):   # skge/util.py:30-50
    d = len(a)
    return np.array([sum(a[j] * b[(j + k) % d] for j in range(d)) for k in range(d)])


def cconv(a, b):   # skge/util.py:8-27
    d = len(a)
    return np.array([sum(a[j] * b[(k - j) % d] for j in range(d)) for k in range(d)])


def test_fft_support():
    assert fft_ok(200) and fft_ok(24) and fft_ok(40) and fft_ok(60) and fft_ok(32)
    assert not fft_ok(28) and not fft_ok(30) and not fft_ok(256) and not fft_ok(44)


@pytest.mark.parametrize("M", [100, 50, 16, 12, 20, 30, 48, 120])
def test_stockham_matches_numpy(M):
    rs = np.random.default_rng(M)
    z = rs.standard_normal(M) + 1j * rs.standard_normal(M)
    np.testing.assert_allclose(stockham(z), np.fft.fft(z), atol=1e-9)
    np.testing.assert_allclose(stockham(z, inv=True), np.fft.ifft(z) * M, atol=1e-9)


@pytest.mark.parametrize("d", [200, 24, 40, 60])
def test_real_packing(d):
    x = np.random.default_rng(d).standard_normal(d)
    np.testing.assert_allclose(real_spectrum(x), np.fft.rfft(x), atol=1e-9)
    np.testing.assert_allclose(real_row(np.fft.rfft(x), d), x, atol=1e-12)


@pytest.mark.parametrize("d", [200, 40])
def test_hole_scores_and_rows_in_the_frequency_domain(d):
    rs = np.random.default_rng(7)
    R, Es, Fs, Eo, Fo = (rs.standard_normal(d) for _ in range(5))
    Rh, Esh, Fsh, Eoh, Foh = (real_spectrum(v) for v in (R, Es, Fs, Eo, Fo))
    M = d // 2
    w = np.full(M + 1, 2.0)
    w[0] = w[M] = 1.0

    def score(ah, bh):   # R . ccorr(a, b) = (1/d) sum_k conj(a_k R_k) b_k
        return np.sum(w * np.real(np.conj(ah * Rh) * bh)) / d

    assert np.isclose(score(Esh, Eoh), R @ ccorr(Es, Eo))
    assert np.isclose(score(Fsh, Eoh), R @ ccorr(Fs, Eo))
    assert np.isclose(score(Esh, Foh), R @ ccorr(Es, Fo))
    gp, g0, g1 = -0.21, 0.17, 0.09
    A, B = ccorr(R, Eo), ccorr(R, Fo)
    C, D = cconv(Es, R), cconv(Fs, R)
    X, Y, Z = ccorr(Es, Eo), ccorr(Fs, Eo), ccorr(Es, Fo)
    for v0, v1 in ((1, 0), (0, 1), (1, 1)):
        # hole.py:76-96 summed per destination row
        want = {"s": v0 * gp * A + v1 * (gp * A + g1 * B),
                "o": v0 * (gp * C + g0 * D) + v1 * gp * C,
                "p": v0 * (gp * X + g0 * Y) + v1 * (gp * X + g1 * Z),
                "s'": g0 * A, "o'": g1 * C}
        cE, cF = (v0 + v1) * gp, (g1 if v1 else 0.0)
        uh = (v0 + v1) * gp * Esh + (g0 if v0 else 0.0) * Fsh
        got = {"s": real_row(np.conj(Rh) * (cE * Eoh + cF * Foh), d),
               "o": real_row(Rh * uh, d),
               "p": real_row(np.conj(uh) * Eoh + cF * np.conj(Esh) * Foh, d),
               "s'": real_row(g0 * np.conj(Rh) * Eoh, d),
               "o'": real_row(g1 * Rh * Esh, d)}
        for key in want:
            np.testing.assert_allclose(got[key], want[key], atol=1e-9, err_msg=key)
