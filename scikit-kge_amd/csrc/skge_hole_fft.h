// HolE in the frequency domain (round 2): the per-positive HolE step of the
// device loops (k_hole_pos, k_hole_pipe) with the circular correlations of
// skge/util.py:8-50 evaluated the way the reference evaluates them -- through
// the DFT (ccorr(a,b) = ifft(conj(fft a) * fft b), cconv(a,b) = ifft(fft a *
// fft b)) -- by a hand-rolled mixed-radix FFT that one wavefront runs in its
// LDS, instead of direct O(d^2) sums.
//
// Real rows of length d are transformed as complex signals of length
// M = d / 2 (z_m = x_{2m} + i x_{2m+1}: a lane's quad x[4l..4l+3] IS
// z[2l..2l+1], so rows enter and leave the transform without shuffles), by a
// Stockham autosort FFT (radix 4, then 2, 3, 5; every stage reads with stride
// M/R and writes in place of the next stage's input, natural order at the
// end).  Lane k <= M/2 then holds the spectrum at k and M - k of every row,
// which is all the real post-/pre-processing and the Hermitian sums need:
//   score(s,o,p) = R . ccorr(E[s], E[o]) = (1/d) sum_k conj(E^s_k R^_k) E^o_k
// (each k < M counted twice, k = 0 and M once), and for a violating positive
// (hole.py:76-96, rows summed per destination, u = (v0+v1) gp E[s] + v0 g0 E[s'])
//   E[s] : conj(R) ((v0+v1) gp E^o + v1 g1 E^o')     E[s'] : g0 conj(R) E^o
//   E[o] : R u^                                        E[o'] : g1 R E^s
//   R[p] : conj(u^) E^o + v1 g1 conj(E^s) E^o'
// become 3-5 inverse transforms.  Per positive: 5 forward + 3-5 inverse
// transforms of length M (~(4+5+5) M complex multiply-adds each at d = 200)
// instead of 2-6 direct correlations of d^2 multiply-adds.
// Twiddles W^t = exp(-2 pi i t / d), t < d, come from a table computed on the
// host in double precision, copied into each wave's LDS; every twiddle of
// every stage is a power of W.
#pragma once
#include "skge_hole.h"

namespace skge {

// d % 4 == 0, M = d / 2 a product of 2, 3, 5, and the pairs (k, M - k),
// k <= M / 2, one per lane
__host__ __device__ __forceinline__ bool hole_fft_ok(int d) {
  if (d % 4 != 0 || d < 4 || d / 4 + 1 > 64) return false;
  int m = d / 2;
  for (int r = 2; r <= 5; ++r)
    while (m % r == 0) m /= r;
  return m == 1;
}
// wave-private floats: two ping-pong buffers of 5 complex rows of length M
__host__ __device__ __forceinline__ int hole_fft_wave_floats(int d) { return 10 * d; }
// workgroup LDS: the twiddle table (d complex), then the waves' regions
__host__ __device__ __forceinline__ size_t hole_fft_lds_bytes(int d, int waves) {
  return (size_t)(2 * d + waves * hole_fft_wave_floats(d)) * sizeof(float);
}
// the device twiddle table W^t = exp(-2 pi i t / d), t < d, computed on the
// host in double precision; allocated once per d (call outside stream capture:
// the runners call it at creation)
const float2* hole_fft_table(int d);

__device__ __forceinline__ float2 cmul(const float2& a, const float2& b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cmulc(const float2& a, const float2& b) {   // conj(a) b
  return make_float2(a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float2 cadd(const float2& a, const float2& b) {
  return make_float2(a.x + b.x, a.y + b.y);
}
__device__ __forceinline__ float2 csub(const float2& a, const float2& b) {
  return make_float2(a.x - b.x, a.y - b.y);
}
__device__ __forceinline__ float2 cscale(float s, const float2& a) {
  return make_float2(s * a.x, s * a.y);
}
__device__ __forceinline__ float2 cconj(const float2& a) { return make_float2(a.x, -a.y); }

// the workgroup's copy of the twiddle table (every thread, then a barrier)
__device__ __forceinline__ void fft_twiddles(float2* tw, const float2* __restrict__ g, int d) {
  for (int t = threadIdx.x; t < d; t += blockDim.x) tw[t] = g[t];
}

// DFT of R points, forward (exp(-2 pi i qt / R)) or inverse (conjugate):
// radix 2 / 4 with additions only, 3 and 5 in the symmetric form (real
// constants times sums and differences of the conjugate-pair inputs)
__device__ __forceinline__ float2 mul_i(const float2& a) { return make_float2(-a.y, a.x); }   // i a
template <int R, bool INV>
__device__ __forceinline__ void fft_dft(const float2 (&u)[R], float2 (&v)[R]) {
  if (R == 2) {
    v[0] = cadd(u[0], u[1]);
    v[1] = csub(u[0], u[1]);
  } else if (R == 4) {
    const float2 a = cadd(u[0], u[2]), b = csub(u[0], u[2]);
    const float2 c = cadd(u[1], u[3]), e = csub(u[1], u[3]);
    v[0] = cadd(a, c);
    v[2] = csub(a, c);
    // forward: v1 = b - i e, v3 = b + i e (inverse: swapped)
    const float2 ie = mul_i(e);
    v[INV ? 1 : 3] = cadd(b, ie);
    v[INV ? 3 : 1] = csub(b, ie);
  } else if (R == 3) {
    constexpr float s3 = 0.86602540378443864676f;   // sin(2 pi / 3)
    const float2 t1 = cadd(u[1], u[2]), t2 = csub(u[1], u[2]);
    v[0] = cadd(u[0], t1);
    const float2 a = make_float2(u[0].x - 0.5f * t1.x, u[0].y - 0.5f * t1.y);
    const float2 ib = mul_i(cscale(s3, t2));
    v[INV ? 2 : 1] = csub(a, ib);
    v[INV ? 1 : 2] = cadd(a, ib);
  } else {   // R == 5
    constexpr float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;   // cos 2pi/5, 4pi/5
    constexpr float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;    // sin 2pi/5, 4pi/5
    const float2 t1 = cadd(u[1], u[4]), t2 = cadd(u[2], u[3]);
    const float2 t3 = csub(u[1], u[4]), t4 = csub(u[2], u[3]);
    v[0] = cadd(u[0], cadd(t1, t2));
    const float2 a1 = make_float2(u[0].x + c1 * t1.x + c2 * t2.x, u[0].y + c1 * t1.y + c2 * t2.y);
    const float2 a2 = make_float2(u[0].x + c2 * t1.x + c1 * t2.x, u[0].y + c2 * t1.y + c1 * t2.y);
    const float2 ib1 = mul_i(make_float2(s1 * t3.x + s2 * t4.x, s1 * t3.y + s2 * t4.y));
    const float2 ib2 = mul_i(make_float2(s2 * t3.x - s1 * t4.x, s2 * t3.y - s1 * t4.y));
    // forward: v1 = a1 - i b1, v4 = a1 + i b1, v2 = a2 - i b2, v3 = a2 + i b2
    v[INV ? 4 : 1] = csub(a1, ib1);
    v[INV ? 1 : 4] = cadd(a1, ib1);
    v[INV ? 3 : 2] = csub(a2, ib2);
    v[INV ? 2 : 3] = cadd(a2, ib2);
  }
}

// one Stockham radix-R stage over nt transforms of length M (x -> y): the
// butterfly i < M/R of a transform reads x[i + q M/R], twiddles input q by
// W_{pR}^{q k} (k = i mod p), and writes y[(i / p) p R + k + t p]
template <int R, bool INV>
__device__ __forceinline__ void fft_stage(const float2* x, float2* y, int M, int p, int nt,
                                          const float2* tw, int d) {
  const int T = M / R, n = nt * T, stw = d / (p * R);
  // b / T and i / p by a float reciprocal: b + 0.5 keeps the quotient at least
  // 1/(2T) >= 1/256 away from an integer (T, p <= 128), far above the product's
  // rounding for b < 2^16
  const float rT = 1.0f / (float)T, rp = 1.0f / (float)p;
  for (int b = lane_id(); b < n; b += 64) {
    const int tr = (int)(((float)b + 0.5f) * rT), i = b - tr * T;
    const int ip = (int)(((float)i + 0.5f) * rp), k = i - ip * p;
    const float2* xs = x + tr * M + i;
    float2 u[R], v[R];
#pragma unroll
    for (int q = 0; q < R; ++q) u[q] = xs[q * T];
    if (p > 1) {
#pragma unroll
      for (int q = 1; q < R; ++q) {
        float2 w = tw[q * k * stw];
        if (INV) w.y = -w.y;
        u[q] = cmul(u[q], w);
      }
    }
    fft_dft<R, INV>(u, v);
    float2* ys = y + tr * M + ip * p * R + k;
#pragma unroll
    for (int t = 0; t < R; ++t) ys[t * p] = v[t];
  }
}

// nt complex transforms of length M, in b0 on entry; returns the buffer that
// holds the result (b0 or b1).  Unscaled in both directions.
template <bool INV>
__device__ __forceinline__ float2* fft_run(float2* b0, float2* b1, int M, int nt,
                                           const float2* tw, int d) {
  float2 *x = b0, *y = b1;
  int p = 1, m = M;
#define SKGE_FFT_STAGES(R)                              \
  while (m % R == 0) {                                  \
    __builtin_amdgcn_wave_barrier();                    \
    fft_stage<R, INV>(x, y, M, p, nt, tw, d);           \
    float2* t_ = x;                                     \
    x = y;                                              \
    y = t_;                                             \
    p *= R;                                             \
    m /= R;                                             \
  }
  SKGE_FFT_STAGES(4)
  SKGE_FFT_STAGES(2)
  SKGE_FFT_STAGES(3)
  SKGE_FFT_STAGES(5)
#undef SKGE_FFT_STAGES
  __builtin_amdgcn_wave_barrier();
  return x;
}

// The same stages for a compile-time transform length M and signal count NT
// (round 3; the device loops' d = 200 -> M = 100): the butterfly indices come
// from divisions by constants and every pass of a stage is unrolled (no loop
// control, no float-reciprocal index arithmetic).  Same arithmetic in the same
// order as fft_stage, so the same bits.
template <int R, bool INV, int M, int NT, int P>
__device__ __forceinline__ void fft_stage_c(const float2* x, float2* y, const float2* tw) {
  constexpr int T = M / R, n = NT * T, stw = 2 * M / (P * R), NP = (n + 63) / 64;
  int l = lane_id();
  // opaque: the lane-constant index arithmetic stays here instead of being
  // hoisted out of the caller's loop into ~40 long-lived registers
  asm volatile("" : "+v"(l));
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int b = l + 64 * j;
    if (64 * (j + 1) <= n || b < n) {
      const int tr = b / T, i = b - tr * T;
      const int ip = i / P, k = i - ip * P;
      const float2* xs = x + tr * M + i;
      float2 u[R], v[R];
#pragma unroll
      for (int q = 0; q < R; ++q) u[q] = xs[q * T];
      if (P > 1) {
#pragma unroll
        for (int q = 1; q < R; ++q) {
          float2 w = tw[q * k * stw];
          if (INV) w.y = -w.y;
          u[q] = cmul(u[q], w);
        }
      }
      fft_dft<R, INV>(u, v);
      float2* ys = y + tr * M + ip * P * R + k;
#pragma unroll
      for (int t = 0; t < R; ++t) ys[t * P] = v[t];
    }
  }
}

// fft_run for a compile-time M and NT (the radix order of fft_run: 4s, a 2,
// 3s, 5s)
template <int M, int NT, bool INV, int P = 1, int MR = M>
__device__ __forceinline__ float2* fft_run_c(float2* x, float2* y, const float2* tw) {
  if constexpr (MR == 1) {
    __builtin_amdgcn_wave_barrier();
    return x;
  } else {
    constexpr int R = MR % 4 == 0 ? 4 : (MR % 2 == 0 ? 2 : (MR % 3 == 0 ? 3 : 5));
    static_assert(MR % R == 0, "the transform length must factor into 2, 3 and 5");
    __builtin_amdgcn_wave_barrier();
    fft_stage_c<R, INV, M, NT, P>(x, y, tw);
    return fft_run_c<M, NT, INV, P * R, MR / R>(y, x, tw);
  }
}

// Pair form (round 4, SKGE_HPIPE_PAIR): the two waves of a 128-thread
// workgroup run ONE positive's transforms together in the workgroup's
// buffers -- wave h takes the stage passes j = h, h + 2, ... of
// fft_stage_c, so each butterfly is the same arithmetic on the same inputs
// (the same bits as fft_run_c) and a stage boundary is a workgroup barrier.
template <int R, bool INV, int M, int NT, int P>
__device__ __forceinline__ void fft_stage_c2(const float2* x, float2* y, const float2* tw, int h) {
  constexpr int T = M / R, n = NT * T, stw = 2 * M / (P * R), NP = (n + 63) / 64;
  int l = lane_id();
  asm volatile("" : "+v"(l));
#pragma unroll
  for (int jj = 0; jj < (NP + 1) / 2; ++jj) {
    const int b = l + 64 * (2 * jj + h);
    if (b < n) {
      const int tr = b / T, i = b - tr * T;
      const int ip = i / P, k = i - ip * P;
      const float2* xs = x + tr * M + i;
      float2 u[R], v[R];
#pragma unroll
      for (int q = 0; q < R; ++q) u[q] = xs[q * T];
      if (P > 1) {
#pragma unroll
        for (int q = 1; q < R; ++q) {
          float2 w = tw[q * k * stw];
          if (INV) w.y = -w.y;
          u[q] = cmul(u[q], w);
        }
      }
      fft_dft<R, INV>(u, v);
      float2* ys = y + tr * M + ip * P * R + k;
#pragma unroll
      for (int t = 0; t < R; ++t) ys[t * P] = v[t];
    }
  }
}

// fft_run_c over the pair (entered after a barrier that published the
// inputs; returns after the barrier that publishes the output)
template <int M, int NT, bool INV, int P = 1, int MR = M>
__device__ __forceinline__ float2* fft_run_c2(float2* x, float2* y, const float2* tw, int h) {
  if constexpr (MR == 1) {
    return x;
  } else {
    constexpr int R = MR % 4 == 0 ? 4 : (MR % 2 == 0 ? 2 : (MR % 3 == 0 ? 3 : 5));
    static_assert(MR % R == 0, "the transform length must factor into 2, 3 and 5");
    fft_stage_c2<R, INV, M, NT, P>(x, y, tw, h);
    __syncthreads();
    return fft_run_c2<M, NT, INV, P * R, MR / R>(y, x, tw, h);
  }
}

// quad-layout real row -> complex signal t of buffer b (z[2l], z[2l+1])
__device__ __forceinline__ void fft_put_row(float2* b, int M, int t, const float4& v, int d) {
  const int l = lane_id();
  if (4 * l < d) *reinterpret_cast<float4*>(b + t * M + 2 * l) = v;
}

// the spectrum at k and M - k of real row t from its complex transform Z:
// X_k = (Z_k + conj Z_{M-k}) / 2 - i W^k (Z_k - conj Z_{M-k}) / 2  (Z_M = Z_0)
__device__ __forceinline__ void fft_real_pair(const float2* Z, int M, int k, const float2* tw,
                                              float2& xk, float2& xmk) {
  const float2 a = Z[k], b = Z[k == 0 ? 0 : M - k];
  {
    const float2 e = cadd(a, cconj(b)), f = csub(a, cconj(b));
    const float2 wf = cmul(tw[k], f);
    xk = make_float2(0.5f * (e.x + wf.y), 0.5f * (e.y - wf.x));
  }
  {
    const float2 e = cadd(b, cconj(a)), f = csub(b, cconj(a));
    const float2 wf = cmul(tw[M - k], f);
    xmk = make_float2(0.5f * (e.x + wf.y), 0.5f * (e.y - wf.x));
  }
}

// inverse pre-processing of a Hermitian half-spectrum (H at k and M - k):
// Z'_k = ((H_k + conj H_{M-k}) + i conj(W^k) (H_k - conj H_{M-k})) / 2, written
// at k (< M) and at M - k (when 0 < k and M - k != k)
__device__ __forceinline__ void fft_real_inv_pair(float2* Z, int M, int k, const float2* tw,
                                                  const float2& hk, const float2& hmk) {
  {
    const float2 e = cadd(hk, cconj(hmk)), f = csub(hk, cconj(hmk));
    const float2 wf = cmulc(tw[k], f);   // conj(W^k) f
    Z[k] = make_float2(0.5f * (e.x - wf.y), 0.5f * (e.y + wf.x));
  }
  if (k > 0 && M - k != k) {
    const float2 e = cadd(hmk, cconj(hk)), f = csub(hmk, cconj(hk));
    const float2 wf = cmulc(tw[M - k], f);
    Z[M - k] = make_float2(0.5f * (e.x - wf.y), 0.5f * (e.y + wf.x));
  }
}

// complex signal t of b -> quad-layout real row, times s
__device__ __forceinline__ float4 fft_get_row(const float2* b, int M, int t, float s, int d) {
  const int l = lane_id();
  if (4 * l >= d) return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  const float4 v = *reinterpret_cast<const float4*>(b + t * M + 2 * l);
  return make_float4(s * v.x, s * v.y, s * v.z, s * v.w);
}

// Re(conj(a r) b) at one k, weighted: the Hermitian sum's term
__device__ __forceinline__ float fft_score_term(const float2& a, const float2& r, const float2& b) {
  const float2 ar = cmul(a, r);
  return ar.x * b.x + ar.y * b.y;
}

// Forward phase of one positive: rows R[p], E[s], E[s'], E[o], E[o'] (quad
// layout) -> spectra at (k, M - k) for lane k <= M/2, and the three raw
// scores R.ccorr(E[s],E[o]), R.ccorr(E[s'],E[o]), R.ccorr(E[s],E[o']).
struct HoleSpec {
  float2 r[2], es[2], fs[2], eo[2], fo[2];   // [0]: k, [1]: M - k
  int k;
  bool on;                                   // lane holds a pair
};
// the spectra at (k, M - k) of the five transformed rows in Z and the three
// raw scores (hole_fft_forward's second half; the pair form calls it in both
// waves, which then hold the same values)
__device__ __forceinline__ HoleSpec hole_fft_spectra(const float2* Z, const float2* tw, int d,
                                                     float& praw, float& raw0, float& raw1) {
  const int M = d / 2;
  HoleSpec h;
  h.k = lane_id();
  h.on = h.k <= M / 2;
  float ps = 0.0f, p0 = 0.0f, p1 = 0.0f;
  if (h.on) {
    const int k = h.k;
    fft_real_pair(Z + 0 * M, M, k, tw, h.r[0], h.r[1]);
    fft_real_pair(Z + 1 * M, M, k, tw, h.es[0], h.es[1]);
    fft_real_pair(Z + 2 * M, M, k, tw, h.fs[0], h.fs[1]);
    fft_real_pair(Z + 3 * M, M, k, tw, h.eo[0], h.eo[1]);
    fft_real_pair(Z + 4 * M, M, k, tw, h.fo[0], h.fo[1]);
    // weights: k and M - k each count twice unless 0 or M; the middle pair once
    const float wk = k == 0 ? 1.0f : 2.0f, wm = k == 0 ? 1.0f : (M - k == k ? 0.0f : 2.0f);
    ps = wk * fft_score_term(h.es[0], h.r[0], h.eo[0]) + wm * fft_score_term(h.es[1], h.r[1], h.eo[1]);
    p0 = wk * fft_score_term(h.fs[0], h.r[0], h.eo[0]) + wm * fft_score_term(h.fs[1], h.r[1], h.eo[1]);
    p1 = wk * fft_score_term(h.es[0], h.r[0], h.fo[0]) + wm * fft_score_term(h.es[1], h.r[1], h.fo[1]);
  }
  const float inv_d = 1.0f / (float)d;
  praw = wave_sum(ps) * inv_d;
  raw0 = wave_sum(p0) * inv_d;
  raw1 = wave_sum(p1) * inv_d;
  return h;
}

__device__ __forceinline__ HoleSpec hole_fft_forward(float* wbuf, const float2* tw, int d,
                                                     const float4& rp, const float4& es,
                                                     const float4& fs, const float4& eo,
                                                     const float4& fo, float& praw, float& raw0,
                                                     float& raw1) {
  const int M = d / 2;
  float2* b0 = reinterpret_cast<float2*>(wbuf);
  float2* b1 = b0 + 5 * M;
  fft_put_row(b0, M, 0, rp, d);
  fft_put_row(b0, M, 1, es, d);
  fft_put_row(b0, M, 2, fs, d);
  fft_put_row(b0, M, 3, eo, d);
  fft_put_row(b0, M, 4, fo, d);
  const float2* Z = M == 100 ? fft_run_c<100, 5, false>(b0, b1, tw)
                             : fft_run<false>(b0, b1, M, 5, tw, d);
  return hole_fft_spectra(Z, tw, d, praw, raw0, raw1);
}

// Inverse phase of a violating positive: the contribution rows of
// hole_pos_rows as real rows in LDS -- the inverse transforms' output, whose
// complex interleave (z_m = x_{2m} + i x_{2m+1}) is the real row in natural
// order -- times 1/M.  Rows: 0 E[s], 1 E[o], 2 R[p], then E[s'] when v0, then
// E[o'] when v1.  Returns the buffer (float view, row t at t * d).
// the inverse transforms' inputs (pre-processed half spectra) of the
// contribution rows t in [lo, hi): 0 E[s], 1 E[o], 2 R[p], then E[s'] (v0),
// E[o'] (v1)
__device__ __forceinline__ void hole_inv_inputs(float2* b0, int M, const float2* tw,
                                                const HoleSpec& h, int v0, int v1, float gp,
                                                float g0, float g1, int lo, int hi) {
  if (!h.on) return;
  const float cE = (float)(v0 + v1) * gp, cF = v1 ? g1 : 0.0f;   // E[s] row
  const float cu = (float)(v0 + v1) * gp, cf = v0 ? g0 : 0.0f;   // u = cu E[s] + cf E[s']
  float2 H[5][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float2 r = h.r[j], eo = h.eo[j], fo = h.fo[j], es = h.es[j];
    const float2 uh = cadd(cscale(cu, es), cscale(cf, h.fs[j]));
    H[0][j] = cmulc(r, cadd(cscale(cE, eo), cscale(cF, fo)));          // E[s]
    H[1][j] = cmul(r, uh);                                            // E[o]
    H[2][j] = cadd(cmulc(uh, eo), cscale(cF, cmulc(es, fo)));         // R[p]
    H[3][j] = cscale(g0, cmulc(r, eo));                               // E[s'] (v0)
    H[4][j] = cscale(g1, cmul(r, es));                                // E[o'] (v1)
  }
  const int k = h.k;
  if (lo <= 0 && 0 < hi) fft_real_inv_pair(b0 + 0 * M, M, k, tw, H[0][0], H[0][1]);
  if (lo <= 1 && 1 < hi) fft_real_inv_pair(b0 + 1 * M, M, k, tw, H[1][0], H[1][1]);
  if (lo <= 2 && 2 < hi) fft_real_inv_pair(b0 + 2 * M, M, k, tw, H[2][0], H[2][1]);
  int t = 3;
  if (v0) {
    if (lo <= t && t < hi) fft_real_inv_pair(b0 + t * M, M, k, tw, H[3][0], H[3][1]);
    ++t;
  }
  if (v1 && lo <= t && t < hi) fft_real_inv_pair(b0 + t * M, M, k, tw, H[4][0], H[4][1]);
}

__device__ __forceinline__ const float* hole_fft_rows(float* wbuf, const float2* tw, int d,
                                                      const HoleSpec& h, int v0, int v1,
                                                      float gp, float g0, float g1) {
  const int M = d / 2;
  float2* b0 = reinterpret_cast<float2*>(wbuf);
  float2* b1 = b0 + 5 * M;
  const int nt = 3 + v0 + v1;
  __builtin_amdgcn_wave_barrier();   // every lane is done reading the forward buffers
  hole_inv_inputs(b0, M, tw, h, v0, v1, gp, g0, g1, 0, 5);
  float2* z;
  if (M == 100 && nt == 5)
    z = fft_run_c<100, 5, true>(b0, b1, tw);
  else if (M == 100 && nt == 4)
    z = fft_run_c<100, 4, true>(b0, b1, tw);
  else
    z = fft_run<true>(b0, b1, M, nt, tw, d);
  return reinterpret_cast<const float*>(z);
}

// Pair form of hole_fft_rows (M = 100): both waves hold the spectra h; wave hw
// writes its share of the inverse inputs (0: rows 0-2, 1: the negatives'
// rows), then the pair runs the transforms.  Same bits as hole_fft_rows.
__device__ __forceinline__ const float* hole_fft_rows_pair(float* wbuf, const float2* tw,
                                                           const HoleSpec& h, int v0, int v1,
                                                           float gp, float g0, float g1, int hw) {
  constexpr int M = 100;
  float2* b0 = reinterpret_cast<float2*>(wbuf);
  float2* b1 = b0 + 5 * M;
  __syncthreads();   // both waves are done reading the forward buffers
  hole_inv_inputs(b0, M, tw, h, v0, v1, gp, g0, g1, hw ? 3 : 0, hw ? 5 : 3);
  __syncthreads();
  float2* z = v0 + v1 == 2 ? fft_run_c2<M, 5, true>(b0, b1, tw, hw)
                           : fft_run_c2<M, 4, true>(b0, b1, tw, hw);
  return reinterpret_cast<const float*>(z);
}

// row t of hole_fft_rows' output, scaled by 1/M, added into accumulator row
// `row`: lane l takes elements l + 64 k, so each float-atomic instruction
// covers contiguous bytes (MI355X_MICROARCH.md "Global float atomics")
template <int KM>
__device__ __forceinline__ void acc_fft_row(const Accum& acc, int row, const float* z, int t,
                                            int d) {
  const float s = 2.0f / (float)d;   // 1/M
  float x[KM];
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    x[k] = e < d ? s * z[t * d + e] : 0.0f;
  }
  acc_row<KM>(acc, row, x, d);
}

}  // namespace skge
