// Scoring + contribution-scatter kernels for explicit pairs / labelled triples.
//
// One wavefront per pair (or triple).  A row of width d lives lane-strided in
// KM = ceil(d/64) registers per lane (skge_device.h), so every gather and
// every float atomic of a row is a sequence of 256-byte contiguous
// wave-instructions.  Contributions are summed into the per-table segment
// accumulator (Accum): the device form of grad_sum_matrix + Sm.dot(G)
// (skge/util.py:53-101).  The division by the occurrence count (the mean)
// happens later, in skge_accum_apply / skge_accum_collect.
#include <stdarg.h>

#include <cmath>
#include <map>
#include <mutex>
#include <vector>

#include "skge_hole.h"
#include "skge_hole_fft.h"
#include "skge_host.h"

namespace skge {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

struct PairArgs {
  const float* E;
  const float* R;  // relation table [M][d] (TransE, HolE) or W [M][d][d] (RESCAL)
  Accum accE, accR;
  const int* pos;
  const int* neg;
  const float* ys;  // logistic only
  int P, d, af;
  float margin;
  float* pscore;
  float* nscore;
  float* coef;
  int* nviol;
  float* loss;
  int record;  // 0: score only (no contribution scatter, no slot writes)
  int* eviol;  // optional per-entity violation counter (TransE pairs)
  const float2* tw;   // HolE FFT form: the twiddle table (hole_fft_table)
};


template <int KM>
__device__ __forceinline__ void to_lds(float* s, const float (&v)[KM], int d) {
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    if (e < d) s[e] = v[k];
  }
}

// c_k = sum_j a_j b_{(j+k) mod d}      (ccorr, skge/util.py:30-50)
template <int KM>
__device__ __forceinline__ void ccorr_lds(const float* sa, const float* sb, int d, float (&out)[KM]) {
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < KM; ++k) out[k] = 0.0f;
  for (int j = 0; j < d; ++j) {
    const float aj = sa[j];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int kk = l + 64 * k;
      int ix = j + kk;
      ix = ix >= d ? ix - d : ix;
      ix = kk < d ? ix : 0;
      out[k] = fmaf(aj, sb[ix], out[k]);
    }
  }
}

// c_k = sum_j a_j b_{(k-j) mod d}      (cconv, skge/util.py:8-27)
template <int KM>
__device__ __forceinline__ void cconv_lds(const float* sa, const float* sb, int d, float (&out)[KM]) {
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < KM; ++k) out[k] = 0.0f;
  for (int j = 0; j < d; ++j) {
    const float aj = sa[j];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int kk = l + 64 * k;
      int ix = kk - j;
      ix = ix < 0 ? ix + d : ix;
      ix = kk < d ? ix : 0;
      out[k] = fmaf(aj, sb[ix], out[k]);
    }
  }
}

// ---- register-tiled circular correlation (HolE, d % 4 == 0, d <= 256) ----
// corr_quad_b (skge_hole.h): lane l owns outputs 4l..4l+3 and slides an
// 8-float window of b along j (b stored twice in LDS so j+k needs no mod);
// cconv(a, b) = ccorr(a', b) with a'_m = a_{(-m) mod d} (stored reversed).
// The quad result goes through a wave-private LDS row back to the lane-
// strided layout of the rest of the kernel.
__device__ __forceinline__ bool hole_fast(int d) { return (d & 3) == 0 && d >= 4 && d <= 256; }
// wave-private LDS floats of the fast HolE pair kernel: four a operands
// (d + 4), four doubled rows (2d + 4), the output row
__host__ __device__ __forceinline__ int hole_fast_lds_floats(int d) { return 13 * d + 32; }

template <int KM>
__device__ __forceinline__ void to_lds_dbl(float* s2, const float (&v)[KM], int d) {
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    if (e < d) {
      s2[e] = v[k];
      s2[e + d] = v[k];
    }
  }
  if (l < 4) s2[2 * d + l] = 0.0f;   // read (unused) by the last window refill
}

// a operand of corr_fast (d + 4 floats): a[d] = a[0]
template <int KM>
__device__ __forceinline__ void to_lds_a(float* s, const float (&v)[KM], int d) {
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    if (e < d) s[e] = v[k];
  }
  if (l == 0) s[d] = v[0];
}

template <int KM>
__device__ __forceinline__ void to_lds_rev(float* s, const float (&v)[KM], int d) {
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    if (e < d) s[e == 0 ? 0 : d - e] = v[k];
  }
  if (l == 0) s[d] = v[0];
}

template <int KM>
__device__ __forceinline__ void corr_fast(const float* sa, const float* sb2, float* sout, int d,
                                          float (&out)[KM], float4* quad = nullptr) {
  const int l = lane_id(), base = 4 * l;
  const float* const b1[1] = {sb2};
  float4 q[1];
  corr_quad_b<1>(sa, b1, d, q);
  if (quad) *quad = q[0];   // zeros past the row
  if (base < d) *reinterpret_cast<float4*>(sout + base) = q[0];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    out[k] = e < d ? sout[e] : 0.0f;
  }
  __builtin_amdgcn_wave_barrier();
}

// out_i = sum_j W[i][j] x_j   (W[p] . E[o], skge/rescal.py:212)
template <int KM>
__device__ __forceinline__ void gemv_rows(const float* __restrict__ Wp, const float* sx, int d, float (&out)[KM]) {
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int i = l + 64 * k;
    float acc = 0.0f;
    if (i < d) {
      const float* row = Wp + (size_t)i * d;
      for (int j = 0; j < d; ++j) acc = fmaf(row[j], sx[j], acc);
    }
    out[k] = acc;
  }
}

// out_j = sum_i x_i W[i][j]   (E[s] . W[p], skge/rescal.py:209)
template <int KM>
__device__ __forceinline__ void gemv_cols(const float* __restrict__ Wp, const float* sx, int d, float (&out)[KM]) {
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < KM; ++k) out[k] = 0.0f;
  for (int i = 0; i < d; ++i) {
    const float xi = sx[i];
    const float* row = Wp + (size_t)i * d;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int j = l + 64 * k;
      if (j < d) out[k] = fmaf(xi, row[j], out[k]);
    }
  }
}

template <int KM>
__device__ __forceinline__ void scale(float (&o)[KM], const float (&v)[KM], float c) {
#pragma unroll
  for (int k = 0; k < KM; ++k) o[k] = c * v[k];
}

// add rows x (coefficient already applied) at a and y at b, merging when a == b
// (the matching counts are committed by commit_pair / commit_triple)

// ---------------------------------------------------------------------------
// TransE pair: skge/transe.py:48-165
// ---------------------------------------------------------------------------
template <int KM, bool L1>
__device__ __forceinline__ bool transe_pair(const PairArgs& a, int i, const int (&ix)[6]) {
  const int d = a.d;
  const int sp = ix[0], op = ix[1], pp = ix[2], sn = ix[3], on = ix[4], pn = ix[5];
  float es[KM], eo[KM], rp[KM], fs[KM], fo[KM], rn[KM];
  load_row<KM>(a.E, sp, d, es);
  load_row<KM>(a.R, pp, d, rp);
  load_row<KM>(a.E, op, d, eo);
  load_row<KM>(a.E, sn, d, fs);
  load_row<KM>(a.R, pn, d, rn);
  load_row<KM>(a.E, on, d, fo);
  float ps = 0.0f, ns = 0.0f, gp[KM], gn[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const float vp = (es[k] + rp[k]) - eo[k];  // score: E[s] + R[p] - E[o]  (transe.py:32)
    const float vn = (fs[k] + rn[k]) - fo[k];
    ps += L1 ? fabsf(vp) : vp * vp;
    ns += L1 ? fabsf(vn) : vn * vn;
    const float tp = (eo[k] - rp[k]) - es[k];  // pg = E[op] - R[pp] - E[sp]  (transe.py:103)
    const float tn = (fo[k] - rn[k]) - fs[k];  // ng = E[on] - R[pn] - E[sn]
    gp[k] = L1 ? signf_np(-tp) : -tp;          // transe.py:115 / 120
    gn[k] = L1 ? signf_np(tn) : tn;            // transe.py:117 / 121
  }
  const float pscore = -wave_sum(ps);
  const float nscore = -wave_sum(ns);
  if (lane_id() == 0) {
    if (a.pscore) a.pscore[i] = pscore;
    if (a.nscore) a.nscore[i] = nscore;
  }
  const bool viol = nscore + a.margin > pscore;  // strict >  (transe.py:73)
  if (!viol) return false;
  float ngp[KM], ngn[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    ngp[k] = -gp[k];
    ngn[k] = -gn[k];
  }
  // entity rows (sp, op, sn, on) -> (+gp, -gp, +gn, -gn)   (transe.py:128-136)
  acc_two<KM>(a.accE, sp, gp, sn, gn, d);
  acc_two<KM>(a.accE, op, ngp, on, ngn, d);
  // relation rows (pp, pn) -> (gp, gn)                      (transe.py:158-160)
  acc_two<KM>(replica(a.accR, i), pp, gp, pn, gn, d);
  return true;
}

// ---------------------------------------------------------------------------
// HolE pair: skge/hole.py:44-100
// ---------------------------------------------------------------------------
template <int KM>
__device__ __forceinline__ bool hole_pair(const PairArgs& a, int i, float* sw, const int (&ix)[6]) {
  const int d = a.d;
  const int sp = ix[0], op = ix[1], pp = ix[2], sn = ix[3], on = ix[4], pn = ix[5];
  const int stride = 64 * KM;
  float* sEs = sw;
  float* sEo = sw + stride;
  float* sRp = sw + 2 * stride;
  float* sFs = sw + 3 * stride;
  float* sFo = sw + 4 * stride;
  float* sRn = sw + 5 * stride;
  float v[KM], rp[KM], rn[KM];
  load_row<KM>(a.E, sp, d, v);
  to_lds<KM>(sEs, v, d);
  load_row<KM>(a.E, op, d, v);
  to_lds<KM>(sEo, v, d);
  load_row<KM>(a.R, pp, d, rp);
  to_lds<KM>(sRp, rp, d);
  load_row<KM>(a.E, sn, d, v);
  to_lds<KM>(sFs, v, d);
  load_row<KM>(a.E, on, d, v);
  to_lds<KM>(sFo, v, d);
  load_row<KM>(a.R, pn, d, rn);
  to_lds<KM>(sRn, rn, d);
  __builtin_amdgcn_wave_barrier();
  float cp[KM], cn[KM];
  ccorr_lds<KM>(sEs, sEo, d, cp);  // ccorr(E[s], E[o])   (hole.py:20)
  ccorr_lds<KM>(sFs, sFo, d, cn);
  float ps = 0.0f, ns = 0.0f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    ps += rp[k] * cp[k];
    ns += rn[k] * cn[k];
  }
  const float praw = wave_sum(ps), nraw = wave_sum(ns);
  if (lane_id() == 0) {
    if (a.pscore) a.pscore[i] = praw;
    if (a.nscore) a.nscore[i] = nraw;
  }
  const float pf = af_f(a.af, praw), nf = af_f(a.af, nraw);
  const bool viol = nf + a.margin > pf;  // hole.py:56
  if (!viol) {
    __builtin_amdgcn_wave_barrier();
    return false;
  }
  const float gp = -af_g_given_f(a.af, pf);  // hole.py:66
  const float gn = af_g_given_f(a.af, nf);   // hole.py:67
  float x[KM], y[KM], t[KM];
  // relation rows (pp, pn): (gp ccorr(E[sp],E[op]), gn ccorr(E[sn],E[on]))  hole.py:76-82
  scale<KM>(x, cp, gp);
  scale<KM>(y, cn, gn);
  acc_two<KM>(replica(a.accR, i), pp, x, pn, y, d);
  // entity rows (sp, sn): gp ccorr(R[pp],E[op]), gn ccorr(R[pn],E[on])   hole.py:93-94
  ccorr_lds<KM>(sRp, sEo, d, t);
  scale<KM>(x, t, gp);
  ccorr_lds<KM>(sRn, sFo, d, t);
  scale<KM>(y, t, gn);
  acc_two<KM>(a.accE, sp, x, sn, y, d);
  // entity rows (op, on): gp cconv(E[sp],R[pp]), gn cconv(E[sn],R[pn])    hole.py:95-96
  cconv_lds<KM>(sEs, sRp, d, t);
  scale<KM>(x, t, gp);
  cconv_lds<KM>(sFs, sRn, d, t);
  scale<KM>(y, t, gn);
  acc_two<KM>(a.accE, op, x, on, y, d);
  __builtin_amdgcn_wave_barrier();
  return true;
}

// HolE pair with the register-tiled correlations (hole_fast(d)); the steps of
// hole_pair with the scores taken as E[s] . ccorr(R[p], E[o]) (hole_score_q,
// the same value as R[p] . ccorr(E[s], E[o]) in exact arithmetic), so the
// sp / sn gradient rows come with the scores; LDS per wave:
// hole_fast_lds_floats(d)
template <int KM>
__device__ __forceinline__ bool hole_pair_fast(const PairArgs& a, int i, float* sw,
                                               const int (&ix)[6]) {
  const int d = a.d;
  const int sp = ix[0], op = ix[1], pp = ix[2], sn = ix[3], on = ix[4], pn = ix[5];
  float* sEs = sw;               // a operands (d + 4): E[sp], E[sn], reversed copies
  float* sFs = sw + d + 4;
  float* rEs = sw + 2 * d + 8;
  float* rFs = sw + 3 * d + 12;
  float* sRp = sw + 4 * d + 16;  // doubled rows (2d + 4)
  float* sRn = sRp + 2 * d + 4;
  float* sEo = sRn + 2 * d + 4;
  float* sFo = sEo + 2 * d + 4;
  float* sout = sFo + 2 * d + 4;
  float es[KM], eo[KM], fs[KM], fo[KM], rp[KM], rn[KM];
  load_row<KM>(a.E, sp, d, es);
  load_row<KM>(a.E, op, d, eo);
  load_row<KM>(a.R, pp, d, rp);
  load_row<KM>(a.E, sn, d, fs);
  load_row<KM>(a.E, on, d, fo);
  load_row<KM>(a.R, pn, d, rn);
  to_lds_a<KM>(sEs, es, d);
  to_lds_a<KM>(sFs, fs, d);
  to_lds_rev<KM>(rEs, es, d);
  to_lds_rev<KM>(rFs, fs, d);
  to_lds_dbl<KM>(sRp, rp, d);
  to_lds_dbl<KM>(sRn, rn, d);
  to_lds_dbl<KM>(sEo, eo, d);
  to_lds_dbl<KM>(sFo, fo, d);
  __builtin_amdgcn_wave_barrier();
  // scores R . ccorr(E[s], E[o]) (hole.py:20) as E[s] . ccorr(R[p], E[o])
  // (hole_score_q): the correlations are the E[sp] / E[sn] gradient rows
  float ap[KM], an[KM];
  float4 qap, qan;
  corr_fast<KM>(sRp, sEo, sout, d, ap, &qap);
  corr_fast<KM>(sRn, sFo, sout, d, an, &qan);
  const int base = 4 * lane_id();
  const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  const float4 qes = base < d ? *reinterpret_cast<const float4*>(sEs + base) : z4;
  const float4 qfs = base < d ? *reinterpret_cast<const float4*>(sFs + base) : z4;
  const float praw = hole_score_q(qes, qap), nraw = hole_score_q(qfs, qan);
  if (lane_id() == 0) {
    if (a.pscore) a.pscore[i] = praw;
    if (a.nscore) a.nscore[i] = nraw;
  }
  const float pf = af_f(a.af, praw), nf = af_f(a.af, nraw);
  const bool viol = nf + a.margin > pf;  // hole.py:56
  if (!viol) {
    __builtin_amdgcn_wave_barrier();
    return false;
  }
  const float gp = -af_g_given_f(a.af, pf);  // hole.py:66
  const float gn = af_g_given_f(a.af, nf);   // hole.py:67
  float x[KM], y[KM], t[KM];
  // relation rows (pp, pn): (gp ccorr(E[sp],E[op]), gn ccorr(E[sn],E[on]))  hole.py:76-82
  corr_fast<KM>(sEs, sEo, sout, d, t);
  scale<KM>(x, t, gp);
  corr_fast<KM>(sFs, sFo, sout, d, t);
  scale<KM>(y, t, gn);
  acc_two<KM>(replica(a.accR, i), pp, x, pn, y, d);
  // entity rows (sp, sn): gp ccorr(R[pp],E[op]), gn ccorr(R[pn],E[on])   hole.py:93-94
  scale<KM>(x, ap, gp);
  scale<KM>(y, an, gn);
  acc_two<KM>(a.accE, sp, x, sn, y, d);
  // entity rows (op, on): gp cconv(E[sp],R[pp]), gn cconv(E[sn],R[pn])    hole.py:95-96
  corr_fast<KM>(rEs, sRp, sout, d, t);
  scale<KM>(x, t, gp);
  corr_fast<KM>(rFs, sRn, sout, d, t);
  scale<KM>(y, t, gn);
  acc_two<KM>(a.accE, op, x, on, y, d);
  __builtin_amdgcn_wave_barrier();
  return true;
}

// ---------------------------------------------------------------------------
// RESCAL pair: skge/rescal.py:78-139 (entity part; dW in k_rescal_wgrad)
// ---------------------------------------------------------------------------
template <int KM>
__device__ __forceinline__ bool rescal_pair(const PairArgs& a, int i, float* sw, const int (&ix)[6]) {
  const int d = a.d;
  const int sp = ix[0], op = ix[1], pp = ix[2], sn = ix[3], on = ix[4], pn = ix[5];
  const int stride = 64 * KM;
  float* sEs = sw;
  float* sEo = sw + stride;
  float* sFs = sw + 2 * stride;
  float* sFo = sw + 3 * stride;
  float es[KM], fs[KM], v[KM];
  load_row<KM>(a.E, sp, d, es);
  to_lds<KM>(sEs, es, d);
  load_row<KM>(a.E, op, d, v);
  to_lds<KM>(sEo, v, d);
  load_row<KM>(a.E, sn, d, fs);
  to_lds<KM>(sFs, fs, d);
  load_row<KM>(a.E, on, d, v);
  to_lds<KM>(sFo, v, d);
  __builtin_amdgcn_wave_barrier();
  const size_t dd = (size_t)d * d;
  float wep[KM], wen[KM];
  gemv_rows<KM>(a.R + pp * dd, sEo, d, wep);  // WEp = W[pp] E[op]   (rescal.py:261)
  gemv_rows<KM>(a.R + pn * dd, sFo, d, wen);
  float ps = 0.0f, ns = 0.0f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    ps += es[k] * wep[k];
    ns += fs[k] * wen[k];
  }
  const float praw = wave_sum(ps), nraw = wave_sum(ns);
  const float pf = af_f(a.af, praw), nf = af_f(a.af, nraw);
  const float gp = -af_g_given_f(a.af, pf);  // rescal.py:275 (all pairs)
  const float gn = af_g_given_f(a.af, nf);
  if (lane_id() == 0) {
    if (a.pscore) a.pscore[i] = praw;
    if (a.nscore) a.nscore[i] = nraw;
    if (a.coef) {
      a.coef[i] = gp;
      a.coef[a.P + i] = gn;
    }
  }
  const bool viol = nf + a.margin > pf;  // rescal.py:269
  if (!viol) {
    __builtin_amdgcn_wave_barrier();
    return false;
  }
  float x[KM], y[KM], t[KM];
  // (sp, sn) <- (gp WEp, gn WEn)                    rescal.py:299-300
  scale<KM>(x, wep, gp);
  scale<KM>(y, wen, gn);
  acc_two<KM>(a.accE, sp, x, sn, y, d);
  // (op, on) <- (gp EWp, gn EWn), EW = E[s] W[p]     rescal.py:296-301
  gemv_cols<KM>(a.R + pp * dd, sEs, d, t);
  scale<KM>(x, t, gp);
  gemv_cols<KM>(a.R + pn * dd, sFs, d, t);
  scale<KM>(y, t, gn);
  acc_two<KM>(a.accE, op, x, on, y, d);
  __builtin_amdgcn_wave_barrier();
  return true;
}

// E.violations[u] += 1 for each distinct u in {sn, on, sp, op} of a violating
// pair (skge/transe.py:78-83): lane j < 4 takes one entity and counts it
// unless an earlier lane holds the same id
__device__ __forceinline__ void count_entity_violation(int* cnt, const int (&ix)[6]) {
  const int l = lane_id();
  const int sp = ix[0], op = ix[1], sn = ix[3], on = ix[4];
  if (l < 4) {
    const int u = l == 0 ? sn : (l == 1 ? on : (l == 2 ? sp : op));
    const bool dup = (l >= 1 && u == sn) || (l >= 2 && u == on) || (l >= 3 && u == sp);
    if (!dup) atomicAdd(cnt + u, 1);
  }
}

template <int MODEL, int KM>
__global__ __launch_bounds__(256) void k_pair_grad(PairArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wave = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  float* sw = smem + wave * 6 * 64 * KM;
  int nv = 0;
  for (int i = blockIdx.x * wpb + wave; i < a.P; i += gridDim.x * wpb) {
    const int ix[6] = {uni(a.pos[3 * i]), uni(a.pos[3 * i + 1]), uni(a.pos[3 * i + 2]),
                       uni(a.neg[3 * i]), uni(a.neg[3 * i + 1]), uni(a.neg[3 * i + 2])};
    bool v = false;
    if (ix[2] < 0) {   // skipped pair (no negative drawn): no score, no contribution
      if (a.coef && lane_id() == 0) {
        a.coef[i] = 0.0f;
        a.coef[a.P + i] = 0.0f;
      }
    } else if (MODEL == TRANSE_L1)
      v = transe_pair<KM, true>(a, i, ix);
    else if (MODEL == TRANSE_L2)
      v = transe_pair<KM, false>(a, i, ix);
    else if (MODEL == HOLE)
      v = hole_pair<KM>(a, i, sw, ix);
    else
      v = rescal_pair<KM>(a, i, sw, ix);
    const Accum aR = replica(a.accR, i);   // dense relation tables may spread over copies
    if (a.record) commit_pair(a.accE, MODEL == RESCAL ? nullptr : &aR, v, ix, i);
    if ((MODEL == TRANSE_L1 || MODEL == TRANSE_L2) && a.eviol && v)
      count_entity_violation(a.eviol, ix);
    nv += v ? 1 : 0;
  }
  __shared__ int lds_nv;
  if (a.nviol) block_count_add(a.nviol, nv, &lds_nv);   // one atomic per workgroup
}

// HolE pairs with the register-tiled correlations (hole_fast(d)): its own
// kernel, so the generic path's registers do not limit its occupancy
template <int KM>
__global__ __launch_bounds__(256) void k_hole_pair_fast(PairArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wave = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  float* sw = smem + wave * hole_fast_lds_floats(a.d);
  int nv = 0;
  for (int i = blockIdx.x * wpb + wave; i < a.P; i += gridDim.x * wpb) {
    const int ix[6] = {uni(a.pos[3 * i]), uni(a.pos[3 * i + 1]), uni(a.pos[3 * i + 2]),
                       uni(a.neg[3 * i]), uni(a.neg[3 * i + 1]), uni(a.neg[3 * i + 2])};
    const bool v = ix[2] >= 0 && hole_pair_fast<KM>(a, i, sw, ix);   // p < 0: skipped pair
    const Accum aR = replica(a.accR, i);
    if (a.record) commit_pair(a.accE, &aR, v, ix, i);
    nv += v ? 1 : 0;
  }
  __shared__ int lds_nv;
  if (a.nviol) block_count_add(a.nviol, nv, &lds_nv);   // one atomic per workgroup
}

// HolE pair in the frequency domain (skge_hole_fft.h): the six rows E[sp],
// E[op], R[pp], E[sn], E[on], R[pn] are transformed together; the scores are
// Hermitian sums (1/d) sum_k conj(E^s_k R^_k) E^o_k, and a violating pair's six
// contribution rows of hole.py:76-96 -- relation gp conj(E^s) E^o, subject
// gp conj(R^) E^o, object gp E^s R^ (and the negative's with gn) -- come from
// six inverse transforms.  LDS per wave: hole_pair_fft_wave_floats(d).
__host__ __device__ __forceinline__ int hole_pair_fft_wave_floats(int d) { return 12 * d; }

template <int KM>
__device__ __forceinline__ bool hole_pair_fft(const PairArgs& a, int i, float* wb,
                                              const float2* tw, const int (&ix)[6]) {
  const int d = a.d, M = d / 2, l = lane_id();
  const int sp = ix[0], op = ix[1], pp = ix[2], sn = ix[3], on = ix[4], pn = ix[5];
  float4 es[1], eo[1], rp[1], fs[1], fo[1], rn[1];
  load_row4<1>(a.E, sp, d, es);
  load_row4<1>(a.E, op, d, eo);
  load_row4<1>(a.R, pp, d, rp);
  load_row4<1>(a.E, sn, d, fs);
  load_row4<1>(a.E, on, d, fo);
  load_row4<1>(a.R, pn, d, rn);
  float2* b0 = reinterpret_cast<float2*>(wb);
  float2* b1 = b0 + 6 * M;
  __builtin_amdgcn_wave_barrier();   // the previous pair's reads of the buffers are done
  fft_put_row(b0, M, 0, rp[0], d);
  fft_put_row(b0, M, 1, es[0], d);
  fft_put_row(b0, M, 2, eo[0], d);
  fft_put_row(b0, M, 3, rn[0], d);
  fft_put_row(b0, M, 4, fs[0], d);
  fft_put_row(b0, M, 5, fo[0], d);
  const float2* Z = M == 100 ? fft_run_c<100, 6, false>(b0, b1, tw)
                             : fft_run<false>(b0, b1, M, 6, tw, d);
  const int k = l;
  const bool on_ = k <= M / 2;
  float2 X[6][2];
  float ps = 0.0f, ns = 0.0f;
  if (on_) {
#pragma unroll
    for (int t = 0; t < 6; ++t) fft_real_pair(Z + t * M, M, k, tw, X[t][0], X[t][1]);
    const float wk = k == 0 ? 1.0f : 2.0f, wm = k == 0 ? 1.0f : (M - k == k ? 0.0f : 2.0f);
    ps = wk * fft_score_term(X[1][0], X[0][0], X[2][0]) + wm * fft_score_term(X[1][1], X[0][1], X[2][1]);
    ns = wk * fft_score_term(X[4][0], X[3][0], X[5][0]) + wm * fft_score_term(X[4][1], X[3][1], X[5][1]);
  }
  const float inv_d = 1.0f / (float)d;
  const float praw = wave_sum(ps) * inv_d, nraw = wave_sum(ns) * inv_d;
  if (l == 0) {
    if (a.pscore) a.pscore[i] = praw;
    if (a.nscore) a.nscore[i] = nraw;
  }
  const float pf = af_f(a.af, praw), nf = af_f(a.af, nraw);
  if (!(nf + a.margin > pf)) return false;   // hole.py:56
  const float gp = -af_g_given_f(a.af, pf);   // hole.py:66
  const float gn = af_g_given_f(a.af, nf);    // hole.py:67
  __builtin_amdgcn_wave_barrier();   // every lane is done reading the forward buffers
  if (on_) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float2 r = X[0][j], e_s = X[1][j], e_o = X[2][j], q = X[3][j], f_s = X[4][j], f_o = X[5][j];
      X[0][j] = cscale(gp, cmulc(e_s, e_o));   // R[pp]: gp ccorr(E[sp], E[op])  hole.py:76-82
      X[1][j] = cscale(gn, cmulc(f_s, f_o));   // R[pn]
      X[2][j] = cscale(gp, cmulc(r, e_o));     // E[sp]: gp ccorr(R[pp], E[op])  hole.py:93-94
      X[3][j] = cscale(gn, cmulc(q, f_o));     // E[sn]
      X[4][j] = cscale(gp, cmul(e_s, r));      // E[op]: gp cconv(E[sp], R[pp]) hole.py:95-96
      X[5][j] = cscale(gn, cmul(f_s, q));      // E[on]
    }
#pragma unroll
    for (int t = 0; t < 6; ++t) fft_real_inv_pair(b0 + t * M, M, k, tw, X[t][0], X[t][1]);
  }
  const float* z = reinterpret_cast<const float*>(
      M == 100 ? fft_run_c<100, 6, true>(b0, b1, tw) : fft_run<true>(b0, b1, M, 6, tw, d));
  const float sc = 2.0f / (float)d;   // 1/M
  float x[KM], y[KM];
  auto rows = [&](int t0) {
#pragma unroll
    for (int kk = 0; kk < KM; ++kk) {
      const int e = l + 64 * kk;
      x[kk] = e < d ? sc * z[t0 * d + e] : 0.0f;
      y[kk] = e < d ? sc * z[(t0 + 1) * d + e] : 0.0f;
    }
  };
  rows(0);
  acc_two<KM>(replica(a.accR, i), pp, x, pn, y, d);
  rows(2);
  acc_two<KM>(a.accE, sp, x, sn, y, d);
  rows(4);
  acc_two<KM>(a.accE, op, x, on, y, d);
  return true;
}

template <int KM>
__global__ __launch_bounds__(256) void k_hole_pair_fft(PairArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wave = threadIdx.x >> 6, wpb = blockDim.x >> 6, d = a.d;
  float2* const tw = reinterpret_cast<float2*>(smem);
  fft_twiddles(tw, a.tw, d);
  __syncthreads();
  float* const wb = smem + 2 * d + wave * hole_pair_fft_wave_floats(d);
  int nv = 0;
  for (int i = blockIdx.x * wpb + wave; i < a.P; i += gridDim.x * wpb) {
    const int ix[6] = {uni(a.pos[3 * i]), uni(a.pos[3 * i + 1]), uni(a.pos[3 * i + 2]),
                       uni(a.neg[3 * i]), uni(a.neg[3 * i + 1]), uni(a.neg[3 * i + 2])};
    const bool v = ix[2] >= 0 && hole_pair_fft<KM>(a, i, wb, tw, ix);   // p < 0: skipped pair
    const Accum aR = replica(a.accR, i);
    if (a.record) commit_pair(a.accE, &aR, v, ix, i);
    nv += v ? 1 : 0;
  }
  __shared__ int lds_nv;
  if (a.nviol) block_count_add(a.nviol, nv, &lds_nv);   // one atomic per workgroup
}

// ---------------------------------------------------------------------------
// HolE pairwise, one positive and BOTH of its pairs per wave (device pair
// loop).  Record j = (s, o, p, s'), o' gives pair 2j = ((s,o,p), (s',o,p)) and
// pair 2j+1 = ((s,o,p), (s,o',p)) (skge/sample.py:41-46, base.py:1411-1416).
// Scores (hole.py:20) through the relation-side correlations (hole_score_q):
//   A = ccorr(R[p], E[o]), B = ccorr(R[p], E[o'])   (one loop, a = R[p])
//   f(s,o,p) = E[s] . A,  f(s',o,p) = E[s'] . A,  f(s,o',p) = E[s] . B
// with k_hole_pair_fast's arithmetic, so the margin decisions (hole.py:56) are
// the pair path's; gp = -g(f(p)), gn = g(f(n)) (hole.py:66-67).  A positive
// with no violating pair is done after these 2 correlations.  Per violating
// pair (v0, v1) the contributions of hole.py:76-96, summed per row, with the
// correlations merged by linearity (u = (v0+v1) gp E[s] + v0 g0 E[s']):
//   E[s] : (v0+v1) gp A + v1 g1 B                 E[s']: g0 A
//   E[o] : cconv(u, R[p])                         E[o']: g1 cconv(E[s], R[p])
//   R[p] : ccorr(u, E[o]) + v1 g1 ccorr(E[s], E[o'])
// = 2 more correlations for v0 alone, 3 for v1 alone, 4 for both (was 7 per
// positive whatever the outcome).  Entity slots 4j..4j+3 name (s, o, s', o')
// with the occurrence counts grad_sum_matrix gives those lists (s: v0 + 2 v1,
// o: 2 v0 + v1, s': v0, o': v1, p: 2 (v0 + v1)), relation slot j names p.
// Rows are held in the quad layout (lane l: elements 4l..4l+3), so d % 4 == 0
// and d <= 256.
// ---------------------------------------------------------------------------
struct HolePosArgs {
  const float* E;
  const float* R;
  Accum accE, accR;
  const int4* rec;   // the epoch's records (s, o, p, s' or -1)
  const int* rec_n1; // o' or -1
  long long start;   // this batch: positives [start, start + count)
  int count, d, af;
  float margin;
  int* nviol;        // this batch's gate word: += violating pairs
  int* fold;         // the previous batch's gate word: added to *total, then cleared
  int* total;
  const float2* tw;  // FFT form: the twiddle table (hole_fft_table)
};

template <int KM, bool FFT>
__global__ __launch_bounds__(256) void k_hole_pos(HolePosArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wave = threadIdx.x >> 6, wpb = blockDim.x >> 6, l = lane_id();
  const int d = a.d;
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.fold) {
    if (a.total) *a.total += *a.fold;
    *a.fold = 0;
  }
  // FFT: the workgroup's twiddle table, then per wave two transform buffers
  float2* const tw = reinterpret_cast<float2*>(smem);
  if constexpr (FFT) {
    fft_twiddles(tw, a.tw, d);
    __syncthreads();
  }
  float* const wb = FFT ? smem + 2 * d + wave * hole_fft_wave_floats(d) : nullptr;
  const HolePosLds L(FFT ? smem : smem + wave * hole_pos_lds_floats(d), d);
  int nv = 0;
  for (int j = blockIdx.x * wpb + wave; j < a.count; j += gridDim.x * wpb) {
    const int4 r4 = a.rec[a.start + j];
    const int s = uni(r4.x), o = uni(r4.y), p = uni(r4.z), neg0 = uni(r4.w);
    const int neg1 = uni(a.rec_n1[a.start + j]);
    const int n0r = neg0 >= 0 ? neg0 : s, n1r = neg1 >= 0 ? neg1 : o;
    float4 es[1], eo[1], rp[1], fs[1], fo[1];
    load_row4<1>(a.E, s, d, es);
    load_row4<1>(a.E, o, d, eo);
    load_row4<1>(a.R, p, d, rp);
    load_row4<1>(a.E, n0r, d, fs);
    load_row4<1>(a.E, n1r, d, fo);
    float praw, raw0, raw1;
    float4 A = {}, B = {};
    HoleSpec hs;
    if constexpr (FFT) {
      hs = hole_fft_forward(wb, tw, d, rp[0], es[0], fs[0], eo[0], fo[0], praw, raw0, raw1);
    } else {
      q_lds_dbl(L.R2, rp[0], d);
      q_lds_dbl(L.O2, eo[0], d);
      q_lds_dbl(L.Q2, fo[0], d);
      __builtin_amdgcn_wave_barrier();
      float4 AB[2];
      {
        const float* const b2[2] = {L.O2, L.Q2};
        corr_quad_b<2>(L.R2, b2, d, AB);
      }
      A = AB[0];
      B = AB[1];
      praw = hole_score_q(es[0], A);
      raw0 = hole_score_q(fs[0], A);
      raw1 = hole_score_q(es[0], B);
    }
    const float pf = af_f(a.af, praw), f0 = af_f(a.af, raw0), f1 = af_f(a.af, raw1);
    const int v0 = uni((neg0 >= 0 && f0 + a.margin > pf) ? 1 : 0);   // hole.py:56
    const int v1 = uni((neg1 >= 0 && f1 + a.margin > pf) ? 1 : 0);
    const Accum aR = replica(a.accR, j);
    if (l < 4)
      commit_slot(a.accE, sel4(l, s, o, neg0, neg1), sel4(l, v0 + 2 * v1, 2 * v0 + v1, v0, v1),
                  4 * j + l);
    else if (l == 4)
      commit_slot(aR, p, 2 * (v0 + v1), j);
    if (v0 + v1 == 0) continue;
    nv += v0 + v1;
    const float gp = -af_g_given_f(a.af, pf);   // hole.py:66
    const float g0 = af_g_given_f(a.af, f0), g1 = af_g_given_f(a.af, f1);   // hole.py:67
    if constexpr (FFT) {
      const float* z = hole_fft_rows(wb, tw, d, hs, v0, v1, gp, g0, g1);
      acc_fft_row<KM>(aR, p, z, 2, d);
      acc_fft_row<KM>(a.accE, s, z, 0, d);
      acc_fft_row<KM>(a.accE, o, z, 1, d);
      if (v0) acc_fft_row<KM>(a.accE, neg0, z, 3, d);
      if (v1) acc_fft_row<KM>(a.accE, neg1, z, 3 + v0, d);
    } else {
      const HoleRows h = hole_pos_rows(L, d, es[0], fs[0], A, B, v0, v1, gp, g0, g1);
      acc_q<KM>(aR, p, h.cr, d, L.U);
      acc_q<KM>(a.accE, s, h.cs, d, L.U);
      acc_q<KM>(a.accE, o, h.co, d, L.U);
      if (v0) acc_q<KM>(a.accE, neg0, h.c0, d, L.U);
      if (v1) acc_q<KM>(a.accE, neg1, h.cq, d, L.U);
    }
    __builtin_amdgcn_wave_barrier();
  }
  __shared__ int lds_nv;
  block_count_add(a.nviol, nv, &lds_nv);   // one atomic per workgroup
}

const float2* hole_fft_table(int d) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, float2*> tabs;   // (device, d)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  auto it = tabs.find({dev, d});
  if (it != tabs.end()) return it->second;
  std::vector<float2> h(d);
  for (int t = 0; t < d; ++t) {
    const double a = -2.0 * M_PI * (double)t / (double)d;
    h[t] = make_float2((float)std::cos(a), (float)std::sin(a));
  }
  float2* p = nullptr;
  if (hipMalloc(&p, d * sizeof(float2)) != hipSuccess ||
      hipMemcpy(p, h.data(), d * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  tabs[{dev, d}] = p;
  return p;
}

// the frequency-domain form of the per-positive HolE kernels (skge_hole_fft.h)
// where it applies; SKGE_HOLE_DIRECT=1 selects the direct correlations
bool hole_use_fft(int d) {
  const char* e = getenv("SKGE_HOLE_DIRECT");
  return hole_fft_ok(d) && !(e && atoi(e));
}

bool hole_pos_ok(int af, const skge_table_t* ent, const skge_table_t* rel, int d) {
  return af >= 0 && af <= 3 && d % 4 == 0 && d >= 4 && d <= 256 && ent && rel &&
         ent->width == d && rel->width == d &&
         (ent->acc_mode == SKGE_ACC_F32 || ent->acc_mode == SKGE_ACC_FX64) &&
         (rel->acc_mode == SKGE_ACC_F32 || rel->acc_mode == SKGE_ACC_FX64) &&
         ent->acc_replicas <= 1 && ent->acc_sum &&
         ent->acc_cnt && rel->acc_sum && rel->acc_cnt;
}

// one batch of the HolE device pair loop (slots: 4 * count entity, count relation)
int launch_hole_pos(hipStream_t st, int af, const skge_table_t* ent, const skge_table_t* rel,
                    int d, const int4* rec, const int* rec_n1, long long start, int count,
                    float margin, int* nviol, int* fold, int* total) {
  int rc;
  if ((rc = check_table(ent, "ent", true)) || (rc = check_table(rel, "rel", true)) ||
      (rc = check_slots(ent, 4ll * count, "ent")) || (rc = check_slots(rel, count, "rel")))
    return rc;
  SKGE_CHECK_ARG(hole_pos_ok(af, ent, rel, d), "HolE positive kernel: unsupported tables");
  HolePosArgs a = {};
  a.E = ent->param;
  a.R = rel->param;
  a.accE = accum_of(ent);
  a.accR = accum_of(rel);
  a.rec = rec;
  a.rec_n1 = rec_n1;
  a.start = start;
  a.count = count;
  a.d = d;
  a.af = af;
  a.margin = margin;
  a.nviol = nviol;
  a.fold = fold;
  a.total = total;
  const int blocks = std::max(1, std::min((count + 3) / 4, 8192));
  const bool fft = hole_use_fft(d);
  if (fft) {
    a.tw = hole_fft_table(d);
    SKGE_CHECK_ARG(a.tw != nullptr, "HolE FFT twiddle table allocation failed");
  }
  const size_t lds = fft ? hole_fft_lds_bytes(d, 4) : (size_t)4 * hole_pos_lds_floats(d) * sizeof(float);
#define SKGE_HPOS(K)                                                                   \
  if (fft)                                                                             \
    hipLaunchKernelGGL((k_hole_pos<K, true>), dim3(blocks), dim3(256), lds, st, a);    \
  else                                                                                 \
    hipLaunchKernelGGL((k_hole_pos<K, false>), dim3(blocks), dim3(256), lds, st, a);
  switch (km_for(d)) {
    case 1: SKGE_HPOS(1) break;
    case 2: SKGE_HPOS(2) break;
    case 3: SKGE_HPOS(3) break;
    default: SKGE_HPOS(4) break;
  }
#undef SKGE_HPOS
  SKGE_CHECK_LAUNCH("hole positive kernel");
  return SKGE_OK;
}

// ---------------------------------------------------------------------------
// logistic loss: HolE skge/hole.py:22-42, RESCAL skge/rescal.py:37-76
// ---------------------------------------------------------------------------
__device__ __forceinline__ void logistic(float y, float score, float* loss_i, float* fs) {
  const float ysc = y * score;
  *loss_i = fmaxf(-ysc, 0.0f) + log1pf(expf(-fabsf(ysc)));  // logaddexp(0, -ys)
  *fs = -(y * (1.0f / (1.0f + expf(ysc))));                   // -(y * sigmoid(-ys))
}

template <int MODEL, int KM>
__global__ __launch_bounds__(256) void k_triple_grad(PairArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wave = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  const int d = a.d;
  const int stride = 64 * KM;
  const bool fast = MODEL == HOLE && KM <= 4 && hole_fast(d);
  float* sEs = smem + wave * (fast ? hole_fast_lds_floats(d) : 3 * stride);
  float* sEo = sEs + stride;
  float* sRp = sEs + 2 * stride;
  // fast layout: E[s], E[s] reversed (d + 4 each), E[o], R[p] doubled, output row
  float* fEs = sEs;
  float* fEsr = sEs + d + 4;
  float* fEo2 = sEs + 2 * d + 8;
  float* fRp2 = fEo2 + 2 * d + 4;
  float* fout = fRp2 + 2 * d + 4;
  float lsum = 0.0f;
  for (int i = blockIdx.x * wpb + wave; i < a.P; i += gridDim.x * wpb) {
    const int s = uni(a.pos[3 * i]), o = uni(a.pos[3 * i + 1]), p = uni(a.pos[3 * i + 2]);
    const float y = a.ys[i];
    float es[KM], eo[KM], x[KM], t[KM];
    load_row<KM>(a.E, s, d, es);
    load_row<KM>(a.E, o, d, eo);
    float score, li, fs;
    if (MODEL == HOLE && KM <= 4 && fast) {
      float rp[KM], c[KM];
      load_row<KM>(a.R, p, d, rp);
      to_lds_a<KM>(fEs, es, d);
      to_lds_rev<KM>(fEsr, es, d);
      to_lds_dbl<KM>(fEo2, eo, d);
      to_lds_dbl<KM>(fRp2, rp, d);
      __builtin_amdgcn_wave_barrier();
      corr_fast<KM>(fEs, fEo2, fout, d, c);
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < KM; ++k) acc += rp[k] * c[k];
      score = wave_sum(acc);
      logistic(y, score, &li, &fs);
      scale<KM>(x, c, fs);  // R: fs ccorr(E[s],E[o])   hole.py:32
      acc_row<KM>(replica(a.accR, i), p, x, d);
      if (lane_id() == 2) commit_slot(replica(a.accR, i), p, 1, i);
      corr_fast<KM>(fRp2, fEo2, fout, d, t);  // E[s]: fs ccorr(R[p],E[o])
      scale<KM>(x, t, fs);
      corr_fast<KM>(fEsr, fRp2, fout, d, t);  // E[o]: fs cconv(E[s],R[p])
      float yv[KM];
      scale<KM>(yv, t, fs);
      acc_two<KM>(a.accE, s, x, o, yv, d);
    } else if (MODEL == HOLE) {
      to_lds<KM>(sEs, es, d);
      to_lds<KM>(sEo, eo, d);
      float rp[KM], c[KM];
      load_row<KM>(a.R, p, d, rp);
      to_lds<KM>(sRp, rp, d);
      __builtin_amdgcn_wave_barrier();
      ccorr_lds<KM>(sEs, sEo, d, c);
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < KM; ++k) acc += rp[k] * c[k];
      score = wave_sum(acc);
      logistic(y, score, &li, &fs);
      scale<KM>(x, c, fs);  // R: fs ccorr(E[s],E[o])   hole.py:32
      acc_row<KM>(replica(a.accR, i), p, x, d);
      if (lane_id() == 2) commit_slot(replica(a.accR, i), p, 1, i);
      ccorr_lds<KM>(sRp, sEo, d, t);  // E[s]: fs ccorr(R[p],E[o])   hole.py:37
      scale<KM>(x, t, fs);
      cconv_lds<KM>(sEs, sRp, d, t);  // E[o]: fs cconv(E[s],R[p])   hole.py:38
      float yv[KM];
      scale<KM>(yv, t, fs);
      acc_two<KM>(a.accE, s, x, o, yv, d);
    } else {
      to_lds<KM>(sEs, es, d);
      to_lds<KM>(sEo, eo, d);
      __builtin_amdgcn_wave_barrier();
      const size_t dd = (size_t)d * d;
      float we[KM], ew[KM];
      gemv_rows<KM>(a.R + p * dd, sEo, d, we);  // WE = W[p] E[o]
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < KM; ++k) acc += es[k] * we[k];
      score = wave_sum(acc);
      logistic(y, score, &li, &fs);
      gemv_cols<KM>(a.R + p * dd, sEs, d, ew);  // EW = E[s] W[p]
      float yv[KM];
      scale<KM>(x, we, fs);  // rescal.py:238: (fs WE over ss, fs EW over os)
      scale<KM>(yv, ew, fs);
      acc_two<KM>(a.accE, s, x, o, yv, d);
      if (lane_id() == 0 && a.coef) a.coef[i] = fs;
    }
    {
      const int l = lane_id();  // entity occurrences (s, o): slots 2i, 2i+1
      if (l < 2) commit_slot(a.accE, l == 0 ? s : o, s == o ? (l == 0 ? 2 : 0) : 1, 2 * i + l);
    }
    if (lane_id() == 0 && a.pscore) a.pscore[i] = score;
    lsum += li;
    __builtin_amdgcn_wave_barrier();
  }
  __shared__ float lds_loss;
  if (a.loss) block_sum_add(a.loss, lsum, &lds_loss);   // one atomic per workgroup
}

// HolE logistic triples in the frequency domain (skge/hole.py:22-42): the
// rows R[p], E[s], E[o] transformed together; score (1/d) sum_k conj(E^s_k
// R^_k) E^o_k; fs from the logistic loss; the rows R[p] fs conj(E^s) E^o,
// E[s] fs conj(R^) E^o, E[o] fs E^s R^ from three inverse transforms.
// LDS per wave: 6d floats (two buffers of three length-d/2 complex rows).
template <int KM>
__global__ __launch_bounds__(256) void k_hole_triple_fft(PairArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wave = threadIdx.x >> 6, wpb = blockDim.x >> 6, d = a.d, M = d / 2, l = lane_id();
  float2* const tw = reinterpret_cast<float2*>(smem);
  fft_twiddles(tw, a.tw, d);
  __syncthreads();
  float2* const b0 = reinterpret_cast<float2*>(smem + 2 * d + wave * 6 * d);
  float2* const b1 = b0 + 3 * M;
  float lsum = 0.0f;
  for (int i = blockIdx.x * wpb + wave; i < a.P; i += gridDim.x * wpb) {
    const int s = uni(a.pos[3 * i]), o = uni(a.pos[3 * i + 1]), p = uni(a.pos[3 * i + 2]);
    const float y = a.ys[i];
    float4 es[1], eo[1], rp[1];
    load_row4<1>(a.E, s, d, es);
    load_row4<1>(a.E, o, d, eo);
    load_row4<1>(a.R, p, d, rp);
    __builtin_amdgcn_wave_barrier();   // the previous triple's reads of the buffers are done
    fft_put_row(b0, M, 0, rp[0], d);
    fft_put_row(b0, M, 1, es[0], d);
    fft_put_row(b0, M, 2, eo[0], d);
    const float2* Z = M == 100 ? fft_run_c<100, 3, false>(b0, b1, tw)
                               : fft_run<false>(b0, b1, M, 3, tw, d);
    const int k = l;
    const bool on = k <= M / 2;
    float2 X[3][2];
    float ps = 0.0f;
    if (on) {
#pragma unroll
      for (int t = 0; t < 3; ++t) fft_real_pair(Z + t * M, M, k, tw, X[t][0], X[t][1]);
      const float wk = k == 0 ? 1.0f : 2.0f, wm = k == 0 ? 1.0f : (M - k == k ? 0.0f : 2.0f);
      ps = wk * fft_score_term(X[1][0], X[0][0], X[2][0]) + wm * fft_score_term(X[1][1], X[0][1], X[2][1]);
    }
    const float score = wave_sum(ps) * (1.0f / (float)d);   // hole.py:20
    float li, fs;
    logistic(y, score, &li, &fs);
    __builtin_amdgcn_wave_barrier();   // every lane is done reading the forward buffers
    if (on) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float2 r = X[0][j], e_s = X[1][j], e_o = X[2][j];
        X[0][j] = cscale(fs, cmulc(e_s, e_o));   // R[p]: fs ccorr(E[s], E[o])   hole.py:32
        X[1][j] = cscale(fs, cmulc(r, e_o));     // E[s]: fs ccorr(R[p], E[o])   hole.py:37
        X[2][j] = cscale(fs, cmul(e_s, r));      // E[o]: fs cconv(E[s], R[p])   hole.py:38
      }
#pragma unroll
      for (int t = 0; t < 3; ++t) fft_real_inv_pair(b0 + t * M, M, k, tw, X[t][0], X[t][1]);
    }
    const float* z = reinterpret_cast<const float*>(
        M == 100 ? fft_run_c<100, 3, true>(b0, b1, tw) : fft_run<true>(b0, b1, M, 3, tw, d));
    const float sc = 2.0f / (float)d;   // 1/M
    float x[KM], yv[KM];
#pragma unroll
    for (int kk = 0; kk < KM; ++kk) {
      const int e = l + 64 * kk;
      x[kk] = e < d ? sc * z[e] : 0.0f;
    }
    acc_row<KM>(replica(a.accR, i), p, x, d);
    if (l == 2) commit_slot(replica(a.accR, i), p, 1, i);
#pragma unroll
    for (int kk = 0; kk < KM; ++kk) {
      const int e = l + 64 * kk;
      x[kk] = e < d ? sc * z[d + e] : 0.0f;
      yv[kk] = e < d ? sc * z[2 * d + e] : 0.0f;
    }
    acc_two<KM>(a.accE, s, x, o, yv, d);
    if (l < 2) commit_slot(a.accE, l == 0 ? s : o, s == o ? (l == 0 ? 2 : 0) : 1, 2 * i + l);
    if (l == 0 && a.pscore) a.pscore[i] = score;
    lsum += li;
  }
  __shared__ float lds_loss;
  if (a.loss) block_sum_add(a.loss, lsum, &lds_loss);   // one atomic per workgroup
}

// ---------------------------------------------------------------------------
// RESCAL dW: acc[p] = sum_i coef_i outer(E[s_i], E[o_i]) over the items with
// relation p (skge/rescal.py:61-70, 113-125).  One 256-thread workgroup owns
// one 64x64 tile of one relation's d x d gradient, so the tile is written
// with plain stores (no atomics).  Items are compacted per 256-item chunk.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_rescal_wgrad(const float* __restrict__ E, Accum accW,
                                                      int d, const int* ta, const float* ca,
                                                      int na, const int* tb, const float* cb,
                                                      int nb) {
  const int nt = (d + 63) / 64;
  const int tiles = nt * nt;
  const int p = blockIdx.x / tiles;
  const int tt = blockIdx.x - p * tiles;
  const int ti = tt / nt, tj = tt - (tt / nt) * nt;
  __shared__ int s_items[256];
  __shared__ float s_coef[256];
  __shared__ int s_n;
  __shared__ float s_es[16][64];
  __shared__ float s_eo[16][64];
  const int t = threadIdx.x;
  const int r0 = (t >> 4) * 4, c0 = (t & 15) * 4;
  float acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = 0.0f;
  int total = 0;
  for (int list = 0; list < 2; ++list) {
    const int* tr = list ? tb : ta;
    const float* cf = list ? cb : ca;
    const int n = list ? nb : na;
    if (tr == nullptr) continue;
    for (int base = 0; base < n; base += 256) {
      if (t == 0) s_n = 0;
      __syncthreads();
      const int it = base + t;
      if (it < n && tr[3 * it + 2] == p) {
        const int slot = atomicAdd(&s_n, 1);
        s_items[slot] = it;
        s_coef[slot] = cf[it];
      }
      __syncthreads();
      const int m = s_n;
      total += m;
      for (int m0 = 0; m0 < m; m0 += 16) {
        for (int q = t; q < 16 * 64; q += 256) {
          const int mi = q >> 6, c = q & 63;
          float vs = 0.0f, vo = 0.0f;
          if (m0 + mi < m) {
            const int it2 = s_items[m0 + mi];
            const int s = tr[3 * it2], o = tr[3 * it2 + 1];
            const int rr = ti * 64 + c, cc = tj * 64 + c;
            if (rr < d) vs = E[(size_t)s * d + rr] * s_coef[m0 + mi];
            if (cc < d) vo = E[(size_t)o * d + cc];
          }
          s_es[mi][c] = vs;
          s_eo[mi][c] = vo;
        }
        __syncthreads();
        const int mm = min(16, m - m0);
        for (int mi = 0; mi < mm; ++mi) {
          float a4[4], b4[4];
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            a4[x] = s_es[mi][r0 + x];
            b4[x] = s_eo[mi][c0 + x];
          }
#pragma unroll
          for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y) acc[x][y] = fmaf(a4[x], b4[y], acc[x][y]);
        }
        __syncthreads();
      }
    }
  }
  if (tt == 0 && t == 0 && accW.touched) accW.touched[p] = total > 0 ? p : -1;   // slot p
  if (total == 0) return;
  float* out = accW.sum + (size_t)p * d * d;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      const int r = ti * 64 + r0 + x, c = tj * 64 + c0 + y;
      if (r < d && c < d) out[(size_t)r * d + c] = acc[x][y];
    }
  if (tt == 0 && t == 0) accW.cnt[p] = total;
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
template <int MODEL>
static int launch_pair(const PairArgs& a, int km, hipStream_t st, bool logistic_mode) {
  const int threads = 256;
  int blocks = (a.P + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  size_t lds = (MODEL == TRANSE_L1 || MODEL == TRANSE_L2) ? 0 : (size_t)4 * 6 * 64 * km * 4;
  const bool hfast = MODEL == HOLE && km <= 4 && (a.d & 3) == 0 && a.d >= 4 && a.d <= 256;
  if (hfast) lds = std::max(lds, (size_t)4 * hole_fast_lds_floats(a.d) * 4);
  if (hfast && logistic_mode && hole_use_fft(a.d)) {
    PairArgs af = a;
    af.tw = hole_fft_table(a.d);
    SKGE_CHECK_ARG(af.tw != nullptr, "HolE FFT twiddle table allocation failed");
    const size_t flds = (size_t)(2 * a.d + 4 * 6 * a.d) * sizeof(float);
    switch (km) {
      case 1: hipLaunchKernelGGL((k_hole_triple_fft<1>), dim3(blocks), dim3(threads), flds, st, af); break;
      case 2: hipLaunchKernelGGL((k_hole_triple_fft<2>), dim3(blocks), dim3(threads), flds, st, af); break;
      case 3: hipLaunchKernelGGL((k_hole_triple_fft<3>), dim3(blocks), dim3(threads), flds, st, af); break;
      default: hipLaunchKernelGGL((k_hole_triple_fft<4>), dim3(blocks), dim3(threads), flds, st, af); break;
    }
    SKGE_CHECK_LAUNCH("hole fft triple launch");
    return SKGE_OK;
  }
  if (hfast && !logistic_mode && hole_use_fft(a.d) && a.record) {
    PairArgs af = a;
    af.tw = hole_fft_table(a.d);
    SKGE_CHECK_ARG(af.tw != nullptr, "HolE FFT twiddle table allocation failed");
    const size_t flds = (size_t)(2 * a.d + 4 * hole_pair_fft_wave_floats(a.d)) * sizeof(float);
    switch (km) {
      case 1: hipLaunchKernelGGL((k_hole_pair_fft<1>), dim3(blocks), dim3(threads), flds, st, af); break;
      case 2: hipLaunchKernelGGL((k_hole_pair_fft<2>), dim3(blocks), dim3(threads), flds, st, af); break;
      case 3: hipLaunchKernelGGL((k_hole_pair_fft<3>), dim3(blocks), dim3(threads), flds, st, af); break;
      default: hipLaunchKernelGGL((k_hole_pair_fft<4>), dim3(blocks), dim3(threads), flds, st, af); break;
    }
    SKGE_CHECK_LAUNCH("hole fft pair launch");
    return SKGE_OK;
  }
  if (hfast && !logistic_mode) {
    switch (km) {
      case 1: hipLaunchKernelGGL((k_hole_pair_fast<1>), dim3(blocks), dim3(threads), lds, st, a); break;
      case 2: hipLaunchKernelGGL((k_hole_pair_fast<2>), dim3(blocks), dim3(threads), lds, st, a); break;
      case 3: hipLaunchKernelGGL((k_hole_pair_fast<3>), dim3(blocks), dim3(threads), lds, st, a); break;
      default: hipLaunchKernelGGL((k_hole_pair_fast<4>), dim3(blocks), dim3(threads), lds, st, a); break;
    }
    SKGE_CHECK_LAUNCH("hole fast pair launch");
    return SKGE_OK;
  }
#define SKGE_LP(K)                                                                             \
  case K:                                                                                      \
    if (logistic_mode)                                                                         \
      hipLaunchKernelGGL((k_triple_grad<MODEL, K>), dim3(blocks), dim3(threads), lds, st, a); \
    else                                                                                       \
      hipLaunchKernelGGL((k_pair_grad<MODEL, K>), dim3(blocks), dim3(threads), lds, st, a);   \
    break;
  switch (km) {
    SKGE_LP(1)
    SKGE_LP(2)
    SKGE_LP(3)
    SKGE_LP(4)
    SKGE_LP(8)
    SKGE_LP(16)
    default:
      set_error("unsupported d");
      return SKGE_ENOTSUP;
  }
#undef SKGE_LP
  SKGE_CHECK_LAUNCH("pair/triple grad launch");
  return SKGE_OK;
}

}  // namespace skge

using namespace skge;

extern "C" int skge_abi_version(void) { return SKGE_ABI_VERSION; }
extern "C" const char* skge_last_error(void) { return skge::g_err; }

static int check_model_tables(int model, const skge_table_t* ent, const skge_table_t* rel, int d) {
  int rc;
  if ((rc = check_table(ent, "ent", true)) != SKGE_OK) return rc;
  if ((rc = check_table(rel, "rel", model != SKGE_RESCAL)) != SKGE_OK) return rc;
  if ((rc = check_f32(ent, "ent")) || (rc = check_f32(rel, "rel"))) return rc;
  // a dense TransE / HolE relation table may hold several accumulator copies
  // (contributions of pair i go to copy i mod replicas; the apply folds them)
  if ((rc = check_single(ent, "ent")) ||
      (model == SKGE_RESCAL && (rc = check_single(rel, "rel"))))
    return rc;
  SKGE_CHECK_ARG(model >= 0 && model <= 3, "unknown model %d", model);
  SKGE_CHECK_ARG(d > 0 && ent->width == d, "entity width %d != d %d", ent->width, d);
  if (model == SKGE_RESCAL)
    SKGE_CHECK_ARG(rel->width == d * d, "W width %d != d*d", rel->width);
  else
    SKGE_CHECK_ARG(rel->width == d, "relation width %d != d %d", rel->width, d);
  SKGE_CHECK_ARG(km_for(d) != 0, "d=%d > 1024 unsupported", d);
  return SKGE_OK;
}

extern "C" int skge_pair_grad(void* stream, int model, int af, const skge_table_t* ent,
                              const skge_table_t* rel, int d, const int* pos, const int* neg,
                              int P, float margin, float* pscore, float* nscore, float* coef,
                              int* nviol) {
  int rc = check_model_tables(model, ent, rel, d);
  if (rc) return rc;
  SKGE_CHECK_ARG(P >= 0, "P < 0");
  SKGE_CHECK_ARG(af >= 0 && af <= 3, "unknown activation %d", af);
  if (P == 0) return SKGE_OK;
  SKGE_CHECK_ARG(pos && neg, "pos/neg NULL");
  PairArgs a = {};
  a.E = ent->param;
  a.R = rel->param;
  a.accE = accum_of(ent);
  if (model != SKGE_RESCAL) a.accR = accum_of(rel);
  a.pos = pos;
  a.neg = neg;
  a.P = P;
  a.d = d;
  a.af = af;
  a.margin = margin;
  a.pscore = pscore;
  a.nscore = nscore;
  a.coef = coef;
  a.nviol = nviol;
  a.record = margin == -INFINITY ? 0 : 1;   // -inf margin: score only
  if (a.record) a.eviol = ent->violations;
  if (a.record) {
    if ((rc = check_slots(ent, 4ll * P, "ent"))) return rc;
    if (model != SKGE_RESCAL && (rc = check_slots(rel, 2ll * P, "rel"))) return rc;
  }
  const int km = km_for(d);
  hipStream_t st = as_stream(stream);
  switch (model) {
    case SKGE_TRANSE_L1: return launch_pair<TRANSE_L1>(a, km, st, false);
    case SKGE_TRANSE_L2: return launch_pair<TRANSE_L2>(a, km, st, false);
    case SKGE_HOLE: return launch_pair<HOLE>(a, km, st, false);
    default: return launch_pair<RESCAL>(a, km, st, false);
  }
}

extern "C" int skge_triple_grad(void* stream, int model, const skge_table_t* ent,
                                const skge_table_t* rel, int d, const int* trip, const float* ys,
                                int T, float* score, float* coef, float* loss) {
  int rc = check_model_tables(model, ent, rel, d);
  if (rc) return rc;
  SKGE_CHECK_ARG(model == SKGE_HOLE || model == SKGE_RESCAL,
                 "logistic loss is defined for HolE and RESCAL only");
  SKGE_CHECK_ARG(T >= 0, "T < 0");
  if (T == 0) return SKGE_OK;
  SKGE_CHECK_ARG(trip && ys, "trip/ys NULL");
  PairArgs a = {};
  a.E = ent->param;
  a.R = rel->param;
  a.accE = accum_of(ent);
  if (model != SKGE_RESCAL) a.accR = accum_of(rel);
  a.pos = trip;
  a.ys = ys;
  a.P = T;
  a.d = d;
  a.pscore = score;
  a.coef = coef;
  a.loss = loss;
  a.record = 1;
  if ((rc = check_slots(ent, 2ll * T, "ent"))) return rc;
  if (model == SKGE_HOLE && (rc = check_slots(rel, T, "rel"))) return rc;
  const int km = km_for(d);
  hipStream_t st = as_stream(stream);
  if (model == SKGE_HOLE) return launch_pair<HOLE>(a, km, st, true);
  return launch_pair<RESCAL>(a, km, st, true);
}

extern "C" int skge_rescal_wgrad(void* stream, const skge_table_t* ent, const skge_table_t* rel,
                                 int d, const int* trip_a, const float* coef_a, int n_a,
                                 const int* trip_b, const float* coef_b, int n_b) {
  int rc = check_model_tables(SKGE_RESCAL, ent, rel, d);
  if (rc) return rc;
  SKGE_CHECK_ARG(rel->acc_sum && rel->acc_cnt, "W accumulator missing");
  if ((rc = check_slots(rel, rel->rows, "W"))) return rc;
  SKGE_CHECK_ARG(n_a >= 0 && n_b >= 0, "negative item count");
  if (n_a + n_b == 0) return SKGE_OK;
  const int nt = (d + 63) / 64;
  const long long blocks = (long long)rel->rows * nt * nt;
  SKGE_CHECK_ARG(blocks < (1ll << 31), "too many relation tiles");
  hipLaunchKernelGGL(k_rescal_wgrad, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                     ent->param, accum_of(rel), d, trip_a, coef_a, n_a, trip_b, coef_b, n_b);
  SKGE_CHECK_LAUNCH("rescal wgrad launch");
  return SKGE_OK;
}
