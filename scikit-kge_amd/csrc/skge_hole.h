// HolE helpers shared by the device pair loop (k_hole_pos, skge_grad.hip) and
// the pipelined HolE runner (skge_pipeline.hip): rows in the quad layout (lane
// l holds elements 4l..4l+3, d % 4 == 0, d <= 256) staged through a
// wave-private LDS region for the direct circular correlations
// (skge/util.py:30-50: ccorr(a,b)_k = sum_j a_j b_{(j+k) mod d}).
#pragma once
#include "skge_device.h"

namespace skge {

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// three doubled rows (2d + 4) and four a operands (d + 4) per wave
__host__ __device__ __forceinline__ int hole_pos_lds_floats(int d) { return 10 * d + 28; }

// a operand (d + 4 floats): a[d..d+3] = a[0..3] for the correlation's last step
__device__ __forceinline__ void q_lds(float* s, const float4& v, int d) {
  const int base = 4 * lane_id();
  if (base < d) *reinterpret_cast<float4*>(s + base) = v;
  if (base == 0) *reinterpret_cast<float4*>(s + d) = v;
}

// doubled row (b operand): s2[e] = s2[e + d] = v_e, 4 zeros after
__device__ __forceinline__ void q_lds_dbl(float* s2, const float4& v, int d) {
  const int l = lane_id(), base = 4 * l;
  if (base < d) {
    *reinterpret_cast<float4*>(s2 + base) = v;
    *reinterpret_cast<float4*>(s2 + base + d) = v;
  }
  if (l < 4) s2[2 * d + l] = 0.0f;
}

// reversed row a'_m = a_{-m mod d}: cconv(a, b) = ccorr(a', b); a'[d] = a'[0]
__device__ __forceinline__ void q_lds_rev(float* s, const float4& v, int d) {
  const int base = 4 * lane_id();
  if (base < d) {
    if (base == 0) s[d] = v.x;
    s[base == 0 ? 0 : d - base] = v.x;
    s[d - base - 1] = v.y;
    s[d - base - 2] = v.z;
    s[d - base - 3] = v.w;
  }
}

// ---- direct circular correlation, quad layout (lane l: outputs 4l..4l+3) ----
// c_k = sum_j a_j b_{(j+k) mod d} (skge/util.py:30-50), b doubled in LDS
// (b2[e] = b2[e + d] = b_e, 4 zeros after), a with a[d] = a[0] (the staging
// helpers below write it).  Each packed FMA pairs two consecutive j of ONE
// output (the two halves are that output's even-j and odd-j partial sums), so
// every b operand is an aligned register pair of the lane's 8-float window
// w = b[4l+j0 .. 4l+j0+7] and no window pair needs a register move:
//   out 4l+0 += {a_j0,a_j0+1}*w01   + {a_j0+2,a_j0+3}*w23
//   out 4l+1 += {a_j0+1,a_j0+2}*w23 + {a_j0+3,a_j0+4}*w45
//   out 4l+2 += {a_j0,a_j0+1}*w23   + {a_j0+2,a_j0+3}*w45
//   out 4l+3 += {a_j0+1,a_j0+2}*w45 + {a_j0+3,a_j0+4}*w67
// The two misaligned a pairs are built once per step and shared by every b.
struct CorrA {
  f2 xy, zw, yz, wx;
};
// A = a[j0 .. j0+3], An = a[j0+4 .. j0+7] (16-B broadcast reads; An is the
// next step's A, and a[d] = a[0] at the last step)
__device__ __forceinline__ CorrA corr_a(const float4& A, const float4& An) {
  return {f2{A.x, A.y}, f2{A.z, A.w}, f2{A.y, A.z}, f2{A.w, An.x}};
}
__device__ __forceinline__ float4 lds4(const float* s) {
  return *reinterpret_cast<const float4*>(s);
}
struct CorrAcc {
  f2 c0, c1, c2, c3;
};
__device__ __forceinline__ void corr_zero(CorrAcc& c) {
  c.c0 = c.c1 = c.c2 = c.c3 = f2{0.0f, 0.0f};
}
__device__ __forceinline__ void corr_step(CorrAcc& c, const CorrA& a, const float4& lo,
                                          const float4& hi) {
  const f2 w01 = {lo.x, lo.y}, w23 = {lo.z, lo.w}, w45 = {hi.x, hi.y}, w67 = {hi.z, hi.w};
  c.c0 = __builtin_elementwise_fma(a.xy, w01, c.c0);
  c.c1 = __builtin_elementwise_fma(a.yz, w23, c.c1);
  c.c2 = __builtin_elementwise_fma(a.xy, w23, c.c2);
  c.c3 = __builtin_elementwise_fma(a.yz, w45, c.c3);
  c.c0 = __builtin_elementwise_fma(a.zw, w23, c.c0);
  c.c1 = __builtin_elementwise_fma(a.wx, w45, c.c1);
  c.c2 = __builtin_elementwise_fma(a.zw, w45, c.c2);
  c.c3 = __builtin_elementwise_fma(a.wx, w67, c.c3);
}
__device__ __forceinline__ float4 corr_out(const CorrAcc& c) {
  return make_float4(c.c0.x + c.c0.y, c.c1.x + c.c1.y, c.c2.x + c.c2.y, c.c3.x + c.c3.y);
}

// NA correlations against one second operand: out[n] = ccorr(sa[n], b)
template <int NA>
__device__ __forceinline__ void corr_quad(const float* const (&sa)[NA], const float* sb2, int d,
                                          float4 (&out)[NA]) {
  const int base = 4 * lane_id();
  CorrAcc c[NA];
#pragma unroll
  for (int n = 0; n < NA; ++n) corr_zero(c[n]);
  if (base < d) {
    float4 lo = lds4(sb2 + base), hi = lds4(sb2 + base + 4), A[NA];
#pragma unroll
    for (int n = 0; n < NA; ++n) A[n] = lds4(sa[n]);
    for (int j0 = 0; j0 < d; j0 += 4) {
      const float4 nx = lds4(sb2 + j0 + 8 + base);
#pragma unroll
      for (int n = 0; n < NA; ++n) {
        const float4 An = lds4(sa[n] + j0 + 4);
        corr_step(c[n], corr_a(A[n], An), lo, hi);
        A[n] = An;
      }
      lo = hi;
      hi = nx;
    }
  }
#pragma unroll
  for (int n = 0; n < NA; ++n) out[n] = corr_out(c[n]);
}

// NB correlations sharing the first operand: out[n] = ccorr(a, b_n)
template <int NB>
__device__ __forceinline__ void corr_quad_b(const float* sa, const float* const (&sb2)[NB], int d,
                                            float4 (&out)[NB]) {
  const int base = 4 * lane_id();
  CorrAcc c[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) corr_zero(c[n]);
  if (base < d) {
    float4 lo[NB], hi[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      lo[n] = *reinterpret_cast<const float4*>(sb2[n] + base);
      hi[n] = *reinterpret_cast<const float4*>(sb2[n] + base + 4);
    }
    float4 A = lds4(sa);
    for (int j0 = 0; j0 < d; j0 += 4) {
      const float4 An = lds4(sa + j0 + 4);
      const CorrA a = corr_a(A, An);
      A = An;
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const float4 nx = *reinterpret_cast<const float4*>(sb2[n] + j0 + 8 + base);
        corr_step(c[n], a, lo[n], hi[n]);
        lo[n] = hi[n];
        hi[n] = nx;
      }
    }
  }
#pragma unroll
  for (int n = 0; n < NB; ++n) out[n] = corr_out(c[n]);
}

// sum of NP correlations, out = sum_n ccorr(a_n, b_n): the relation-row
// contribution of several pairs in one accumulator set
template <int NP>
__device__ __forceinline__ float4 corr_quad_sum(const float* const (&sa)[NP],
                                                const float* const (&sb2)[NP], int d) {
  const int base = 4 * lane_id();
  CorrAcc c;
  corr_zero(c);
  if (base < d) {
    float4 lo[NP], hi[NP];
#pragma unroll
    for (int n = 0; n < NP; ++n) {
      lo[n] = *reinterpret_cast<const float4*>(sb2[n] + base);
      hi[n] = *reinterpret_cast<const float4*>(sb2[n] + base + 4);
    }
    float4 A[NP];
#pragma unroll
    for (int n = 0; n < NP; ++n) A[n] = lds4(sa[n]);
    for (int j0 = 0; j0 < d; j0 += 4) {
#pragma unroll
      for (int n = 0; n < NP; ++n) {
        const float4 nx = lds4(sb2[n] + j0 + 8 + base);
        const float4 An = lds4(sa[n] + j0 + 4);
        corr_step(c, corr_a(A[n], An), lo[n], hi[n]);
        A[n] = An;
        lo[n] = hi[n];
        hi[n] = nx;
      }
    }
  }
  return corr_out(c);
}

// lane partial of a quad-layout dot product (zeros past the row)
__device__ __forceinline__ float dot_quad(const float4& x, const float4& y) {
  return fmaf(x.w, y.w, fmaf(x.z, y.z, fmaf(x.y, y.y, x.x * y.x)));
}

__device__ __forceinline__ float4 axpby4(float a, const float4& x, float b, const float4& y) {
  return make_float4(fmaf(a, x.x, b * y.x), fmaf(a, x.y, b * y.y), fmaf(a, x.z, b * y.z),
                     fmaf(a, x.w, b * y.w));
}
__device__ __forceinline__ float4 scale4(float a, const float4& x) {
  return make_float4(a * x.x, a * x.y, a * x.z, a * x.w);
}

// HolE score through the relation-side correlation:
//   R . ccorr(a, b) = sum_k R_k sum_j a_j b_{j+k} = sum_j a_j ccorr(R, b)_j,
// so a positive and its two negatives are scored from A = ccorr(R[p], E[o])
// and B = ccorr(R[p], E[o']) -- the very rows the E[s] / E[s'] gradients use
// (hole.py:93-94) -- instead of three ccorr(E, E) evaluations.  Every HolE
// pairwise kernel with d % 4 == 0, d <= 256 scores this way, with this
// arithmetic (quad partial, then the wave sum), so their margin decisions agree.
__device__ __forceinline__ float hole_score_q(const float4& a, const float4& Acorr) {
  return wave_sum(dot_quad(a, Acorr));
}

// score R . c with k_hole_pair_fast's arithmetic: lane-strided products
// summed over k, then the wave sum (c staged through the wave's LDS)
template <int KM>
__device__ __forceinline__ float score_q(const float4& c, const float* sR, int d, float* stage) {
  q_lds(stage, c, d);
  __builtin_amdgcn_wave_barrier();
  const int l = lane_id();
  float ps = 0.0f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    const float r = e < d ? sR[e] : 0.0f, x = e < d ? stage[e] : 0.0f;
    ps += r * x;
  }
  __builtin_amdgcn_wave_barrier();
  return wave_sum(ps);
}

// a quad-layout contribution row, re-laid lane-strided through the wave's LDS
// stage so every float-atomic wave-instruction covers contiguous bytes
// (MI355X_MICROARCH.md "Global float atomics": scattered lanes are far slower)
template <int KM>
__device__ __forceinline__ void acc_q(const Accum& acc, int row, const float4& v, int d,
                                      float* stage) {
  q_lds(stage, v, d);
  __builtin_amdgcn_wave_barrier();
  float x[KM];
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    x[k] = e < d ? stage[e] : 0.0f;
  }
  __builtin_amdgcn_wave_barrier();
  acc_row<KM>(acc, row, x, d);
}


// wave-private LDS of the per-positive HolE kernels: three doubled b operands
// (R[p], E[o], E[o']) and four a operands / stages
struct HolePosLds {
  float *R2, *O2, *Q2, *U, *Ur, *Er, *W;
  __device__ HolePosLds(float* w, int d)
      : R2(w), O2(w + 2 * d + 4), Q2(w + 4 * d + 8), U(w + 6 * d + 12), Ur(w + 7 * d + 16),
        Er(w + 8 * d + 20), W(w + 9 * d + 24) {}
};

// The per-positive HolE step after the margin test (v0 + v1 > 0): the violating
// pairs' contribution rows (see above).  The rows (quad layout) and A, B are
// in registers, R[p] / E[o] / E[o'] doubled in L.
struct HoleRows {
  float4 cs, co, c0, cq, cr;
};
__device__ __forceinline__ HoleRows hole_pos_rows(const HolePosLds& L, int d, const float4& es,
                                                  const float4& fs, const float4& A,
                                                  const float4& B, int v0, int v1, float gp,
                                                  float g0, float g1) {
  HoleRows h;
  const float cu = (float)(v0 + v1) * gp, cf = v0 ? g0 : 0.0f;
  const float4 u = axpby4(cu, es, cf, fs);
  q_lds(L.U, u, d);
  q_lds_rev(L.Ur, u, d);
  if (v1) {
    q_lds_rev(L.Er, es, d);
    q_lds(L.W, scale4(g1, es), d);
  }
  __builtin_amdgcn_wave_barrier();
  if (v1) {
    if (v0) {
      const float* const a2[2] = {L.Ur, L.Er};
      float4 cc[2];
      corr_quad<2>(a2, L.R2, d, cc);
      h.co = cc[0];
      h.cq = scale4(g1, cc[1]);
    } else {   // u = gp E[s]: one cconv serves both rows
      const float* const a1[1] = {L.Er};
      float4 cc[1];
      corr_quad<1>(a1, L.R2, d, cc);
      h.co = scale4(gp, cc[0]);
      h.cq = scale4(g1, cc[0]);
    }
    const float* const sa[2] = {L.U, L.W};
    const float* const sb[2] = {L.O2, L.Q2};
    h.cr = corr_quad_sum<2>(sa, sb, d);
  } else {
    const float* const a1[1] = {L.Ur};
    float4 cc[1];
    corr_quad<1>(a1, L.R2, d, cc);
    h.co = cc[0];
    h.cq = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const float* const sa[1] = {L.U};
    const float* const sb[1] = {L.O2};
    h.cr = corr_quad_sum<1>(sa, sb, d);
  }
  const float fv0 = (float)v0, fv1 = (float)v1;
#define SKGE_HC(M)                                         \
  h.cs.M = fv0 * (gp * A.M) + fv1 * (gp * A.M + g1 * B.M); \
  h.c0.M = g0 * A.M;
  SKGE_HC(x)
  SKGE_HC(y)
  SKGE_HC(z)
  SKGE_HC(w)
#undef SKGE_HC
  __builtin_amdgcn_wave_barrier();   // L.U is the atomics' stage after this
  return h;
}


}  // namespace skge
