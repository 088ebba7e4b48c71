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

__host__ __device__ __forceinline__ int hole_pos_lds_floats(int d) { return 10 * d + 12; }

__device__ __forceinline__ void q_lds(float* s, const float4& v, int d) {
  const int base = 4 * lane_id();
  if (base < d) *reinterpret_cast<float4*>(s + base) = v;
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

// reversed row a'_m = a_{-m mod d}: cconv(a, b) = ccorr(a', b)
__device__ __forceinline__ void q_lds_rev(float* s, const float4& v, int d) {
  const int base = 4 * lane_id();
  if (base < d) {
    s[base == 0 ? 0 : d - base] = v.x;
    s[d - base - 1] = v.y;
    s[d - base - 2] = v.z;
    s[d - base - 3] = v.w;
  }
}

// NA correlations against one second operand: out[n] (quad layout) =
// ccorr(sa[n], b) with b doubled in sb2; per output the FMA sequence of corr_fast
template <int NA>
__device__ __forceinline__ void corr_quad(const float* const (&sa)[NA], const float* sb2, int d,
                                          float4 (&out)[NA]) {
  const int base = 4 * lane_id();
  f2 c01[NA], c23[NA], e01[NA], e23[NA];
#pragma unroll
  for (int n = 0; n < NA; ++n) {
    c01[n] = f2{0.0f, 0.0f};
    c23[n] = f2{0.0f, 0.0f};
    e01[n] = f2{0.0f, 0.0f};
    e23[n] = f2{0.0f, 0.0f};
  }
  if (base < d) {
    float4 lo = *reinterpret_cast<const float4*>(sb2 + base);
    float4 hi = *reinterpret_cast<const float4*>(sb2 + base + 4);
    for (int j0 = 0; j0 < d; j0 += 4) {
      const float4 nx = *reinterpret_cast<const float4*>(sb2 + j0 + 8 + base);
      const f2 w01 = {lo.x, lo.y}, w12 = {lo.y, lo.z}, w23 = {lo.z, lo.w}, w34 = {lo.w, hi.x};
      const f2 w45 = {hi.x, hi.y}, w56 = {hi.y, hi.z};
#pragma unroll
      for (int n = 0; n < NA; ++n) {
        const float4 a = *reinterpret_cast<const float4*>(sa[n] + j0);   // broadcast
        const f2 ax = {a.x, a.x}, ay = {a.y, a.y}, az = {a.z, a.z}, aw = {a.w, a.w};
        c01[n] = __builtin_elementwise_fma(ax, w01, c01[n]);
        c23[n] = __builtin_elementwise_fma(ax, w23, c23[n]);
        e01[n] = __builtin_elementwise_fma(ay, w12, e01[n]);
        e23[n] = __builtin_elementwise_fma(ay, w34, e23[n]);
        c01[n] = __builtin_elementwise_fma(az, w23, c01[n]);
        c23[n] = __builtin_elementwise_fma(az, w45, c23[n]);
        e01[n] = __builtin_elementwise_fma(aw, w34, e01[n]);
        e23[n] = __builtin_elementwise_fma(aw, w56, e23[n]);
      }
      lo = hi;
      hi = nx;
    }
  }
#pragma unroll
  for (int n = 0; n < NA; ++n) {
    const f2 u = c01[n] + e01[n], v = c23[n] + e23[n];
    out[n] = make_float4(u.x, u.y, v.x, v.y);
  }
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


}  // namespace skge
