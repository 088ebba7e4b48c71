// Measured gather / scatter roofline (report the path against
// "(ii) a measured gather+RMW-scatter roofline: a microbenchmark that
// gathers/updates random 4d-byte rows from a table of the same size").
//
// One launch moves the same algorithmic bytes as one launch of the training
// kernels, with none of their dependencies (no sampler, no margin test, no
// count claims, no cross-workgroup hand-off):
//   * n_rmw waves (dispatched first, like the pipelined runner's apply role)
//     each read a random row of P, A (fp32) and S (packed sums, 2 B / element)
//     and write all three back -- the 20d bytes of an applied row;
//   * n_gather waves each gather rows_per_wave random rows of P (4d bytes
//     each, 16-byte lanes) and add atom_rows_per_wave rows of 64-bit atomics
//     into S (2d bytes each) -- the scoring role's row traffic.
// Measurement only: not part of the training path.
#include "skge_host.h"

namespace skge {

struct RoofArgs {
  float* P;
  float* A;
  unsigned long long* S;
  int rows, d, n_gather, rows_per_wave, atom_rows, n_rmw;
  uint32_t salt;
  unsigned long long addend;   // 0 at run time (kept opaque to the compiler)
  float* out;
};

template <int KQ>
__global__ __launch_bounds__(256) void k_roofline(RoofArgs a) {
  const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int l = lane_id(), d = a.d, nq = d >> 2;
  if (w < a.n_rmw) {
    const int row = (int)(fmix32((uint32_t)w * 0x9E3779B1u ^ a.salt) % (uint32_t)a.rows);
    float4* p = reinterpret_cast<float4*>(a.P + (size_t)row * d);
    float4* s = reinterpret_cast<float4*>(a.A + (size_t)row * d);
    unsigned long long* q = a.S + (size_t)row * nq;
    float4 pv[KQ], av[KQ];
    unsigned long long sv[KQ];
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      const int i = 64 * m + l, ic = i < nq ? i : nq - 1;
      pv[m] = p[ic];
      av[m] = s[ic];
      sv[m] = q[ic];
    }
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      const int i = 64 * m + l;
      if (i < nq) {
        p[i] = pv[m];
        s[i] = av[m];
        q[i] = sv[m] + a.addend;
      }
    }
    return;
  }
  const int g = w - a.n_rmw;
  if (g >= a.n_gather) return;
  float acc = 0.0f;
  for (int r = 0; r < a.rows_per_wave; ++r) {
    const int row =
        (int)(fmix32((uint32_t)(g * 8 + r) * 0x85EBCA77u ^ a.salt) % (uint32_t)a.rows);
    float4 v[KQ];
    load_row4<KQ>(a.P, row, d, v);
#pragma unroll
    for (int m = 0; m < KQ; ++m) acc += (v[m].x + v[m].y) + (v[m].z + v[m].w);
  }
  acc = wave_sum(acc);
  for (int r = 0; r < a.atom_rows; ++r) {
    const int row =
        (int)(fmix32((uint32_t)(g * 8 + r) * 0x27D4EB2Fu ^ a.salt ^ 0x5bd1e995u) % (uint32_t)a.rows);
    unsigned long long* q = a.S + (size_t)row * nq;
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      const int i = 64 * m + l;
      if (i < nq) atomicAdd(q + i, a.addend);
    }
  }
  if (l == 0) a.out[g] = acc;
}

}  // namespace skge

using namespace skge;

extern "C" int skge_roofline_gather(void* stream, float* P, float* A, void* S, int rows, int d,
                                    int n_gather, int rows_per_wave, int atom_rows_per_wave,
                                    int n_rmw, uint32_t salt, float* out) {
  SKGE_CHECK_ARG(P && A && S && out, "NULL argument");
  SKGE_CHECK_ARG(rows > 0 && d > 0 && d % 4 == 0 && d <= 1024, "bad table shape");
  SKGE_CHECK_ARG(n_gather >= 0 && n_rmw >= 0 && rows_per_wave >= 0 && atom_rows_per_wave >= 0 &&
                     rows_per_wave <= 8 && atom_rows_per_wave <= 8,
                 "bad geometry");
  RoofArgs a{P, A, (unsigned long long*)S, rows, d, n_gather, rows_per_wave, atom_rows_per_wave,
             n_rmw, salt, 0ull, out};
  const long long waves = (long long)n_gather + n_rmw;
  if (waves == 0) return SKGE_OK;
  const int blocks = (int)((waves + 3) / 4);
  const int kq = (d / 4 + 63) / 64;
  hipStream_t st = as_stream(stream);
  if (kq <= 1) hipLaunchKernelGGL((k_roofline<1>), dim3(blocks), dim3(256), 0, st, a);
  else if (kq <= 2) hipLaunchKernelGGL((k_roofline<2>), dim3(blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((k_roofline<4>), dim3(blocks), dim3(256), 0, st, a);
  SKGE_CHECK_LAUNCH("roofline");
  return SKGE_OK;
}
