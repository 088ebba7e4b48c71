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

// Hand-off latency probe: the pipelined runner's publish / wait form between
// two workgroups (blocks 0 and 1: different XCDs under round-robin placement),
// ping-ponged `rounds` times.  One hop = a 16-B write-through (sc1) payload
// store, a vmcnt(0) drain, an sc1 flag store (publish_row); the other side
// polls the flag with sc1 loads + s_sleep(2) and re-reads the payload with an
// sc1 load (ensure_applied).  Block 0 times the rounds with s_memrealtime
// (10 ns ticks): out[0] = ticks, out[1] = payload mismatches, out[2] = 1 when
// a bounded wait gave up.  Lines: flag 0, flag 1, payload 0, payload 1 at
// 128-B strides.  Measurement only: not part of the training path.
__global__ __launch_bounds__(64) void k_handoff_probe(unsigned* buf, int rounds,
                                                      unsigned long long* out) {
  const int me = blockIdx.x, l = lane_id();
  unsigned* const my_flag = buf + 32 * me;
  unsigned* const peer_flag = buf + 32 * (me ^ 1);
  unsigned* const my_pay = buf + 64 + 32 * me;
  unsigned* const peer_pay = buf + 64 + 32 * (me ^ 1);
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned bad = 0, gave_up = 0;
  for (int i = 0; i < rounds && !gave_up; ++i) {
    const unsigned v = 2u * (unsigned)i + 1u;
    auto wait_for = [&](unsigned want) {
      unsigned spins = 0;
      while (__hip_atomic_load(peer_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 20)) {
          gave_up = 1;
          return;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const unsigned got = __hip_atomic_load(peer_pay + (l & 3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bad += (l < 4 && got != want + (unsigned)l) ? 1u : 0u;
    };
    auto publish = [&]() {
      if (l < 4) __hip_atomic_store(my_pay + l, v + (unsigned)l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (l == 0) __hip_atomic_store(my_flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    if (me == 0) {
      publish();
      wait_for(v);
    } else {
      wait_for(v);
      publish();
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  bad = (unsigned)wave_sum_int((int)bad);
  if (l == 0) {
    if (me == 0) out[0] = t1 - t0;
    atomicAdd(out + 1, (unsigned long long)bad);
    if (gave_up) atomicOr(out + 2, 1ull);
  }
}

}  // namespace skge

using namespace skge;

extern "C" int skge_handoff_probe(void* stream, void* buf, int rounds, uint64_t* out) {
  SKGE_CHECK_ARG(buf && out && rounds > 0 && rounds <= (1 << 20), "bad argument");
  hipStream_t st = as_stream(stream);
  SKGE_CHECK_HIP(hipMemsetAsync(buf, 0, 1024, st));
  SKGE_CHECK_HIP(hipMemsetAsync(out, 0, 3 * sizeof(uint64_t), st));
  hipLaunchKernelGGL(k_handoff_probe, dim3(2), dim3(64), 0, st, (unsigned*)buf, rounds,
                     (unsigned long long*)out);
  SKGE_CHECK_LAUNCH("handoff probe");
  return SKGE_OK;
}

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
