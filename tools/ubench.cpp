// Calibration microbenchmarks for the per-batch kernels' building blocks
// (gfx950).  Build: hipcc -O3 --offload-arch=gfx950 tools/ubench.cpp -o tools/ubench
// Each case is launched back to back (eager and inside one hipGraph) with the
// WN18 batch geometry: 1414 waves (one per positive), 200-float rows, a
// 40943-row table; prints microseconds per launch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int D = 200, N = 40943, KM = 4;

__device__ inline unsigned hsh(unsigned x) { x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16; return x; }

__global__ void k_empty(int n) {}

// persistent grid: `iters` grid-wide barriers (one agent-scope counter, WG
// leaders arrive then poll); bounded spins, err[0] set on timeout
__global__ __launch_bounds__(256) void k_gridbar(unsigned* ctr, int iters, unsigned* err) {
  const unsigned nwg = gridDim.x;
  for (int it = 1; it <= iters; ++it) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      unsigned spins = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < nwg * it) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) { atomicOr(err, 1u); break; }
      }
    }
    __syncthreads();
  }
}

template <int ROWS, bool ATOM, bool CHAIN, bool CNT>
__global__ __launch_bounds__(256) void k_rows(const float* __restrict__ E, float* acc, int* cnt,
                                              const int* __restrict__ idx, float* out, int nw, unsigned salt) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (w >= nw) return;
  int base = w;
  if (CHAIN) base = __builtin_amdgcn_readfirstlane(idx[w]);
  float s = 0.f;
  float v[ROWS][KM];
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    const int row = hsh(base * 8 + r + salt) % N;
#pragma unroll
    for (int k = 0; k < KM; ++k) { int e = l + 64 * k; v[r][k] = e < D ? E[(size_t)row * D + e] : 0.f; }
  }
#pragma unroll
  for (int r = 0; r < ROWS; ++r)
#pragma unroll
    for (int k = 0; k < KM; ++k) s += v[r][k];
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if (ATOM) {
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
      const int row = hsh(base * 8 + r + salt + 77) % N;
#pragma unroll
      for (int k = 0; k < KM; ++k) { int e = l + 64 * k; if (e < D) atomicAdd(acc + (size_t)row * D + e, v[r][k] * 1e-30f); }
    }
  }
  if (CNT && l < ROWS) atomicAdd(cnt + hsh(base * 8 + l + salt + 77) % N, 1);
  if (l == 0) out[w] = s;
}

// apply-like: slot -> row -> read 3 rows, write 3 rows
__global__ __launch_bounds__(256) void k_applylike(float* P, float* A, float* S, const int* __restrict__ slots, int nw) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (w >= nw) return;
  const int row = __builtin_amdgcn_readfirstlane(slots[w]);
  if (row < 0) return;
  float p[KM], a[KM], s[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) { int e = l + 64 * k; size_t o = (size_t)row * D + e;
    p[k] = e < D ? P[o] : 0; a[k] = e < D ? A[o] : 0; s[k] = e < D ? S[o] : 0; }
  float ss = 0;
#pragma unroll
  for (int k = 0; k < KM; ++k) { float g = s[k]; a[k] += g * g; p[k] -= 0.1f * g / fmaxf(sqrtf(a[k]), 1e-7f); ss += p[k] * p[k]; }
  for (int m = 32; m >= 1; m >>= 1) ss += __shfl_xor(ss, m, 64);
  const float inv = 1.0f / sqrtf(ss + 1e-30f);
#pragma unroll
  for (int k = 0; k < KM; ++k) { int e = l + 64 * k; size_t o = (size_t)row * D + e;
    if (e < D) { P[o] = p[k] * inv; A[o] = a[k]; S[o] = 0.f; } }
}

template <typename F>
static void timeit(const char* name, F launch, hipStream_t st, int iters = 200) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 20; ++i) launch();
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(a, st));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  // graph of the same launches
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st)); CK(hipStreamSynchronize(st));
  CK(hipEventRecord(a, st));
  CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms2; CK(hipEventElapsedTime(&ms2, a, b));
  printf("%-34s eager %7.2f us/launch   graph %7.2f us/launch\n", name, 1e3f * ms / iters, 1e3f * ms2 / iters);
  CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
}

int main() {
  hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  float *E, *acc, *out, *P, *A, *S; int *cnt, *idx, *slots;
  const size_t nbytes = (size_t)N * D * 4;
  CK(hipMalloc(&E, nbytes)); CK(hipMalloc(&acc, nbytes)); CK(hipMalloc(&P, nbytes)); CK(hipMalloc(&A, nbytes));
  CK(hipMalloc(&S, nbytes)); CK(hipMalloc(&out, 1 << 20)); CK(hipMalloc(&cnt, N * 4)); CK(hipMalloc(&idx, 1 << 20));
  CK(hipMalloc(&slots, 1 << 20));
  CK(hipMemset(E, 0, nbytes)); CK(hipMemset(acc, 0, nbytes)); CK(hipMemset(P, 0, nbytes));
  CK(hipMemset(A, 0, nbytes)); CK(hipMemset(S, 0, nbytes)); CK(hipMemset(cnt, 0, N * 4));
  std::vector<int> h(1 << 18);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (int)((i * 2654435761u) % 40000);
  CK(hipMemcpy(idx, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  std::vector<int> hs(8192);
  for (int i = 0; i < 8192; ++i) hs[i] = (i % 20 == 0) ? -1 : (int)((i * 2654435761u) % N);
  CK(hipMemcpy(slots, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
  const int nw = 1414, blocks = (nw + 3) / 4;
  unsigned salt = 1;
  timeit("empty 354x256", [&] { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, st, 0); }, st);
  timeit("empty 1x64", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, 0); }, st);
  timeit("gather 5 rows", [&] { hipLaunchKernelGGL((k_rows<5, false, false, false>), dim3(blocks), dim3(256), 0, st, E, acc, cnt, idx, out, nw, salt++); }, st);
  timeit("idx -> gather 5 rows", [&] { hipLaunchKernelGGL((k_rows<5, false, true, false>), dim3(blocks), dim3(256), 0, st, E, acc, cnt, idx, out, nw, salt++); }, st);
  timeit("gather 5 + atomics 5 rows", [&] { hipLaunchKernelGGL((k_rows<5, true, false, false>), dim3(blocks), dim3(256), 0, st, E, acc, cnt, idx, out, nw, salt++); }, st);
  timeit("gather 5 + atomics 5 + cnt", [&] { hipLaunchKernelGGL((k_rows<5, true, false, true>), dim3(blocks), dim3(256), 0, st, E, acc, cnt, idx, out, nw, salt++); }, st);
  timeit("idx -> gather 5 + atomics 5 + cnt", [&] { hipLaunchKernelGGL((k_rows<5, true, true, true>), dim3(blocks), dim3(256), 0, st, E, acc, cnt, idx, out, nw, salt++); }, st);
  timeit("gather 5 + atomics 2 rows", [&] { hipLaunchKernelGGL((k_rows<2, true, false, false>), dim3(blocks), dim3(256), 0, st, E, acc, cnt, idx, out, nw, salt++); }, st);
  const int nws = 5656 + 1414;
  timeit("applylike 7070 waves", [&] { hipLaunchKernelGGL(k_applylike, dim3((nws + 3) / 4), dim3(256), 0, st, P, A, S, slots, nws); }, st);
  timeit("applylike 5656 waves", [&] { hipLaunchKernelGGL(k_applylike, dim3((5656 + 3) / 4), dim3(256), 0, st, P, A, S, slots, 5656); }, st);
  timeit("applylike 1414 waves", [&] { hipLaunchKernelGGL(k_applylike, dim3((1414 + 3) / 4), dim3(256), 0, st, P, A, S, slots, 1414); }, st);
  unsigned *ctr, *err;
  CK(hipMalloc(&ctr, 4)); CK(hipMalloc(&err, 4)); CK(hipMemset(err, 0, 4));
  for (int nwg : {256, 512, 1024}) {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int iters = 200;
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemsetAsync(ctr, 0, 4, st));
      CK(hipEventRecord(e0, st));
      hipLaunchKernelGGL(k_gridbar, dim3(nwg), dim3(256), 0, st, ctr, iters, err);
      CK(hipEventRecord(e1, st)); CK(hipStreamSynchronize(st));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned he; CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
      if (rep) printf("grid barrier %4d WGs x256            %7.2f us/barrier%s\n", nwg, 1e3f * ms / iters, he ? " (TIMEOUT)" : "");
    }
  }
  return 0;
}
