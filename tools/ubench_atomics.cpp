// Atomic-scatter microbenchmarks at the WN18 batch geometry (gfx950):
// 1414 waves, each adding 5 rows of d=200 into a 40943-row table, as
//   f32   : 200 x global_atomic_add_f32 per row (4 instructions of 64 lanes)
//   u64   : 50 x global_atomic_add_u64 per row (packed int16x4; 1 instruction)
// with the 5th row going to one of `nrel` hot rows (relation contention) or
// to a random row.  Prints us per launch inside a hipGraph of 100 launches.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_atomics.cpp -o tools/ubench_atomics
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int D = 200, N = 40943, NW = 1414;

__device__ inline unsigned hsh(unsigned x) { x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16; return x; }

template <bool U64, int ROWS>
__global__ __launch_bounds__(256) void k_scatter(float* accf, unsigned long long* accu, float* hotf,
                                                 unsigned long long* hotu, int nrel, unsigned salt) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (w >= NW) return;
  for (int r = 0; r < ROWS; ++r) {
    const bool hot = nrel > 0 && r == ROWS - 1;
    const int row = hot ? (int)(hsh(w * 8 + r + salt) % nrel) : (int)(hsh(w * 8 + r + salt) % N);
    if (U64) {
      unsigned long long* base = (hot ? hotu : accu) + (size_t)row * (D / 4);
      if (l < D / 4) atomicAdd(base + l, 0x0001000100010001ull);
    } else {
      float* base = (hot ? hotf : accf) + (size_t)row * D;
      for (int k = 0; k < 4; ++k) { int e = l + 64 * k; if (e < D) atomicAdd(base + e, 1.0f); }
    }
  }
}

// fire-and-forget stores of the same shape (for comparison)
__global__ __launch_bounds__(256) void k_store(unsigned long long* accu, unsigned salt) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (w >= NW) return;
  for (int r = 0; r < 5; ++r) {
    const int row = (int)(hsh(w * 8 + r + salt) % N);
    if (l < D / 4) accu[(size_t)row * (D / 4) + l] = 1ull;
  }
}

__global__ void k_empty() {}

template <typename F>
static void timeit(const char* name, F launch, hipStream_t st, int iters = 100) {
  hipGraph_t g; hipGraphExec_t ge;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < iters; ++i) launch(i);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st)); CK(hipStreamSynchronize(st));
  CK(hipEventRecord(a, st));
  CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  printf("%-44s %7.2f us/launch\n", name, 1e3f * ms / iters);
  CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
}

int main() {
  hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  float *accf, *hotf; unsigned long long *accu, *hotu;
  CK(hipMalloc(&accf, (size_t)N * D * 4)); CK(hipMalloc(&accu, (size_t)N * D * 2));
  CK(hipMalloc(&hotf, 1 << 20)); CK(hipMalloc(&hotu, 1 << 20));
  CK(hipMemset(accf, 0, (size_t)N * D * 4)); CK(hipMemset(accu, 0, (size_t)N * D * 2));
  CK(hipMemset(hotf, 0, 1 << 20)); CK(hipMemset(hotu, 0, 1 << 20));
  const int blocks = (NW + 3) / 4;
  timeit("empty", [&](int) { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, st); }, st);
  timeit("store u64 5 rows", [&](int i) { hipLaunchKernelGGL(k_store, dim3(blocks), dim3(256), 0, st, accu, (unsigned)i); }, st);
  for (int nrel : {0, 18, 1, 64, 1024}) {
    char nm[128];
    snprintf(nm, sizeof nm, "f32 5 rows, hot rows %d", nrel);
    timeit(nm, [&](int i) { hipLaunchKernelGGL((k_scatter<false, 5>), dim3(blocks), dim3(256), 0, st, accf, accu, hotf, hotu, nrel, (unsigned)i); }, st);
    snprintf(nm, sizeof nm, "u64 5 rows, hot rows %d", nrel);
    timeit(nm, [&](int i) { hipLaunchKernelGGL((k_scatter<true, 5>), dim3(blocks), dim3(256), 0, st, accf, accu, hotf, hotu, nrel, (unsigned)i); }, st);
  }
  timeit("u64 4 rows (no relation row)", [&](int i) { hipLaunchKernelGGL((k_scatter<true, 4>), dim3(blocks), dim3(256), 0, st, accf, accu, hotf, hotu, 0, (unsigned)i); }, st);
  timeit("u64 1 row hot 18", [&](int i) { hipLaunchKernelGGL((k_scatter<true, 1>), dim3(blocks), dim3(256), 0, st, accf, accu, hotf, hotu, 18, (unsigned)i); }, st);
  timeit("f32 1 row hot 18", [&](int i) { hipLaunchKernelGGL((k_scatter<false, 1>), dim3(blocks), dim3(256), 0, st, accf, accu, hotf, hotu, 18, (unsigned)i); }, st);
  return 0;
}
