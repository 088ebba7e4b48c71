// Device-side helpers shared by the skge HIP kernels (gfx950 / CDNA4).
//
// Row layout convention used by every kernel: a wave (64 lanes) owns one
// embedding row of width d; lane l holds elements l, l+64, l+128, ...
// (KM = ceil(d/64) registers).  Each wave-instruction therefore touches 256
// contiguous bytes of a row, which is the full-rate shape both for plain
// loads and for global float atomics (MI355X_MICROARCH.md "Global float
// atomics", row "access shape").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SKGE_WAVE 64

namespace skge {

enum Model : int { TRANSE_L1 = 0, TRANSE_L2 = 1, HOLE = 2, RESCAL = 3 };
enum Act : int { AF_LINEAR = 0, AF_SIGMOID = 1, AF_TANH = 2, AF_RELU = 3 };
enum Opt : int { OPT_SGD = 0, OPT_ADAGRAD = 1 };
enum Post : int { POST_NONE = 0, POST_NORMALIZE = 1, POST_NORMLESS1 = 2 };

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// xor-butterfly all-reduce: every lane ends with the bitwise-identical sum
// (each level adds the same two operands, commutatively), so decisions taken
// on the reduced value (the margin test) are wave-uniform.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// activation functions, skge/actfun.py:13-57
__device__ __forceinline__ float af_f(int af, float x) {
  switch (af) {
    case AF_SIGMOID: return 1.0f / (1.0f + expf(-x));
    case AF_TANH: return tanhf(x);
    case AF_RELU: return fmaxf(0.0f, x);
    default: return x;
  }
}
__device__ __forceinline__ float af_g_given_f(int af, float fx) {
  switch (af) {
    case AF_SIGMOID: return fx * (1.0f - fx);
    case AF_TANH: return 1.0f - fx * fx;
    case AF_RELU: return fx > 0.0f ? 1.0f : 0.0f;
    default: return 1.0f;
  }
}

__device__ __forceinline__ float signf_np(float x) {  // numpy.sign
  return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f);
}

// Segment-sum accumulator for one parameter table (the device form of
// grad_sum_matrix + Sm.dot(G), skge/util.py:53-101): a dense fp32 sum
// [rows][width], an occurrence count per row, and fixed-slot touched records
// (see skge_table_t in include/skge_hip.h).  Invariant between batches:
// sum == 0 and cnt == 0.
struct Accum {
  float* sum;
  int* cnt;
  int* touched;
  int width;
};

// Count `c` occurrences of `row` and record it in `slot` if this was the
// first count of the row in the batch (else -1).  Called by one lane per
// (row, slot); different lanes' calls are independent, so a wave issues all
// its returning atomics at once (one round trip, not one per row).
__device__ __forceinline__ void commit_slot(const Accum& a, int row, int c, int slot) {
  if (c > 0) {
    const int old = atomicAdd(a.cnt + row, c);
    a.touched[slot] = old == 0 ? row : -1;
  } else {
    a.touched[slot] = -1;
  }
}

__device__ __forceinline__ int sel4(int l, int a, int b, int c, int d) {
  return l == 0 ? a : (l == 1 ? b : (l == 2 ? c : d));
}

template <int KM>
__device__ __forceinline__ void acc_row(const Accum& a, int row, const float (&v)[KM], int d) {
  float* base = a.sum + (size_t)row * a.width;
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    if (e < d) atomicAdd(base + e, v[k]);
  }
}

template <int KM>
__device__ __forceinline__ void load_row(const float* __restrict__ T, int row, int d, float (&v)[KM]) {
  const float* base = T + (size_t)row * d;
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    v[k] = e < d ? base[e] : 0.0f;
  }
}

// 64-bit mixing (splitmix64 finaliser) for counter-based random numbers and
// hashing; stateless, so every (key, counter) maps to an independent draw.
__device__ __host__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// uniform integer in [0, n) from 32 random bits (multiply-shift)
__device__ __forceinline__ int rand_below(uint64_t r, int n) {
  return (int)(((r >> 32) * (uint64_t)(uint32_t)n) >> 32);
}

// Set of training triples (s, o, p) for the RandomModeSampler rejection test
// `tuple(nex) not in self.xs` (skge/sample.py:44): open addressing over
// 16-byte slots {s, o, p, tag} (tag 0 = empty), preceded by a one-hash bit
// filter of 8 bits per slot, so a query for a non-member (the common case)
// usually costs one 4-byte load.
struct TripleSet {
  const int4* slots;
  const uint32_t* filter;
  uint64_t mask;   // capacity - 1 (power of two)
  uint64_t fmask;  // filter bits - 1
};

__device__ __host__ __forceinline__ uint64_t triple_hash(int s, int o, int p) {
  return mix64(((uint64_t)(uint32_t)s << 32 | (uint32_t)o) ^ mix64((uint64_t)(uint32_t)p + 0x51ED27ull));
}

__device__ __forceinline__ bool set_contains(const TripleSet& ts, int s, int o, int p) {
  const uint64_t hv = triple_hash(s, o, p);
  const uint64_t bit = (hv >> 29) & ts.fmask;
  if (((ts.filter[bit >> 5] >> (bit & 31)) & 1u) == 0) return false;
  uint64_t h = hv & ts.mask;
  for (uint64_t probe = 0; probe <= ts.mask; ++probe) {
    const int4 v = ts.slots[h];
    if (v.w == 0) return false;
    if (v.x == s && v.y == o && v.z == p) return true;
    h = (h + 1) & ts.mask;
  }
  return false;
}

}  // namespace skge
