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

// DPP lane moves within 16-lane rows (VALU, no LDS round trip): quad_perm
// [1,0,3,2] (lane ^ 1), [2,3,0,1] (lane ^ 2), row_half_mirror (lane i of an
// 8-lane half takes lane 7 - i), row_mirror (lane i takes 15 - i)
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, true);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, dpp_i<CTRL>(__builtin_bit_cast(int, v)));
}
__device__ __forceinline__ float lane_f(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

// All-reduce over the wave (every lane active): four DPP adds give every lane
// its 16-lane row's sum -- after the quad steps the lanes of a quad hold the
// same value, so the mirrors add the other quad / half exactly like an xor --
// then the four row sums, read with v_readlane, are added as (r0 + r1) +
// (r2 + r3).  Every lane ends with the bitwise-identical sum, so decisions
// taken on it (the margin test) are wave-uniform.
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xb1>(v);
  v += dpp_f<0x4e>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}

__device__ __forceinline__ int wave_sum_int(int v) {
  v += dpp_i<0xb1>(v);
  v += dpp_i<0x4e>(v);
  v += dpp_i<0x141>(v);
  v += dpp_i<0x140>(v);
  return (__builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16)) +
         (__builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48));
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

// The packed (TransE-L1) row updates' AdaGrad step and projection scale in
// the hardware's fast forms (v_sqrt_f32, v_rcp_f32: ~1 ulp instead of the
// correctly rounded sequences).  Their gradients are exact small-integer sums
// over the count (the mean itself stays correctly rounded), so H >= 1/32767
// and the step's relative error stays ~1e-7: far inside the 1e-5 parity bar.
// Shared by every packed apply (row_update, i16_finish): bitwise the same.
__device__ __forceinline__ float adagrad_step_fast(float lr, float g, float a) {
  return (lr * g) * __builtin_amdgcn_rcpf(fmaxf(__builtin_amdgcn_sqrtf(a), 1e-7f));
}
__device__ __forceinline__ float proj_scale_fast(int post, float ss) {
  return __builtin_amdgcn_rcpf(post == POST_NORMALIZE ? __builtin_amdgcn_sqrtf(ss)
                                                      : (ss < 1.0f ? 1.0f : ss));
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
  float* sum;      // fp32 [rows][width], or int64 [rows][width/4] in ACC_I16X4 mode
  int* cnt;
  int* touched;    // nullptr: dense table (no slot records)
  int width;
  int mode;
  int replicas;    // >= 1; copies of sum/cnt, [replicas][rows][...]
  int rows;
  int* err = nullptr;   // ACC_FX64: the device error word (bit 4: a sum wrapped)
};

enum AccMode : int { ACC_F32 = 0, ACC_I16X4 = 1, ACC_I32X2 = 2, ACC_FX64 = 3, ACC_I8X4 = 4 };

// accumulator dwords per row
__device__ __host__ __forceinline__ int acc_row_dwords(int mode, int width) {
  return mode == ACC_I16X4 ? (width >> 1)
                           : (mode == ACC_FX64 ? 2 * width : (mode == ACC_I8X4 ? (width >> 2) : width));
}

// ACC_FX64 (the deterministic reduce mode): a float contribution becomes a
// 64-bit fixed-point integer with 40 fractional bits (one rounding, to the
// nearest multiple of 2^-40 ~ 9.1e-13, deterministic), sums are exact integer
// atomics -- the same bits whatever order the adds arrive in -- and the apply
// converts the sum back once.  Range: |sum| < 2^23 per element and batch,
// i.e. (a row's occurrences in the batch) x max |contribution| < 8.4e6 -- WN18
// RESCAL at nb = 2 (~5e4 pairs of one relation, |E_s E_o| <= 1) stays far
// inside.  Every add is a returned atomic and checks its own signed overflow
// (old and addend of one sign, the result of the other), so any wrap of a
// partial sum sets skge_device_error bit 4 (raised by the runners'
// synchronize()) when it happens; the applies also flag a decoded sum at or
// past 2^22 (half the range).
constexpr float FX_SCALE = 1099511627776.0f;            // 2^40
__device__ __forceinline__ long long fx_enc(float v) { return __float2ll_rn(v * FX_SCALE); }
__device__ __forceinline__ float fx_dec(long long x) {
  return (float)((double)x * (1.0 / 1099511627776.0));
}

// the copy a producer item adds into (dense replicated tables)
__device__ __forceinline__ Accum replica(const Accum& a, long long item) {
  if (a.replicas <= 1) return a;
  Accum r = a;
  const int k = (int)(item % a.replicas);
  const size_t row_dw = (size_t)acc_row_dwords(a.mode, a.width);
  r.sum = a.sum + (size_t)k * a.rows * row_dw;
  r.cnt = a.cnt + (size_t)k * a.rows;
  return r;
}



// Counters many waves add to are sharded over NSHARD words on lines of their
// own: no-return atomics on ONE word serialise at the memory side (~12 ns
// each, MI355X_MICROARCH.md "fanin"), which for ~1.4k adders per launch costs
// more than the launch's real work.
constexpr int NSHARD = 64, SHARD_STRIDE = 32;   // 32 ints = one 128-B line
__device__ __forceinline__ int* shard_of(int* base) {
  const int wave = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  return base + (wave & (NSHARD - 1)) * SHARD_STRIDE;
}

// float version (a loss): one global atomic per workgroup
__device__ __forceinline__ void block_sum_add(float* dst, float v, float* lds_word) {
  if (threadIdx.x == 0) *lds_word = 0.0f;
  __syncthreads();
  if (lane_id() == 0 && v != 0.0f) atomicAdd(lds_word, v);
  __syncthreads();
  if (threadIdx.x == 0 && dst && *lds_word != 0.0f) atomicAdd(dst, *lds_word);
}

// one wave (lanes 0..63): add the shards' total to *dst (if any) and clear them
__device__ __forceinline__ void fold_shards(int* shards, int* dst) {
  const int l = lane_id();
  int v = 0;
  if (l < NSHARD) {
    v = shards[l * SHARD_STRIDE];
    shards[l * SHARD_STRIDE] = 0;
  }
  v = wave_sum_int(v);
  if (l == 0 && dst && v) atomicAdd(dst, v);
}

// workgroup total of a per-wave count, added to *dst with ONE atomic (every
// wave of the workgroup must call it)
__device__ __forceinline__ void block_count_add(int* dst, int v, int* lds_word) {
  if (threadIdx.x == 0) *lds_word = 0;
  __syncthreads();
  if (lane_id() == 0 && v) atomicAdd(lds_word, v);
  __syncthreads();
  if (threadIdx.x == 0 && dst && *lds_word) atomicAdd(dst, *lds_word);
}

// Count `c` occurrences of `row` (no-return atomic) and record the row in
// `slot` (or -1 when c == 0).  Several slots may name the same row; the
// consumer claims each row once with an atomicExch on its count (k_apply).
// Called by one lane per (row, slot): a wave's count atomics all issue at
// once and nothing waits for them.
__device__ __forceinline__ void commit_slot(int* cnt, int* touched, int row, int c, int slot) {
  if (c > 0) atomicAdd(cnt + row, c);
  if (touched) touched[slot] = c > 0 ? row : -1;
}
__device__ __forceinline__ void commit_slot(const Accum& a, int row, int c, int slot) {
  commit_slot(a.cnt, a.touched, row, c, slot);
}

// 32-bit finaliser (murmur3 fmix32): cheap counter-based hashing
__device__ __host__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ int sel4(int l, int a, int b, int c, int d) {
  return l == 0 ? a : (l == 1 ? b : (l == 2 ? c : d));
}

template <int KM>
__device__ __forceinline__ void acc_row(const Accum& a, int row, const float (&v)[KM], int d) {
  const int l = lane_id();
  if (a.mode == ACC_FX64) {   // deterministic: exact fixed-point integer sums
    unsigned long long* base = reinterpret_cast<unsigned long long*>(a.sum) + (size_t)row * a.width;
    bool wrapped = false;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int e = l + 64 * k;
      if (e < d && v[k] != 0.0f) {
        const long long add = fx_enc(v[k]);
        const unsigned long long old = atomicAdd(base + e, (unsigned long long)add);
        const long long res = (long long)(old + (unsigned long long)add);
        wrapped = wrapped || ((((long long)old ^ res) & (add ^ res)) < 0);
      }
    }
    if (wrapped && a.err) atomicOr(a.err, 4);
    return;
  }
  float* base = a.sum + (size_t)row * a.width;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    if (e < d) atomicAdd(base + e, v[k]);
  }
}

template <int KM>
__device__ __forceinline__ void acc_two(const Accum& acc, int a, const float (&x)[KM], int b,
                                        const float (&y)[KM], int d) {
  if (a == b) {
    float t[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) t[k] = x[k] + y[k];
    acc_row<KM>(acc, a, t, d);
  } else {
    acc_row<KM>(acc, a, x, d);
    acc_row<KM>(acc, b, y, d);
  }
}

// Occurrence counts + touched slots of one pair (slot maps: skge_hip.h).
// Entity list (sp, op, sn, on), relation list (pp, pn), each occurrence
// counted once per violating pair, as grad_sum_matrix counts duplicates.
// Lanes 0-3 / 4-5 issue their returning atomics concurrently.
__device__ __forceinline__ void commit_pair(const Accum& aE, const Accum* aR, bool viol,
                                            const int (&ix)[6], int i) {
  const int l = lane_id();
  const int v = viol ? 1 : 0;
  const int sp = ix[0], op = ix[1], pp = ix[2], sn = ix[3], on = ix[4], pn = ix[5];
  int c0 = v, c1 = v, c2 = v, c3 = v;
  if (sp == sn) {
    c0 += c2;
    c2 = 0;
  }
  if (op == on) {
    c1 += c3;
    c3 = 0;
  }
  if (l < 4) {
    commit_slot(aE, sel4(l, sp, op, sn, on), sel4(l, c0, c1, c2, c3), 4 * i + l);
  } else if (aR != nullptr && l < 6) {
    int r0 = v, r1 = v;
    if (pp == pn) {
      r0 += r1;
      r1 = 0;
    }
    commit_slot(*aR, l == 4 ? pp : pn, l == 4 ? r0 : r1, 2 * i + (l - 4));
  }
}


// Row gather.  Lanes past the row end load the row's last element (a valid
// address) and zero it with a select: a conditional load would make hipcc
// branch around each load and wait for it (serialising the gathers).
template <int KM>
__device__ __forceinline__ void load_row(const float* __restrict__ T, int row, int d, float (&v)[KM]) {
  const float* base = T + (size_t)row * d;
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    const float x = base[e < d ? e : d - 1];
    v[k] = e < d ? x : 0.0f;
  }
}

// ---- "quad" row layout (TransE-L1 packed path): lane l holds elements
// 4q .. 4q+3, q = 64m + l, as a float4, m < KQ = ceil(d / 256) (d % 4 == 0):
// a 1 KB row slice is ONE 16-byte-per-lane wave-instruction, and a lane's four
// elements are what one exact int16x4 accumulator qword holds. ----
template <int KQ>
__device__ __forceinline__ void load_row4(const float* __restrict__ T, int row, int d,
                                          float4 (&v)[KQ]) {
  const float4* base = reinterpret_cast<const float4*>(T + (size_t)row * d);
  const int l = lane_id(), nq = d >> 2;
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l;
    const float4 x = base[q < nq ? q : nq - 1];
    v[m] = q < nq ? x : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
}

// four small integers (exactly representable floats) as one int64 whose
// 16-bit fields are added independently by a 64-bit integer add: the fields
// borrow/carry into each other, which the signed decode below undoes exactly
// as long as every field's running total stays within +-32767
__device__ __forceinline__ unsigned long long pack_i16x4(const float4& c) {
  const long long v = (((long long)c.w * 65536 + (long long)c.z) * 65536 + (long long)c.y) * 65536 +
                      (long long)c.x;
  return (unsigned long long)v;
}
__device__ __forceinline__ float4 unpack_i16x4(unsigned long long u) {
  long long x = (long long)u;
  const long long f0 = (short)(x & 0xFFFF);
  x = (x - f0) >> 16;
  const long long f1 = (short)(x & 0xFFFF);
  x = (x - f1) >> 16;
  const long long f2 = (short)(x & 0xFFFF);
  x = (x - f2) >> 16;
  return make_float4((float)f0, (float)f1, (float)f2, (float)x);
}

// four int8 fields per uint32 (the same carry/borrow scheme, 8-bit fields): a
// TransE-L1 entity row whose per-batch count is <= 127 has every field total
// within +-127, so the wrapped 32-bit sum read as int32 is the exact packed
// sum -- half the atomic and accumulator bytes of int16x4
__device__ __forceinline__ unsigned int pack_i8x4_sum(const float4& c) {
  const int v = (((int)c.w * 256 + (int)c.z) * 256 + (int)c.y) * 256 + (int)c.x;
  return (unsigned int)v;
}
__device__ __forceinline__ float4 unpack_i8x4_sum(unsigned int u) {
  int x = (int)u;
  const int f0 = (signed char)(x & 0xFF);
  x = (x - f0) >> 8;
  const int f1 = (signed char)(x & 0xFF);
  x = (x - f1) >> 8;
  const int f2 = (signed char)(x & 0xFF);
  x = (x - f2) >> 8;
  return make_float4((float)f0, (float)f1, (float)f2, (float)x);
}

template <int KQ>
__device__ __forceinline__ void acc_row4_i8(unsigned int* sum, int row, const float4 (&c)[KQ],
                                            int d) {
  unsigned int* base = sum + (size_t)row * (d >> 2);
  const int l = lane_id(), nq = d >> 2;
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l;
    if (q < nq) atomicAdd(base + q, pack_i8x4_sum(c[m]));
  }
}

// two int32 fields per int64 (the same carry/borrow scheme, 32-bit fields):
// the relation rows' sums, which every positive of a batch with that relation
// adds into, so a 16-bit field would bound the batch by the relation's
// frequency; 32-bit fields are exact for any batch below 2^29 positives
__device__ __forceinline__ unsigned long long pack_i32x2(float lo, float hi) {
  return (unsigned long long)((long long)hi * 4294967296ll + (long long)lo);
}
__device__ __forceinline__ float2 unpack_i32x2(unsigned long long u) {
  const long long x = (long long)u;
  const long long f0 = (int)(x & 0xFFFFFFFFll);
  return make_float2((float)f0, (float)((x - f0) >> 32));
}

template <int KQ>
__device__ __forceinline__ void add_row4_i16(unsigned long long* base, const float4 (&c)[KQ],
                                             int d) {
  const int l = lane_id(), nq = d >> 2;
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l;
    if (q < nq) atomicAdd(base + q, pack_i16x4(c[m]));
  }
}
template <int KQ>
__device__ __forceinline__ void acc_row4_i16(const Accum& a, int row, const float4 (&c)[KQ],
                                             int d) {
  add_row4_i16<KQ>(reinterpret_cast<unsigned long long*>(a.sum) + (size_t)row * (d >> 2), c, d);
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
