// Counter-based randomness of the device batch loop: the keyed epoch
// permutation (the stand-in for numpy's shuffle, skge/base.py:1257) and the
// RandomModeSampler draws (skge/sample.py:41-46).
#pragma once
#include "skge_device.h"

namespace skge {

// ---- keyed permutation of [0, T): 4-round Feistel + cycle walking ----
struct Perm {
  uint64_t T;
  int half;
  uint64_t key;
};

// half <= 32, so each half fits 32 bits and the round function is fmix32
__device__ __host__ __forceinline__ uint64_t feistel(uint64_t x, int half, uint64_t key) {
  const uint64_t mask = (1ull << half) - 1;
  uint64_t L = x >> half, R = x & mask;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t kr = (uint32_t)(key >> (16 * r)) ^ (0x9E3779B9u * (uint32_t)(r + 1));
    const uint64_t F = (uint64_t)fmix32((uint32_t)R ^ kr) & mask;
    const uint64_t nL = R;
    R = L ^ F;
    L = nL;
  }
  return (L << half) | R;
}

__device__ __host__ __forceinline__ uint64_t perm_index(uint64_t j, const Perm& pm) {
  uint64_t x = j;
  do {
    x = feistel(x, pm.half, pm.key);
  } while (x >= pm.T);
  return x;
}

inline int perm_half(int64_t T) {
  int bits = 1;
  while ((1ll << bits) < T) ++bits;
  return (bits + 1) / 2;
}

__device__ __forceinline__ uint64_t epoch_perm_key(uint64_t seed, uint64_t ek) {
  return mix64(seed ^ mix64(ek * 0xD6E8FEB86659FD93ull + 1));
}

__device__ __forceinline__ uint64_t epoch_sample_key(uint64_t seed, uint64_t ek) {
  return mix64(mix64(seed + 0xA0761D6478BD642Full) ^ (ek * 0xE7037ED1A0B428DBull));
}

// Counter-based draw `randint(n_ent)` for try `tr` of mode `mode` of global
// positive j in the epoch keyed by skey.
__device__ __forceinline__ int draw(uint64_t skey, long long j, int mode, int tr, int n) {
  uint32_t h = fmix32((uint32_t)j * 0x9E3779B1u ^ (uint32_t)skey);
  h = fmix32(h ^ (uint32_t)(skey >> 32) ^ ((uint32_t)((unsigned long long)j >> 32) * 0x85EBCA77u) ^
             ((uint32_t)mode * 0x27D4EB2Fu + (uint32_t)tr * 0x165667B1u));
  return (int)(((uint64_t)h * (uint32_t)n) >> 32);
}

}  // namespace skge
