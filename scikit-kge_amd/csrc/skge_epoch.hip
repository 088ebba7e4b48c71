// Device-resident mini-batch loop for TransE (the throughput path):
//   PairwiseStochasticTrainer._optim / _process_batch (skge/base.py:1242-1291,
//   1394-1427) with RandomModeSampler(1, [0, 1]) (skge/sample.py:28-46).
//
// Differences from the host loop are statistical only: the epoch shuffle is
// a keyed pseudo-random bijection of [0, T) instead of numpy's MT19937
// shuffle, and the sampler draws come from a counter-based generator.  The
// arithmetic per pair is the same as skge_pair_grad's (parity-tested by
// replaying the recorded negatives through the oracle).
#include <algorithm>
#include <vector>

#include "skge_host.h"
#include "skge_sampler.h"

namespace skge {

// ---- triple set build: claim a slot by CAS on the tag, then fill it ----
__global__ void k_set_build(const int* __restrict__ trip, long long T, int4* slots,
                            unsigned long long mask, uint32_t* filter, unsigned long long fmask) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < T;
       i += (long long)gridDim.x * blockDim.x) {
    const int s = trip[3 * i], o = trip[3 * i + 1], p = trip[3 * i + 2];
    const uint64_t hv = triple_hash(s, o, p);
    const uint64_t bit = (hv >> 29) & fmask;
    atomicOr(&filter[bit >> 5], 1u << (bit & 31));
    uint64_t h = hv & mask;
    for (uint64_t probe = 0; probe <= mask; ++probe) {
      if (atomicCAS(&slots[h].w, 0, 1) == 0) {
        slots[h].x = s;
        slots[h].y = o;
        slots[h].z = p;
        break;
      }
      h = (h + 1) & mask;
    }
  }
}

struct SampleArgs {
  const float* E;
  const float* R;
  Accum accE, accR;
  const int* trip;
  long long T;
  TripleSet set;
  long long start;
  int count, d, n_ent, ntries, half;
  uint64_t seed;
  const uint64_t* epoch_key;
  float margin;
  int* nviol;
  int* nviol_total;
  int* vshards;   // runner: violations go to these shards (folded at the epoch end), not nviol_total
  int* neg_out;
};

// a wave's violation count: sharded (runner) or one atomic per workgroup
__device__ __forceinline__ void count_violations(const SampleArgs& a, int nv) {
  __shared__ int lds_nv;
  if (a.vshards) {
    if (lane_id() == 0 && nv) atomicAdd(shard_of(a.vshards), nv);
  } else {
    block_count_add(a.nviol_total, nv, &lds_nv);
  }
  if (a.nviol) block_count_add(a.nviol, nv, &lds_nv);
}

// RandomModeSampler._sample (skge/sample.py:41-46), tries first_try.. for the
// modes still unresolved: lanes 0-3 try mode 0 (corrupt s), lanes 4-7 mode 1
// (corrupt o), four tries per mode per round; the lowest accepted try wins,
// as in the sequential loop.
__device__ __forceinline__ void sample_rest(const SampleArgs& a, uint64_t skey, long long j, int s,
                                        int o, int p, int first_try, int& neg0, int& neg1) {
  const int l = lane_id();
  for (int round = 0; first_try + round * 4 < a.ntries; ++round) {
    const int mode = (l >> 2) & 1;
    const int tr = first_try + round * 4 + (l & 3);
    const bool want = mode == 0 ? neg0 < 0 : neg1 < 0;
    const bool active = l < 8 && tr < a.ntries && want;
    int c = 0;
    bool ok = false;
    if (active) {
      c = draw(skey, j, mode, tr, a.n_ent);
      ok = mode == 0 ? !set_contains(a.set, c, o, p) : !set_contains(a.set, s, c, p);
    }
    const uint64_t m0 = __ballot(active && ok && mode == 0);
    const uint64_t m1 = __ballot(active && ok && mode == 1);
    if (m0) neg0 = __shfl(c, __ffsll((unsigned long long)m0) - 1, 64);
    if (m1) neg1 = __shfl(c, __ffsll((unsigned long long)m1) - 1, 64);
    if (neg0 >= 0 && neg1 >= 0) break;
  }
}

template <int KM, bool L1>
__global__ __launch_bounds__(256) void k_transe_sample_grad(SampleArgs a) {
  const int wpb = blockDim.x >> 6;
  const int l = lane_id();
  const int d = a.d;
  const uint64_t ek = *a.epoch_key;
  const Perm pm = {(uint64_t)a.T, a.half, epoch_perm_key(a.seed, ek)};
  const uint64_t skey = epoch_sample_key(a.seed, ek);
  int nv = 0;
  for (int w = blockIdx.x * wpb + (threadIdx.x >> 6); w < a.count; w += gridDim.x * wpb) {
    const long long j = a.start + w;
    const long long t = (long long)perm_index((uint64_t)j, pm);
    // first tries of both modes do not depend on the positive: load their rows
    // speculatively, in the same memory round trip as the triple itself
    const int cand0 = draw(skey, j, 0, 0, a.n_ent), cand1 = draw(skey, j, 1, 0, a.n_ent);
    float fs[KM], fo[KM];
    load_row<KM>(a.E, cand0, d, fs);
    load_row<KM>(a.E, cand1, d, fo);
    const int s = __builtin_amdgcn_readfirstlane(a.trip[3 * t]);
    const int o = __builtin_amdgcn_readfirstlane(a.trip[3 * t + 1]);
    const int p = __builtin_amdgcn_readfirstlane(a.trip[3 * t + 2]);
    float es[KM], eo[KM], rp[KM];
    load_row<KM>(a.E, s, d, es);
    load_row<KM>(a.E, o, d, eo);
    load_row<KM>(a.R, p, d, rp);
    // rejection test of the first tries (lane 0: (cand0, o, p), lane 1: (s, cand1, p))
    bool ok = true;
    if (l < 2) ok = l == 0 ? !set_contains(a.set, cand0, o, p) : !set_contains(a.set, s, cand1, p);
    const uint64_t okm = __ballot(ok);
    int neg0 = (okm & 1ull) ? cand0 : -1;
    int neg1 = (okm & 2ull) ? cand1 : -1;
    if (neg0 < 0 || neg1 < 0) {   // rare: a first draw hit a training triple
      sample_rest(a, skey, j, s, o, p, 1, neg0, neg1);
      neg0 = __builtin_amdgcn_readfirstlane(neg0);
      neg1 = __builtin_amdgcn_readfirstlane(neg1);
      if (neg0 >= 0 && neg0 != cand0) load_row<KM>(a.E, neg0, d, fs);
      if (neg1 >= 0 && neg1 != cand1) load_row<KM>(a.E, neg1, d, fo);
    }
    float ps = 0.0f, n0 = 0.0f, n1 = 0.0f, gp[KM], g0[KM], g1[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const float vp = (es[k] + rp[k]) - eo[k];
      const float v0 = (fs[k] + rp[k]) - eo[k];  // pair 0: (s', o, p)
      const float v1 = (es[k] + rp[k]) - fo[k];  // pair 1: (s, o', p)
      ps += L1 ? fabsf(vp) : vp * vp;
      n0 += L1 ? fabsf(v0) : v0 * v0;
      n1 += L1 ? fabsf(v1) : v1 * v1;
      const float tp = (eo[k] - rp[k]) - es[k];  // transe.py:103
      const float t0 = (eo[k] - rp[k]) - fs[k];  // transe.py:104 for pair 0
      const float t1 = (fo[k] - rp[k]) - es[k];  // ... for pair 1
      gp[k] = L1 ? signf_np(-tp) : -tp;
      g0[k] = L1 ? signf_np(t0) : t0;
      g1[k] = L1 ? signf_np(t1) : t1;
    }
    const float pscore = -wave_sum(ps);
    const float ns0 = -wave_sum(n0), ns1 = -wave_sum(n1);
    const int v0 = (neg0 >= 0 && ns0 + a.margin > pscore) ? 1 : 0;
    const int v1 = (neg1 >= 0 && ns1 + a.margin > pscore) ? 1 : 0;
    if (a.neg_out && l == 0) {
      a.neg_out[2 * (long long)w] = neg0;
      a.neg_out[2 * (long long)w + 1] = neg1;
    }
    {
      // occurrence counts + touched slots (entity slots 4w+{s,o,s',o'}, relation slot w):
      // pair 0 lists (sp,op,sn,on) = (s,o,s',o), pair 1 = (s,o,s,o')
      const int cE = sel4(l, v0 + 2 * v1, 2 * v0 + v1, v0, v1);
      const int rE = sel4(l, s, o, neg0, neg1);
      const Accum aR = replica(a.accR, j);
      if (l < 5) {
        const bool ent = l < 4;
        commit_slot(ent ? a.accE.cnt : aR.cnt, ent ? a.accE.touched : aR.touched,
                    ent ? rE : p, ent ? cE : 2 * (v0 + v1), ent ? 4 * w + l : w);
      }
    }
    if (v0 + v1 == 0) continue;
    nv += v0 + v1;
    const float fv0 = (float)v0, fv1 = (float)v1;
    float cs[KM], co[KM], c0[KM], c1[KM], cr[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      // pair 0 rows (sp,op,sn,on) = (s,o,s',o): (+gp,-gp,+g0,-g0)
      // pair 1 rows (sp,op,sn,on) = (s,o,s,o'): (+gp,-gp,+g1,-g1)
      cs[k] = fv0 * gp[k] + fv1 * (gp[k] + g1[k]);
      co[k] = -(fv0 * (gp[k] + g0[k]) + fv1 * gp[k]);
      c0[k] = g0[k];
      c1[k] = -g1[k];
      cr[k] = fv0 * (gp[k] + g0[k]) + fv1 * (gp[k] + g1[k]);
    }
    acc_row<KM>(a.accE, s, cs, d);
    acc_row<KM>(a.accE, o, co, d);
    if (v0) acc_row<KM>(a.accE, neg0, c0, d);
    if (v1) acc_row<KM>(a.accE, neg1, c1, d);
    acc_row<KM>(replica(a.accR, j), p, cr, d);
  }
  count_violations(a, nv);
}

// TransE-L1, one positive in the quad row layout: the permuted triple, its
// RandomModeSampler negatives (mode 0 corrupts s, mode 1 corrupts o), the
// three L1 scores, the strict margin tests and the sign sub-gradients of the
// positive (gp) and of both negatives (g0, g1) (skge/transe.py:32-46, 73,
// 103-117).  Shared by the packed two-launch kernel and the data-parallel
// scorer, so both make bitwise the same decisions.
struct PosL1 {
  int s, o, p, neg0, neg1, v0, v1;
};
template <int KQ>
__device__ __forceinline__ PosL1 transe_l1_front(const SampleArgs& a, const Perm& pm,
                                                 uint64_t skey, long long j, float4 (&gp)[KQ],
                                                 float4 (&g0)[KQ], float4 (&g1)[KQ]) {
  const int l = lane_id();
  const int d = a.d;
  const long long t = (long long)perm_index((uint64_t)j, pm);
  // first tries of both modes do not depend on the positive: their rows load
  // in the same memory round trip as the triple
  const int cand0 = draw(skey, j, 0, 0, a.n_ent), cand1 = draw(skey, j, 1, 0, a.n_ent);
  float4 fs[KQ], fo[KQ];
  load_row4<KQ>(a.E, cand0, d, fs);
  load_row4<KQ>(a.E, cand1, d, fo);
  PosL1 r;
  r.s = __builtin_amdgcn_readfirstlane(a.trip[3 * t]);
  r.o = __builtin_amdgcn_readfirstlane(a.trip[3 * t + 1]);
  r.p = __builtin_amdgcn_readfirstlane(a.trip[3 * t + 2]);
  const int s = r.s, o = r.o, p = r.p;
  float4 es[KQ], eo[KQ], rp[KQ];
  load_row4<KQ>(a.E, s, d, es);
  load_row4<KQ>(a.E, o, d, eo);
  load_row4<KQ>(a.R, p, d, rp);
  bool ok = true;
  if (l < 2) ok = l == 0 ? !set_contains(a.set, cand0, o, p) : !set_contains(a.set, s, cand1, p);
  const uint64_t okm = __ballot(ok);
  int neg0 = (okm & 1ull) ? cand0 : -1;
  int neg1 = (okm & 2ull) ? cand1 : -1;
  if (neg0 < 0 || neg1 < 0) {   // rare: a first draw hit a training triple
    sample_rest(a, skey, j, s, o, p, 1, neg0, neg1);
    neg0 = __builtin_amdgcn_readfirstlane(neg0);
    neg1 = __builtin_amdgcn_readfirstlane(neg1);
    if (neg0 >= 0 && neg0 != cand0) load_row4<KQ>(a.E, neg0, d, fs);
    if (neg1 >= 0 && neg1 != cand1) load_row4<KQ>(a.E, neg1, d, fo);
  }
  float ps = 0.0f, n0 = 0.0f, n1 = 0.0f;
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
#define SKGE_EL(X)                                                                    \
  {                                                                                   \
    const float vp = (es[m].X + rp[m].X) - eo[m].X;   /* transe.py:32 */              \
    const float v0 = (fs[m].X + rp[m].X) - eo[m].X;                                   \
    const float v1 = (es[m].X + rp[m].X) - fo[m].X;                                   \
    ps += fabsf(vp);                                                                  \
    n0 += fabsf(v0);                                                                  \
    n1 += fabsf(v1);                                                                  \
    gp[m].X = signf_np(-((eo[m].X - rp[m].X) - es[m].X)); /* transe.py:103,115 */     \
    g0[m].X = signf_np((eo[m].X - rp[m].X) - fs[m].X);    /* transe.py:104,117 */     \
    g1[m].X = signf_np((fo[m].X - rp[m].X) - es[m].X);                                \
  }
    SKGE_EL(x)
    SKGE_EL(y)
    SKGE_EL(z)
    SKGE_EL(w)
#undef SKGE_EL
  }
  const float pscore = -wave_sum(ps);
  const float ns0 = -wave_sum(n0), ns1 = -wave_sum(n1);
  r.neg0 = neg0;
  r.neg1 = neg1;
  r.v0 = (neg0 >= 0 && ns0 + a.margin > pscore) ? 1 : 0;   // strict >, transe.py:73
  r.v1 = (neg1 >= 0 && ns1 + a.margin > pscore) ? 1 : 0;
  return r;
}

// One positive's occurrence counts, touched slots (entity slots
// 4w+{s,o,s',o'}, relation slot w) and exact packed contributions:
// pair 0 lists (sp,op,sn,on) = (s,o,s',o), pair 1 = (s,o,s,o')
// (skge/transe.py:128-160 before the segment mean).
template <int KQ>
__device__ __forceinline__ void transe_l1_commit(const SampleArgs& a, long long j, int w,
                                                 const PosL1& r, const float4 (&gp)[KQ],
                                                 const float4 (&g0)[KQ], const float4 (&g1)[KQ]) {
  const int l = lane_id();
  const int d = a.d;
  const int v0 = r.v0, v1 = r.v1;
  {
    const int cE = sel4(l, v0 + 2 * v1, 2 * v0 + v1, v0, v1);
    const int rE = sel4(l, r.s, r.o, r.neg0, r.neg1);
    const Accum aR = replica(a.accR, j);
    if (l < 5) {
      const bool ent = l < 4;
      commit_slot(ent ? a.accE.cnt : aR.cnt, ent ? a.accE.touched : aR.touched,
                  ent ? rE : r.p, ent ? cE : 2 * (v0 + v1), ent ? 4 * w + l : w);
    }
  }
  if (v0 + v1 == 0) return;
  const float fv0 = (float)v0, fv1 = (float)v1;
  float4 cs[KQ], co[KQ], c0[KQ], c1[KQ], cr[KQ];
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
#define SKGE_CO(X)                                                   \
  cs[m].X = fv0 * gp[m].X + fv1 * (gp[m].X + g1[m].X);               \
  co[m].X = -(fv0 * (gp[m].X + g0[m].X) + fv1 * gp[m].X);            \
  c0[m].X = g0[m].X;                                                 \
  c1[m].X = -g1[m].X;                                                \
  cr[m].X = fv0 * (gp[m].X + g0[m].X) + fv1 * (gp[m].X + g1[m].X);
    SKGE_CO(x)
    SKGE_CO(y)
    SKGE_CO(z)
    SKGE_CO(w)
#undef SKGE_CO
  }
  acc_row4_i16<KQ>(a.accE, r.s, cs, d);
  acc_row4_i16<KQ>(a.accE, r.o, co, d);
  if (v0) acc_row4_i16<KQ>(a.accE, r.neg0, c0, d);
  if (v1) acc_row4_i16<KQ>(a.accE, r.neg1, c1, d);
  acc_row4_i16<KQ>(replica(a.accR, j), r.p, cr, d);
}

// TransE-L1 variant with exact packed int16x4 accumulation (ACC_I16X4) and the
// quad row layout: the sign contributions are small integers, so four
// elements share one 64-bit integer atomic, and every row gather / row atomic
// is a single 16-byte-per-lane wave-instruction (d <= 256).
template <int KQ>
__global__ __launch_bounds__(256) void k_transe_l1_sample_grad_i16(SampleArgs a) {
  const int wpb = blockDim.x >> 6;
  const int l = lane_id();
  const uint64_t ek = *a.epoch_key;
  const Perm pm = {(uint64_t)a.T, a.half, epoch_perm_key(a.seed, ek)};
  const uint64_t skey = epoch_sample_key(a.seed, ek);
  int nv = 0;
  for (int w = blockIdx.x * wpb + (threadIdx.x >> 6); w < a.count; w += gridDim.x * wpb) {
    const long long j = a.start + w;
    float4 gp[KQ], g0[KQ], g1[KQ];
    const PosL1 r = transe_l1_front<KQ>(a, pm, skey, j, gp, g0, g1);
    if (a.neg_out && l == 0) {
      a.neg_out[2 * (long long)w] = r.neg0;
      a.neg_out[2 * (long long)w + 1] = r.neg1;
    }
    nv += r.v0 + r.v1;
    transe_l1_commit<KQ>(a, j, w, r, gp, g0, g1);
  }
  count_violations(a, nv);
}

__global__ void k_perm(long long T, int half, uint64_t seed, const uint64_t* ekp, long long* out,
                       long long n) {
  const Perm pm = {(uint64_t)T, half, epoch_perm_key(seed, *ekp)};
  for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += (long long)gridDim.x * blockDim.x)
    out[j] = (long long)perm_index((uint64_t)j, pm);
}

__global__ void k_advance(uint64_t* ek) { *ek += 1; }

// epoch end of the runner: fold the violation shards, advance the key (one wave)
__global__ void k_epoch_end(uint64_t* ek, int* shards, int* nviol_total) {
  fold_shards(shards, nviol_total);
  if (threadIdx.x == 0) *ek += 1;
}

static int launch_sample(const SampleArgs& a, bool l1, hipStream_t st) {
  const int km = km_for(a.d);
  int blocks = (a.count + 3) / 4;
  if (blocks < 1) blocks = 1;
  if (blocks > 16384) blocks = 16384;
  if (a.accE.mode == ACC_I16X4) {
    if (!l1 || a.accR.mode != ACC_I16X4 || (a.d & 3) || a.d > 1024) {
      set_error("packed accumulators need TransE-L1, both tables packed, d %% 4 == 0, "
                "d <= 1024");
      return SKGE_EINVAL;
    }
    const int kq = (a.d / 4 + 63) / 64;
#define SKGE_SP(K) \
  hipLaunchKernelGGL((k_transe_l1_sample_grad_i16<K>), dim3(blocks), dim3(256), 0, st, a)
    if (kq <= 1) SKGE_SP(1);
    else if (kq <= 2) SKGE_SP(2);
    else SKGE_SP(4);
#undef SKGE_SP
    SKGE_CHECK_LAUNCH("transe l1 packed sample grad");
    return SKGE_OK;
  }
  if (a.accR.mode != ACC_F32 && a.accR.mode != ACC_FX64) {
    set_error("mixed accumulator modes");
    return SKGE_EINVAL;
  }
#define SKGE_SG(K)                                                                               \
  case K:                                                                                        \
    if (l1)                                                                                      \
      hipLaunchKernelGGL((k_transe_sample_grad<K, true>), dim3(blocks), dim3(256), 0, st, a);   \
    else                                                                                         \
      hipLaunchKernelGGL((k_transe_sample_grad<K, false>), dim3(blocks), dim3(256), 0, st, a);  \
    break;
  switch (km) {
    SKGE_SG(1)
    SKGE_SG(2)
    SKGE_SG(3)
    SKGE_SG(4)
    SKGE_SG(8)
    SKGE_SG(16)
    default:
      set_error("d=%d unsupported", a.d);
      return SKGE_ENOTSUP;
  }
#undef SKGE_SG
  SKGE_CHECK_LAUNCH("transe sample grad");
  return SKGE_OK;
}

}  // namespace skge

using namespace skge;

extern "C" size_t skge_triple_set_bytes(int64_t capacity) {
  return (size_t)capacity * sizeof(int4) + (size_t)capacity;   // slots + 8 filter bits per slot
}

static TripleSet triple_set_of(const void* set, int64_t capacity) {
  TripleSet ts;
  ts.slots = (const int4*)set;
  ts.filter = (const uint32_t*)((const int4*)set + capacity);
  ts.mask = (uint64_t)(capacity - 1);
  ts.fmask = (uint64_t)(8 * capacity - 1);
  return ts;
}

extern "C" int skge_triple_set_build(void* stream, const int* trip, int64_t T, void* set,
                                     int64_t capacity) {
  SKGE_CHECK_ARG(trip && set, "NULL argument");
  SKGE_CHECK_ARG(capacity >= 4 && (capacity & (capacity - 1)) == 0,
                 "capacity must be a power of 2 >= 4");
  SKGE_CHECK_ARG(capacity >= 2 * T, "capacity must be >= 2*T");
  SKGE_CHECK_ARG(capacity <= (1ll << 32), "capacity too large");
  hipStream_t st = as_stream(stream);
  SKGE_CHECK_HIP(hipMemsetAsync(set, 0, skge_triple_set_bytes(capacity), st));
  if (T == 0) return SKGE_OK;
  long long blocks = (T + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  TripleSet ts = triple_set_of(set, capacity);
  hipLaunchKernelGGL(k_set_build, dim3((unsigned)blocks), dim3(256), 0, st, trip, (long long)T,
                     (int4*)ts.slots, (unsigned long long)ts.mask, (uint32_t*)ts.filter,
                     (unsigned long long)ts.fmask);
  SKGE_CHECK_LAUNCH("triple set build");
  return SKGE_OK;
}

static int fill_sample_args(SampleArgs& a, int l1, const skge_table_t* ent, const skge_table_t* rel,
                            int d, const int* trip, int64_t T, const void* set_slots,
                            int64_t set_capacity, uint64_t seed, const uint64_t* epoch_key,
                            float margin, int ntries, int* nviol, int* nviol_total) {
  int rc;
  if ((rc = check_table(ent, "ent", true))) return rc;
  if ((rc = check_table(rel, "rel", true))) return rc;
  if ((rc = check_single(ent, "ent"))) return rc;
  SKGE_CHECK_ARG(ent->width == d && rel->width == d, "table widths must equal d");
  SKGE_CHECK_ARG(km_for(d) != 0, "d=%d unsupported", d);
  SKGE_CHECK_ARG(trip && set_slots && epoch_key, "NULL argument");
  SKGE_CHECK_ARG(T > 0, "T must be > 0");
  SKGE_CHECK_ARG(set_capacity > 0 && (set_capacity & (set_capacity - 1)) == 0, "bad set capacity");
  SKGE_CHECK_ARG(ntries >= 1, "ntries >= 1");
  a = SampleArgs{};
  a.E = ent->param;
  a.R = rel->param;
  a.accE = accum_of(ent);
  a.accR = accum_of(rel);
  a.trip = trip;
  a.T = T;
  a.set = triple_set_of(set_slots, set_capacity);
  a.d = d;
  a.n_ent = ent->rows;
  a.ntries = ntries;
  a.half = perm_half(T);
  a.seed = seed;
  a.epoch_key = epoch_key;
  a.margin = margin;
  a.nviol = nviol;
  a.nviol_total = nviol_total;
  a.vshards = nullptr;
  (void)l1;
  return SKGE_OK;
}

extern "C" int skge_transe_sample_grad(void* stream, int l1, const skge_table_t* ent,
                                       const skge_table_t* rel, int d, const int* trip, int64_t T,
                                       const void* set_slots, int64_t set_capacity, int64_t start,
                                       int count, uint64_t seed, const uint64_t* epoch_key,
                                       float margin, int ntries, int* nviol, int* nviol_total,
                                       int* neg_out) {
  SampleArgs a;
  int rc = fill_sample_args(a, l1, ent, rel, d, trip, T, set_slots, set_capacity, seed, epoch_key,
                            margin, ntries, nviol, nviol_total);
  if (rc) return rc;
  SKGE_CHECK_ARG(start >= 0 && count >= 0 && start + count <= T, "batch out of range");
  if (count == 0) return SKGE_OK;
  if ((rc = check_slots(ent, 4ll * count, "ent")) || (rc = check_slots(rel, count, "rel")))
    return rc;
  a.start = start;
  a.count = count;
  a.neg_out = neg_out;
  return launch_sample(a, l1 != 0, as_stream(stream));
}

extern "C" int skge_epoch_permutation(void* stream, int64_t T, uint64_t seed,
                                      const uint64_t* epoch_key, int64_t* perm_out, int64_t n) {
  SKGE_CHECK_ARG(T > 0 && n >= 0 && n <= T && perm_out && epoch_key, "bad arguments");
  if (n == 0) return SKGE_OK;
  long long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_perm, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), (long long)T,
                     perm_half(T), seed, epoch_key, (long long*)perm_out, (long long)n);
  SKGE_CHECK_LAUNCH("epoch permutation");
  return SKGE_OK;
}

extern "C" int skge_epoch_advance(void* stream, uint64_t* epoch_key) {
  SKGE_CHECK_ARG(epoch_key, "NULL epoch key");
  hipLaunchKernelGGL(k_advance, dim3(1), dim3(1), 0, as_stream(stream), epoch_key);
  SKGE_CHECK_LAUNCH("epoch advance");
  return SKGE_OK;
}

// ---- native epoch runner: one hipGraph per epoch ----
struct skge_runner {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  int nlaunch = 0;
  int* shards = nullptr;
};

static void runner_free(skge_runner_t* r) {
  if (!r) return;
  if (r->exec) (void)hipGraphExecDestroy(r->exec);
  if (r->graph) (void)hipGraphDestroy(r->graph);
  if (r->shards) (void)hipFree(r->shards);
  delete r;
}

extern "C" skge_runner_t* skge_runner_create(void* stream, int l1, const skge_table_t* ent,
                                             const skge_table_t* rel, int d, const int* trip,
                                             int64_t T, const void* set_slots,
                                             int64_t set_capacity, int nbatches, uint64_t seed,
                                             uint64_t* epoch_key, float margin, int ntries,
                                             int* nviol, int* nviol_total) {
  SampleArgs a;
  if (fill_sample_args(a, l1, ent, rel, d, trip, T, set_slots, set_capacity, seed, epoch_key,
                       margin, ntries, nviol, nviol_total))
    return nullptr;
  if (nbatches < 1 || nbatches > T) {
    set_error("nbatches must be in [1, T]");
    return nullptr;
  }
  if (stream == nullptr) {
    set_error("runner needs a non-default stream (graph capture)");
    return nullptr;
  }
  hipStream_t st = as_stream(stream);
  // batch geometry of StochasticTrainer._optim (skge/base.py:1246-1268)
  const int64_t bs = T / nbatches;
  std::vector<std::pair<int64_t, int64_t>> batches;
  for (int64_t s0 = 0; s0 < T; s0 += bs) batches.push_back({s0, (s0 + bs <= T) ? bs : T - s0});
  skge_runner_t* r = new skge_runner_t();
  skge_table_t tabs[2] = {*ent, *rel};
  if (hipMalloc(&r->shards, NSHARD * SHARD_STRIDE * 4) != hipSuccess ||
      hipMemset(r->shards, 0, NSHARD * SHARD_STRIDE * 4) != hipSuccess) {
    set_error("runner: device allocation failed");
    runner_free(r);
    return nullptr;
  }
  a.vshards = r->shards;
  if (hipStreamSynchronize(st) != hipSuccess ||
      hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    set_error("hipStreamBeginCapture failed");
    runner_free(r);
    return nullptr;
  }
  int rc = SKGE_OK;
  // large batches: when a batch's entity slot records outnumber the table's
  // rows, the entity table is applied densely (one wave per row, claimed as
  // with slots) instead of one wave per slot record -- no duplicate slots whose
  // waves load a row they then lose the claim for.  WN18 d = 200, same box:
  // nb = 2 219 -> 254 M triples/s, nb = 10 203 -> 211 M (tools/large_batch_ab.py;
  // the pipelined runner, the default there, does 605 / 396 M).
  // SKGE_APPLY_DENSE=0: slot records always.
  const char* de = getenv("SKGE_APPLY_DENSE");
  const int dense_mode = de ? atoi(de) : 1;
  for (auto& b : batches) {
    a.start = b.first;
    a.count = (int)b.second;
    a.neg_out = nullptr;
    int ns[2] = {(int)(4 * b.second), (int)b.second};
    if ((rc = check_slots(ent, ns[0], "ent")) || (rc = check_slots(rel, ns[1], "rel"))) break;
    if ((rc = launch_sample(a, l1 != 0, st))) break;
    skge_table_t at[2] = {tabs[0], tabs[1]};
    if (dense_mode > 0 && ns[0] >= ent->rows) {
      at[0].acc_touched = nullptr;
      ns[0] = ent->rows;
    }
    if ((rc = skge_accum_apply(stream, at, 2, ns))) break;
    r->nlaunch += 2;
  }
  if (!rc) {
    hipLaunchKernelGGL(k_epoch_end, dim3(1), dim3(64), 0, st, epoch_key, r->shards, nviol_total);
    r->nlaunch += 1;
  }
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(st, &g);
  if (rc || e != hipSuccess) {
    if (!rc) set_error("hipStreamEndCapture: %s", hipGetErrorString(e));
    if (g) (void)hipGraphDestroy(g);
    runner_free(r);
    return nullptr;
  }
  r->graph = g;
  e = hipGraphInstantiate(&r->exec, g, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    set_error("hipGraphInstantiate: %s", hipGetErrorString(e));
    runner_free(r);
    return nullptr;
  }
  return r;
}

extern "C" int skge_runner_run(skge_runner_t* r, void* stream, int nepochs) {
  SKGE_CHECK_ARG(r && r->exec, "bad runner");
  for (int i = 0; i < nepochs; ++i) SKGE_CHECK_HIP(hipGraphLaunch(r->exec, as_stream(stream)));
  return SKGE_OK;
}

extern "C" int skge_runner_nlaunches(const skge_runner_t* r) { return r ? r->nlaunch : -1; }

extern "C" void skge_runner_destroy(skge_runner_t* r) { runner_free(r); }
