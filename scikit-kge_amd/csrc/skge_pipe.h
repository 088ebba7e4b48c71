// Shared by the pipelined runners (skge_pipeline.hip: TransE;
// skge_hole_pipe.hip: HolE): the launch arguments, the row update every
// apply shares, the claim / hand-off protocol and the relation-row helpers.
// The protocol itself is described at the top of skge_pipeline.hip.
#pragma once
#include "skge_host.h"

namespace skge {


// Packed int16x4 entity sums are exact while every field's total stays within
// +-32767.  Each occurrence adds a coefficient no larger in magnitude than the
// count it adds (s: |v0 gp + v1 (gp + g1)| <= v0 + 2 v1, ...), so a row whose
// count c is <= 32767 cannot have wrapped; the apply flags any larger count
// (the host picks packed sums only when its bound keeps counts below that,
// skge_amd/device.py packed_count_bound).  Relation rows use int32x2 sums
// (|v0 (gp + g0) + v1 (gp + g1)| <= 2 (v0 + v1) per positive): exact for any
// batch size this runner accepts.
constexpr int PACKED_MAX = 32767;
enum : int { ERR_WAIT = 1, ERR_PACKED = 2 };
// hot rows (PipeTab::hot): replicas per row; a row is hot when its expected
// slots per batch are >= HOT_MIN and >= HOT_REL x the average row's; at most
// HOT_MAX rows.  WN18 Zipf(1.1), nb = 100, same box: HOT_MIN 16 / 8 / 4 ->
// 110.6 / 116.1 / 117.4 M triples/s (4 replicas); 16 replicas 108.2 M (the
// readers' fold: 97 VGPRs, 4 waves per SIMD; 4 replicas: 74 VGPRs, 6).  The
// relative bar keeps a uniform KG's rows at large batches out (WN18 nb = 2:
// ~3.5 slots per row and batch; hot rows there cost 531 / 519 vs 540 M).
// (HOT_MIN 2 / 3, HOT_REL 4: within noise of these, same box)
constexpr int HOT_REPS = 4, HOT_MIN = 4, HOT_REL = 8, HOT_MAX = 256;

struct UpdParams {
  int opt, post;
  float lr, rin, rout, fdiv;   // g = (sum + rin*P)/div + rout*P, div = fdiv > 0 ? fdiv : count
};

struct PipeTab {               // entity table
  float* P;
  float* A;                    // AdaGrad state or nullptr (SGD)
  unsigned long long* sum[2];  // exact int16x4 sums, by batch parity
  int* cnt[2];
  int* touched[2];             // slot records of the batch
  int* pend[2];                // [rows]: id of the launch that last accumulated into the row
  int* own[2];                 // large batches, [rows] by batch parity: a slot naming the row
                               // (plain stores, one survives): the A role applies a row from
                               // that slot only, so duplicate slots cost no claim
  int* done;                   // [rows]: id of the launch whose update of the row was last applied
  // hot rows (skewed KGs): rows expected in >= HOT_MIN slots per batch add
  // their sums and counts into HOT_REPS replicas (positive w into replica
  // w % HOT_REPS) instead of one row and record no slot or mark; their values
  // live in hP / hA during a run (hot_value), and readers never wait for them
  const int* hot;              // [rows]: hot index h, or -1 (nullptr: no hot rows)
  const int* hot_rows;         // [nhot]: the hot rows
  int nhot, hw;                // hw: 8-B words per replica row (sums, whole 128-B lines)
  unsigned long long* hsum[3]; // [nhot][HOT_REPS][hw] by launch id % 3
  int* hcnt[3];                // [nhot][HOT_REPS] by launch id % 3
  float* hP[2];                // [nhot][d]: the value after launch g in hP[g & 1]
  float* hA[2];                // AdaGrad state likewise (nullptr: SGD)
  UpdParams u;
  int* claims;                 // profile only: rows applied in this launch (sharded)
  int* err;                    // ERR_* bits
};

struct RelTab {                // relation table
  float* P[2];                 // P[0]: the caller's parameters; P[1]: the other buffer
  float* A[2];                 // AdaGrad state, likewise (nullptr: SGD)
  unsigned long long* acc[3];  // [rows][rw]: int16x4 sums in words [0, d/4), count in word d/4
                               // (w32: int32x2 sums in words [0, d/2), count in word d/2)
  int rows, rw;
  int folded;                  // replicas folded into replica 0 after each batch (k_rel_fold*)
  int reps;                    // HolE: accumulator replicas per copy (row p of replica k at
                               // k * rows + p); positive w adds into replica w % reps
  UpdParams u;
  int* updated;                // profile only: rows with a nonzero count (sharded)
};

// The fused TransE runner's entity table (k_pipe_fused, round 5).  Rows live
// in one of two buffers; a row updated in launch g is written to the buffer
// its previous value is NOT in, so the pre-update value stays readable for
// the whole launch.  Sums, counts and slot records rotate over three copies
// by launch id: launch g adds into copy g % 3, reads and applies copy
// (g - 1) % 3 and zeroes copy (g - 2) % 3 (the copy launch g + 1 adds into).
struct FusedTab {
  float* P[2];        // P[0]: the caller's parameters; P[1]: the runner's second buffer
  float* A[2];        // AdaGrad state, likewise (nullptr: SGD)
  void* sum[3];       // exact packed sums (int8x4 / int16x4) by launch id % 3
  int* cnt[3];
  int* touched[3];    // slot records by launch id % 3: row | buffer << 30 (the buffer
                      // holding the row after that launch), -1: no row
  int4* meta;         // [rows]: x / y: id of the last even / odd launch that accumulated
                      // into the row; z: (id of the launch that last wrote the row << 1) |
                      // the buffer it wrote; w: id of the last launch that claimed its apply
};
constexpr int SLOT_BUF = 1 << 30;

struct PipeArgs {
  PipeTab E;
  RelTab R;
  FusedTab F;                  // fused runner (k_pipe_fused) only
  int pprev_slots;             // fused: slots of the launch before the previous one (zeroed)
  int nwork;                   // fused: work items (max of this, the previous and the
                               // pre-previous launch's positives)
  const int4* rec;             // [T]: (s, o, p, s') of the epoch's positive j
  const int* rec_n1;           // [T]: o'
  long long start;             // B role: this batch's positives [start, start + count)
  int count;
  int lo, hi;                  // B role: the positives [lo, hi) of the batch this launch scores
                               // (data-parallel ranks: their slice; else 0, count)
  uint32_t* dprec;             // data-parallel: one record per scored positive (pipe_dp_record_words)
  int prev_slots;              // A role: entity slots of the previous batch
  int b, nb1;                  // batch index in the epoch (nb1: the flush), batches per epoch
  const uint64_t* epoch_key;
  int d, nA;                   // nA: workgroups of the A role
  int af;                      // HolE: activation (skge/actfun.py)
  float margin;
  int* nviol_total;            // the caller's counter: += the epoch's violations, at the flush
  int* nviol_shards;           // [NSHARD][SHARD_STRIDE]: this epoch's violations so far
  int* stats_viol;             // profile only: violating pairs of this launch (sharded)
  unsigned long long* trace;   // diagnostics only: per-wave timestamps of one launch
  const float2* tw;            // HolE FFT form: the twiddle table (hole_fft_table)
  int* err;                    // set when a bounded wait gives up
  int pair_r1;                 // HolE pair form: the wave (0 / 1) that loads and updates R[p]
};

// Data-parallel record of one scored positive (k_pipe_batch with dprec): word
// 0 = v0 | v1 << 1, then for a violating positive one word per quad q holding
// the ternary codes (0: 0, 1: +1, 2: -1) of its sign vectors gp, g0, g1 in
// bytes 0-2 (the header s, o, p, s', o' every rank has from the epoch's
// records).  Words rounded up to 16 B.
__host__ __device__ inline int pipe_dp_record_words(int d) { return (1 + (d >> 2) + 3) & ~3; }

__device__ __forceinline__ uint32_t tern4q(const float4& v) {
  auto t = [](float x) -> uint32_t { return x > 0.0f ? 1u : (x < 0.0f ? 2u : 0u); };
  return t(v.x) | (t(v.y) << 2) | (t(v.z) << 4) | (t(v.w) << 6);
}
__device__ __forceinline__ float4 untern4q(uint32_t b) {
  auto u = [](uint32_t c) -> float { return (float)(int)(c & 1u) - (float)(int)((c >> 1) & 1u); };
  return make_float4(u(b), u(b >> 2), u(b >> 4), u(b >> 6));
}

// Launch id: consecutive within an epoch (batches 0..nb1-1, then the flush)
// and across epochs (epoch e+1's batch 0 follows epoch e's flush); >= 2, so
// zero-initialised marks never look pending.
__device__ __forceinline__ int launch_id(const PipeArgs& a) {
  return (int)(*a.epoch_key * (uint64_t)(a.nb1 + 1)) + a.b + 2;
}

// 16-B write-through (sc1) row accesses through a buffer descriptor over one
// row (MI355X_MICROARCH.md: 4-B sc1 stores are ~6x the 16-B time per byte).
// Lanes past the row fall outside the descriptor: loads return 0, stores drop.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int AUX_SC1 = 16;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const float* T, int row, int d) {
  row = __builtin_amdgcn_readfirstlane(row);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(T) + (size_t)row * d, 0, d * 4,
                                           0x00020000);
}

template <int KQ>
__device__ __forceinline__ void load_row4_sc1(const float* T, int row, int d, float4 (&v)[KQ]) {
  const __amdgpu_buffer_rsrc_t rs = row_rsrc(T, row, d);
  const int l = lane_id();
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, (64 * m + l) * 16, 0, AUX_SC1);
    v[m] = *reinterpret_cast<const float4*>(&x);
  }
}

template <int KQ>
__device__ __forceinline__ void store_row4_sc1(float* T, int row, int d, const float4 (&v)[KQ]) {
  const __amdgpu_buffer_rsrc_t rs = row_rsrc(T, row, d);
  const int l = lane_id();
#pragma unroll
  for (int m = 0; m < KQ; ++m)
    __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(&v[m]), rs,
                                           (64 * m + l) * 16, 0, AUX_SC1);
}

// plain 16-B row stores (lanes past the row skipped)
template <int KQ>
__device__ __forceinline__ void store_row4(float* T, int row, int d, const float4 (&v)[KQ]) {
  float4* r = reinterpret_cast<float4*>(T + (size_t)row * d);
  const int l = lane_id(), nq = d >> 2;
#pragma unroll
  for (int m = 0; m < KQ; ++m)
    if (64 * m + l < nq) r[64 * m + l] = v[m];
}

// A claimed row's new value and state: while scoring waves of the launch may
// read it (wt), write-through stores, a drain, then the done word; at the
// flush (no scoring waves; the next launch sees plain stores) plain stores
//
// Only P is read by the launch's scoring waves (the AdaGrad state is read by
// the row's next applier, a later launch), so only P's stores are
// write-through and drained before the done word; the state and the zeroed
// packed sums follow as plain stores after it (the kernel boundary publishes
// them), keeping them out of the drain the waiters wait on.
template <int KQ>
__device__ __forceinline__ void publish_row(const PipeTab& t, int row, int d, const float4 (&p)[KQ],
                                            const float4 (&a)[KQ], int gp, bool wt) {
  if (!wt) {
    store_row4<KQ>(t.P, row, d, p);
    if (t.A) store_row4<KQ>(t.A, row, d, a);
    return;
  }
  store_row4_sc1<KQ>(t.P, row, d, p);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every store of this wave has landed
  if (lane_id() == 0)
    __hip_atomic_store(t.done + row, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t.A) store_row4<KQ>(t.A, row, d, a);
}

// load a quad-layout row of P, A (optional) and packed sums (clamped,
// unconditional loads; lanes past the row read the last quad)
template <int KQ>
__device__ __forceinline__ void load_upd_row(const float* P, const float* A,
                                             const unsigned long long* S, int d, float4 (&p)[KQ],
                                             float4 (&a)[KQ], unsigned long long (&sv)[KQ]) {
  const int l = lane_id(), nq = d >> 2;
  const float4* prow = reinterpret_cast<const float4*>(P);
  const float4* arow = reinterpret_cast<const float4*>(A);
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l, qc = q < nq ? q : nq - 1;
    sv[m] = S[qc];
    p[m] = prow[qc];
    a[m] = A ? arow[qc] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
}

// One row's update from its exact packed sums (W32: int32x2 in sv / sw, else
// int16x4 in sv) and occurrence count c > 0: segment
// mean + AdaGrad / SGD + projection; the same arithmetic as apply_row_i16
// (skge_update.hip) and the reference (skge/param.py:130, 147-155;
// skge/transe.py normalize).  Lanes past the row end with zeros.
// (row_update_s: the same from the sums already decoded to floats, zero past
// the row -- the fused runner's form; every packed apply shares this code, so
// a row's update has the same bits whichever kernel computes it)
template <int KQ>
__device__ __forceinline__ void row_update_s(const UpdParams& t, int c, int d,
                                             const float4 (&sms)[KQ], float4 (&p)[KQ],
                                             float4 (&a)[KQ]) {
  const int l = lane_id(), nq = d >> 2;
  const bool ada = t.opt == OPT_ADAGRAD;
  const float div = t.fdiv > 0.0f ? t.fdiv : (float)c;
  float ss = 0.0f;
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const bool in = 64 * m + l < nq;
    const float4 sm = sms[m];
#define SKGE_UP(X)                                                      \
  {                                                                     \
    const float g = (sm.X + t.rin * p[m].X) / div + t.rout * p[m].X;    \
    float pv = p[m].X;                                                  \
    if (ada) {                                                          \
      a[m].X = a[m].X + g * g;                        /* param.py:147 */\
      pv = pv - adagrad_step_fast(t.lr, g, a[m].X);   /* 152-155 */     \
    } else {                                                            \
      pv = pv - t.lr * g;                             /* param.py:130 */\
    }                                                                   \
    p[m].X = in ? pv : 0.0f;                                            \
    ss += p[m].X * p[m].X;                                              \
  }
    SKGE_UP(x)
    SKGE_UP(y)
    SKGE_UP(z)
    SKGE_UP(w)
#undef SKGE_UP
  }
  if (t.post != POST_NONE) {
    ss = wave_sum(ss);
    const float inv = proj_scale_fast(t.post, ss);   // param.py:165-166 / 171-173
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      p[m].x = p[m].x * inv;
      p[m].y = p[m].y * inv;
      p[m].z = p[m].z * inv;
      p[m].w = p[m].w * inv;
    }
  }
}

template <int KQ, bool W32>
__device__ __forceinline__ void row_update(const UpdParams& t, int c, int d,
                                           const unsigned long long (&sv)[KQ],
                                           const unsigned long long (&sw)[KQ], float4 (&p)[KQ],
                                           float4 (&a)[KQ]) {
  const int l = lane_id(), nq = d >> 2;
  float4 sm[KQ];
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const bool in = 64 * m + l < nq;
    if (W32) {   // int32x2 sums: quad q in words sv (elements 0, 1) and sw (2, 3)
      const float2 lo = unpack_i32x2(in ? sv[m] : 0ull), hi = unpack_i32x2(in ? sw[m] : 0ull);
      sm[m] = make_float4(lo.x, lo.y, hi.x, hi.y);
    } else {     // int16x4 sums
      sm[m] = unpack_i16x4(in ? sv[m] : 0ull);
    }
  }
  row_update_s<KQ>(t, c, d, sm, p, a);
}

// Claim a pending entity row's update (the first wave to swap its count out
// applies it) and, if claimed, apply it from accumulator copy `pp` and publish
// it as launch `gp` (write-through stores, drain, done word).  The row's sums,
// parameters and state are loaded in the same memory round trip as the claim:
// nobody writes them before the claim is won, and a loser discards them.
template <int KQ, bool E8 = false>
__device__ __forceinline__ void claim_and_apply(const PipeTab& t, int pp, int row, int d, int gp,
                                                bool wt = true) {
  const int l = lane_id(), nq = d >> 2;
  int c = 0;
  if (l == 0) c = atomicExch(t.cnt[pp] + row, 0);
  unsigned long long* srow = t.sum[pp] + (size_t)row * nq;
  unsigned int* srow8 = reinterpret_cast<unsigned int*>(t.sum[pp]) + (size_t)row * nq;
  unsigned long long sv[KQ];
  float4 p[KQ], a[KQ];
  if (E8) {   // int8x4 sums: one dword per quad, re-packed as int16x4 for row_update
    unsigned int s8[KQ];
    const float4* prow = reinterpret_cast<const float4*>(t.P + (size_t)row * d);
    const float4* arow = reinterpret_cast<const float4*>(t.A + (size_t)row * d);
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      const int q = 64 * m + l, qc = q < nq ? q : nq - 1;
      s8[m] = srow8[qc];
      p[m] = prow[qc];
      a[m] = t.A ? arow[qc] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
#pragma unroll
    for (int m = 0; m < KQ; ++m) sv[m] = pack_i16x4(unpack_i8x4_sum(s8[m]));
  } else {
    load_upd_row<KQ>(t.P + (size_t)row * d, t.A ? t.A + (size_t)row * d : nullptr, srow, d, p, a,
                     sv);
  }
  c = __builtin_amdgcn_readfirstlane(c);
  if (c == 0) return;   // another wave owns the row
  // a field may have wrapped: 16-bit fields past 32767, 8-bit fields past 127
  if (c > (E8 ? 127 : PACKED_MAX) && l == 0) atomicOr(t.err, ERR_PACKED);
  row_update<KQ, false>(t.u, c, d, sv, sv, p, a);
  publish_row<KQ>(t, row, d, p, a, gp, wt);
  // the consumed sums zeroed after the publish (publish_row)
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l;
    if (q < nq) {
      if (E8)
        srow8[q] = 0u;
      else
        srow[q] = 0ull;
    }
  }
  if (t.claims && l == 0) atomicAdd(shard_of(t.claims), 1);
}

// Hot rows (PipeTab::hot): nobody waits for them.  Their values live in two
// buffers by launch-id parity -- hP[g & 1] holds the value after launch g's
// update -- and their sums / counts in three replica copies by launch id % 3
// (launch g adds into copy g % 3, consumes (g-1) % 3, zeroes (g-2) % 3).  The
// value a launch-g reader needs is the one after batch b-1's update: the
// previous value hP[(g-1) & 1] updated with copy (g-1) % 3 -- inputs nobody
// writes during launch g -- so every reader computes it itself, with the
// applier's code (the same bits), in one round trip: the row, its state, the
// replica counts and all replica sums (added as 64-bit words: the words one
// row would have accumulated).  Returns the count (0: no update; p, a = the
// previous value and state).  Lanes past the row end with zeros.
template <int KQ>
__device__ __forceinline__ int hot_value(const PipeTab& t, int h, int g, int d, float4 (&p)[KQ],
                                         float4 (&a)[KQ]) {
  const int l = lane_id(), nq = d >> 2;
  const int src = (g - 1) & 1, cp = (g - 1) % 3;
  const float4* prow = reinterpret_cast<const float4*>(t.hP[src] + (size_t)h * d);
  const float4* arow = reinterpret_cast<const float4*>(t.hA[src] + (size_t)h * d);
  const unsigned long long* hrow = t.hsum[cp] + (size_t)h * HOT_REPS * t.hw;
  const int cl = l < HOT_REPS ? t.hcnt[cp][h * HOT_REPS + l] : 0;
  // replicas per round trip
  constexpr int G = KQ == 1 ? HOT_REPS : 4;
  unsigned long long sv[KQ], x[G][KQ];
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l, qc = q < nq ? q : nq - 1;
    sv[m] = 0ull;
    p[m] = prow[qc];
    a[m] = t.hA[src] ? arow[qc] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
#pragma unroll 1
  for (int k0 = 0; k0 < HOT_REPS; k0 += G) {
#pragma unroll
    for (int k = 0; k < G; ++k)
#pragma unroll
      for (int m = 0; m < KQ; ++m) {
        const int q = 64 * m + l;
        x[k][m] = q < nq ? hrow[(size_t)(k0 + k) * t.hw + q] : 0ull;
      }
#pragma unroll
    for (int k = 0; k < G; ++k)
#pragma unroll
      for (int m = 0; m < KQ; ++m) sv[m] += x[k][m];
  }
  const int c = wave_sum_int(cl);
  if (c) {
    row_update<KQ, false>(t.u, c, d, sv, sv, p, a);   // (zeroes the lanes past the row)
  } else {
#pragma unroll
    for (int m = 0; m < KQ; ++m)
      if (64 * m + l >= nq) p[m] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  return c;
}

// Launch g's item for hot row h: its value after the launch into hP[g & 1]
// (plain stores: read only by later launches), the replica copy two launches
// old zeroed (launch g + 1 adds into it)
template <int KQ>
__device__ __forceinline__ void apply_hot(const PipeTab& t, int h, int g, int d) {
  const int l = lane_id(), nq = d >> 2;
  float4 p[KQ], a[KQ];
  const int c = hot_value<KQ>(t, h, g, d, p, a);
  store_row4<KQ>(t.hP[g & 1], h, d, p);
  if (t.hA[0]) store_row4<KQ>(t.hA[g & 1], h, d, a);
  const int old = (g - 2) % 3;
  unsigned long long* hrow = t.hsum[old] + (size_t)h * HOT_REPS * t.hw;
#pragma unroll
  for (int k = 0; k < HOT_REPS; ++k)
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      const int q = 64 * m + l;
      if (q < nq) hrow[(size_t)k * t.hw + q] = 0ull;
    }
  if (l < HOT_REPS) t.hcnt[old][h * HOT_REPS + l] = 0;
  if (c > PACKED_MAX && l == 0) atomicOr(t.err, ERR_PACKED);
  if (c && t.claims && l == 0) atomicAdd(shard_of(t.claims), 1);
}

// Large batches: up to GRP_ROWS owner rows of a 64-slot group at once -- all
// claims in one atomic instruction (lane j claims row j), all rows' loads in
// one round trip, every claimed row updated and stored write-through, ONE
// drain, then the done words -- instead of a claim / load / store / drain
// chain per row.
#ifndef SKGE_PIPE_GRP_ROWS
// WN18 nb = 2, same box: 8 rows 467 M, 4 rows 482-488 M (124 -> 85 VGPRs);
// round 5 (with the flush's plain stores; 4 -> 2 rows: 90 -> 77 VGPRs, 5 -> 6
// waves per SIMD): 4 rows 521-523 M, 2 rows 530 M, 1 row 503 M
#define SKGE_PIPE_GRP_ROWS 2
#endif
constexpr int GRP_ROWS = SKGE_PIPE_GRP_ROWS;
template <int KQ, bool E8>
__device__ __forceinline__ void claim_and_apply_rows(const PipeTab& t, int pp, int rl, int n,
                                                     int d, int gp, bool wt) {
  const int l = lane_id(), nq = d >> 2;
  int c = 0;
  if (l < n) c = atomicExch(t.cnt[pp] + rl, 0);   // lane j holds row j (j < n)
  float4 p[GRP_ROWS][KQ], a[GRP_ROWS][KQ];
  unsigned long long sv[GRP_ROWS][KQ];
  int row[GRP_ROWS];
#pragma unroll
  for (int j = 0; j < GRP_ROWS; ++j) {
    row[j] = __builtin_amdgcn_readlane(rl, j < n ? j : 0);
    const float4* prow = reinterpret_cast<const float4*>(t.P + (size_t)row[j] * d);
    const float4* arow = reinterpret_cast<const float4*>(t.A + (size_t)row[j] * d);
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      const int q = 64 * m + l, qc = q < nq ? q : nq - 1;
      if (E8)
        sv[j][m] = reinterpret_cast<const unsigned int*>(t.sum[pp])[(size_t)row[j] * nq + qc];
      else
        sv[j][m] = t.sum[pp][(size_t)row[j] * nq + qc];
      p[j][m] = prow[qc];
      a[j][m] = t.A ? arow[qc] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
  }
  int any = 0;
#pragma unroll
  for (int j = 0; j < GRP_ROWS; ++j) {
    const int cj = __builtin_amdgcn_readlane(c, j);
    if (j >= n || cj == 0) continue;   // past the rows, or another wave owns the row
    any = 1;
    if (cj > (E8 ? 127 : PACKED_MAX) && l == 0) atomicOr(t.err, ERR_PACKED);
    if (E8) {
#pragma unroll
      for (int m = 0; m < KQ; ++m) sv[j][m] = pack_i16x4(unpack_i8x4_sum((unsigned int)sv[j][m]));
    }
    row_update<KQ, false>(t.u, cj, d, sv[j], sv[j], p[j], a[j]);
    if (wt) {
      store_row4_sc1<KQ>(t.P, row[j], d, p[j]);
    } else {   // the flush: no reader in this launch
      store_row4<KQ>(t.P, row[j], d, p[j]);
    }
  }
  if (!any) return;
  if (wt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every store of this wave has landed
    if (l < n && c != 0)
      __hip_atomic_store(t.done + rl, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // the state and the zeroed sums: plain stores after the done words
  // (publish_row)
#pragma unroll
  for (int j = 0; j < GRP_ROWS; ++j) {
    if (j >= n || __builtin_amdgcn_readlane(c, j) == 0) continue;
    if (t.A) store_row4<KQ>(t.A, row[j], d, a[j]);
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      const int q = 64 * m + l;
      if (q < nq) {
        if (E8)
          reinterpret_cast<unsigned int*>(t.sum[pp])[(size_t)row[j] * nq + q] = 0u;
        else
          t.sum[pp][(size_t)row[j] * nq + q] = 0ull;
      }
    }
  }
  if (t.claims && l == 0) {
    int k = 0;
#pragma unroll
    for (int j = 0; j < GRP_ROWS; ++j) k += (j < n && __builtin_amdgcn_readlane(c, j) != 0);
    atomicAdd(shard_of(t.claims), k);
  }
}

// B role: make sure launch gp's update of entity `row` (pending at launch
// start) has landed -- apply it if nobody has claimed it yet, else wait for
// its publisher
template <int KQ, bool E8 = false>
__device__ __forceinline__ void ensure_applied(const PipeTab& t, int pp, int row, int d, int gp,
                                               int* err) {
  if (__hip_atomic_load(t.done + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gp) return;
  claim_and_apply<KQ, E8>(t, pp, row, d, gp);
  unsigned spins = 0;
  while (__hip_atomic_load(t.done + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gp) {
    __builtin_amdgcn_s_sleep(2);
    if (++spins > (1u << 22)) {   // ~0.5 s: never hang the GPU; report instead
      if (lane_id() == 0) atomicOr(err, ERR_WAIT);
      break;
    }
    if ((spins & 1023u) == 0 &&   // once one wait has given up, the rest stop too
        __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      break;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the re-read below the poll
}

// relation row R_b[row] (the value batch b scores with): R_{b-1}[row] from
// buffer rd updated with batch b-1's sums (accumulator copy ra).  W32: int32x2
// sums, words 2q, 2q+1 hold quad q and word 2 nq the count; else int16x4
// sums, word q holds quad q and word nq the count.  Every load is issued
// before the count is read (kept in load_upd_row's shape: hipcc would sink
// loads used only under `if (c)` below the count's wait).  Lanes past the row
// end with zeros whether or not the row was updated (they enter the scores).
template <int KQ, bool W32>
__device__ __forceinline__ void rel_row(const RelTab& t, int row, int d, int rd, int ra,
                                        float4 (&p)[KQ], float4 (&a)[KQ], int& c) {
  const int l = lane_id(), nq = d >> 2;
  const unsigned long long* acc = t.acc[ra] + (size_t)row * t.rw;
  unsigned long long sv[KQ], sw[KQ];
  if (W32) {
    const float4* prow = reinterpret_cast<const float4*>(t.P[rd] + (size_t)row * d);
    const float4* arow = reinterpret_cast<const float4*>(t.A[rd] + (size_t)row * d);
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      const int q = 64 * m + l, qc = q < nq ? q : nq - 1;
      const ulonglong2 w = reinterpret_cast<const ulonglong2*>(acc)[qc];
      sv[m] = w.x;
      sw[m] = w.y;
      p[m] = prow[qc];
      a[m] = t.A[rd] ? arow[qc] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
  } else {
    load_upd_row<KQ>(t.P[rd] + (size_t)row * d, t.A[rd] ? t.A[rd] + (size_t)row * d : nullptr,
                     acc, d, p, a, sv);
  }
  c = __builtin_amdgcn_readfirstlane((int)acc[W32 ? 2 * nq : nq]);
  if (c) {
    row_update<KQ, W32>(t.u, c, d, sv, sw, p, a);   // (zeroes the lanes past the row)
  }
  else {
#pragma unroll
    for (int m = 0; m < KQ; ++m)
      if (64 * m + l >= nq) p[m] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
}

__device__ __forceinline__ unsigned long long now_10ns() { return __builtin_amdgcn_s_memrealtime(); }

// A kernel argument made opaque to the compiler (kept in SGPRs, or spilled to
// VGPR lanes): under SGPR pressure hipcc otherwise re-loads argument fields
// from the kernarg segment where they are used, and the scoring wave's
// scatter section paid one dependent scalar-memory round trip per pointer.
template <typename T>
__device__ __forceinline__ T* opaque_ptr(T* p) {
  unsigned long long v = reinterpret_cast<unsigned long long>(p);
  asm volatile("" : "+s"(v));
  return reinterpret_cast<T*>(v);
}

// A role, relation row w: write R_b[w] (from R_{b-1} and batch b-1's sums) to
// buffer rw for the next launch, clear the accumulator copy two launches old
// (at the flush also the previous one: no scoring wave reads it any more)
template <int KQ, bool W32>
__device__ __forceinline__ void rel_publish(const PipeArgs& a, int w, int rd, int rw, int ra_prev,
                                            int ra_old) {
  const int l = lane_id(), d = a.d, nq = d >> 2;
  const int rcw = W32 ? 2 * nq : nq;
  float4 p[KQ], av[KQ];
  int c;
  rel_row<KQ, W32>(a.R, w, d, rd, ra_prev, p, av, c);
  float4* prow = reinterpret_cast<float4*>(a.R.P[rw] + (size_t)w * d);
  float4* arow = a.R.A[rw] ? reinterpret_cast<float4*>(a.R.A[rw] + (size_t)w * d) : nullptr;
  unsigned long long* old = a.R.acc[ra_old] + (size_t)w * a.R.rw;
  unsigned long long* prev = a.R.acc[ra_prev] + (size_t)w * a.R.rw;
  const bool flush = a.b == a.nb1;
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l;
    if (q < nq) {
      prow[q] = p[m];
      if (arow) arow[q] = av[m];
    }
  }
  for (int q = l; q <= rcw; q += 64) {
    old[q] = 0ull;
    if (flush) prev[q] = 0ull;
  }
  if (c && a.R.updated && l == 0) atomicAdd(shard_of(a.R.updated), 1);
  if (!W32 && c > PACKED_MAX && l == 0) atomicOr(a.err, ERR_PACKED);
}

// large batches (owner marks, k_pipe_batch's GRP instances): 3-wave
// workgroups (WN18 nb = 2, same box: 508-510 -> 520 M triples/s; 128: 517 M;
// nb = 100 unchanged by either, so it keeps SKGE_PIPE_WG)
constexpr int PIPE_WG_GRP = 192;
#ifndef SKGE_PIPE_WG
#define SKGE_PIPE_WG 256   // threads per workgroup
#endif

constexpr int HPIPE_OCC = 2;   // HolE: scoring waves per SIMD the apply-workgroup cap assumes (direct form)

// skge_hole_pipe.hip's launchers (host side)
void launch_hole_pipe(int km, bool pair, bool fft, dim3 gr, dim3 bl, size_t lds, hipStream_t st,
                      const PipeArgs& a);
void launch_rel_fold_f(dim3 gr, hipStream_t st, const PipeArgs& a);

}  // namespace skge
