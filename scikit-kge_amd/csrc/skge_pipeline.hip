// Pipelined device batch loop for TransE-L1 (the throughput path, one launch
// per mini-batch).
//
// The reference processes mini-batches strictly in sequence: batch b reads
// the parameters produced by batch b-1's updates (skge/base.py:1268-1284,
// 1306-1316).  The two-launch loop (skge_epoch.hip) honours that with a
// score/scatter kernel and an apply kernel per batch.  Here batch b's scoring
// and batch b-1's updates share ONE launch:
//
//   * all negatives of the epoch are drawn up front (k_epoch_sample: the same
//     counter-based draws and rejection test as k_transe_sample_grad, so the
//     epoch's pairs are identical), giving per-positive records (s, o, p, s', o');
//   * launch g scores batch b ("B" role) while the first nA workgroups apply
//     batch b-1's updates ("A" role);
//   * entity rows (many, each touched by few positives): accumulators
//     double-buffered by batch parity.  A B wave about to read a row batch
//     b-1 touched (pend[row] == g-1, recorded by the previous launch) makes
//     sure that row's update has landed first: it claims (atomicExch on the
//     count) and applies it itself, or waits (bounded) on the row's `done`
//     word.  Appliers publish with write-through (sc1) stores, a vmcnt(0)
//     drain, then the done word; waiters poll it with sc1 loads and re-read
//     the row with sc1 loads (MI355X_MICROARCH.md, hand-off forms, row 1).  A
//     claimer never waits, so dispatch order never matters;
//   * relation rows (few, each read by most positives of a batch): no waiting
//     at all.  Parameters and AdaGrad state are double-buffered (R_b lives in
//     buffer W(b)), accumulators triple-buffered by launch id.  Every B wave
//     recomputes R_b[p] from R_{b-1}[p] and batch b-1's sum itself (a few
//     hundred bytes of L2-hot reads); one A wave per row writes R_b[p] for the
//     next launch and clears the accumulator copy two launches old;
//   * hot entity rows (skewed KGs, skge_pipe.h PipeTab::hot): a hub's sums and
//     count go to one of HOT_REPS replicas per positive and a dedicated apply
//     item folds them, so its ~hundreds of adds per batch do not serialise on
//     one row's addresses.
//
// Every row update depends only on that row's own (exact integer) sums, count,
// parameters and AdaGrad state, computed by the same code (row_update), so the
// result is bitwise identical to the two-launch loop (tested).
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "skge_hole.h"
#include "skge_hole_fft.h"
#include "skge_pipe.h"
#include "skge_sampler.h"

namespace skge {

// HolE pair form: hub rows as TransE's (skge_hole_pipe.hip hot_value_f); 0
// builds the round-5 form for same-box A/Bs (tools/ab_lib.sh)
#ifndef SKGE_HPIPE_HOT
#define SKGE_HPIPE_HOT 1
#endif

// k_pipe_batch (large batches: more than 16k slot records per batch; smaller
// batches run k_pipe_fused below): nA apply workgroups (dispatched first: they
// start the hand-offs the scoring waves may wait on), then the scoring ones.
// GRP: owner marks, GRP_ROWS owner rows per apply round trip.
// DP: the data-parallel form (a slice [lo, hi) of the batch scored, records
// written); its own instance, so the one-GPU kernel keeps round 5's code (the
// slice bounds and the record branch in the shared instance cost 10.45 ->
// 11.15 us per launch, same box: VERDICT r05 item 4's A/B)
template <int KQ, bool W32, bool E8, bool GRP = false, bool HOT = false, bool DP = false>
__global__ __launch_bounds__(GRP ? PIPE_WG_GRP : SKGE_PIPE_WG) void k_pipe_batch(PipeArgs a) {
  const int wpb = blockDim.x >> 6;
  const int l = lane_id();
  const int d = a.d, nq = d >> 2;
  const int rcw = W32 ? 2 * nq : nq;   // relation accumulator: the count word
  const int g = launch_id(a), gp = g - 1;
  const int cp = a.b & 1, pp = cp ^ 1;   // entity accumulator copies: this / previous batch
  const int rd = a.b & 1;                // relation buffer holding R_{b-1}
  const int rw = a.b < a.nb1 ? rd ^ 1 : 0;   // ... receiving R_b (the flush: the caller's)
  const int ra_prev = (g - 1) % 3, ra_cur = g % 3, ra_old = (g - 2) % 3;
  const int nB = (int)gridDim.x - a.nA;
  // apply workgroups first: they start the hand-offs the scoring waves may wait
  // on (measured: 6% faster than scoring first, 9% faster than interleaved)
  const int blk = (int)blockIdx.x;
  const int blk_a = blk, blk_b = blk - a.nA;
  if (blk < a.nA) {
    // ---- A role: write R_b, then apply the previous batch's entity rows ----
    const int nR = a.R.rows;
    // owner marks (large batches): items are groups of 64 slots, scanned
    // lane-parallel; else one slot per item
    const int* const ownp = a.E.own[pp];
    const int nH = a.E.nhot, nRH = nR + nH;   // then one item per hot row
    const int total = nRH + (ownp ? (a.prev_slots + 63) / 64 : a.prev_slots);
    const int wa = blk_a * wpb + (threadIdx.x >> 6);
    const unsigned long long ta0 = a.trace ? now_10ns() : 0ull;
    // the flush scores nothing: plain stores (WN18 nb = 2, same box: 496 -> 539 M)
    const bool wt = a.b < a.nb1;
    if (a.b == a.nb1 && wa == 0)   // the flush: fold the epoch's violation count
      fold_shards(a.nviol_shards, a.nviol_total);
    for (int w = wa; w < total; w += a.nA * wpb) {
      if (w < nR) {
        rel_publish<KQ, W32>(a, w, rd, rw, ra_prev, ra_old);
      } else if (w < nRH) {
        if (HOT) apply_hot<KQ>(a.E, w - nR, g, d);
      } else if (ownp) {
        // 64 slots: their rows and owner marks in two vector loads; only the
        // slot each row's owner mark names applies it (no claim on duplicates)
        const int i = 64 * (w - nRH) + l;
        const int r = i < a.prev_slots ? a.E.touched[pp][i] : -1;
        const bool mine = r >= 0 && ownp[r] == i;
        uint64_t m = __ballot(mine);
        if (GRP) {   // GRP_ROWS owner rows per round trip
          while (m) {
            // compact the next GRP_ROWS owners into lanes 0..n-1
            const int rank = __popcll(m & ((1ull << l) - 1ull));
            const bool take = ((m >> l) & 1ull) && rank < GRP_ROWS;
            const uint64_t tk = __ballot(take);
            const int n = __popcll(tk);
            // lane j < n receives the row of the j-th taken lane
            int src = 0;
            {
              uint64_t t2 = tk;
              for (int j = 0; j < GRP_ROWS && t2; ++j) {
                const int k = __ffsll((unsigned long long)t2) - 1;
                t2 &= t2 - 1;
                if (l == j) src = k;
              }
            }
            const int rl = __builtin_amdgcn_ds_bpermute(src << 2, r);
            claim_and_apply_rows<KQ, E8>(a.E, pp, rl, n, d, gp, wt);
            m &= ~tk;
          }
        } else {
          while (m) {
            const int k = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const int row = __builtin_amdgcn_readlane(r, k);
            claim_and_apply<KQ, E8>(a.E, pp, row, d, gp, wt);
          }
        }
      } else {
        const int row = __builtin_amdgcn_readfirstlane(a.E.touched[pp][w - nRH]);
        if (row >= 0) claim_and_apply<KQ, E8>(a.E, pp, row, d, gp, wt);
      }
    }
    if (a.trace && l == 0) {
      unsigned long long* tr = a.trace + 2 + 6 * (size_t)a.count + 2 * (size_t)wa;
      tr[0] = ta0;
      tr[1] = now_10ns();
    }
    return;
  }
  // ---- B role: score batch b, scatter into accumulator copies cp / ra_cur ----
  int* const cnt_cp = opaque_ptr(a.E.cnt[cp]);
  int* const tch_cp = opaque_ptr(a.E.touched[cp]);
  int* const pend_cp = opaque_ptr(a.E.pend[cp]);
  int* const own_cp = a.E.own[cp];
  unsigned long long* const racc0 = opaque_ptr(a.R.acc[ra_cur]);
  const size_t rrep = (size_t)a.R.rows * a.R.rw;   // words per relation replica
  const int rmask = a.R.reps - 1;                  // reps: a power of two (k_rel_fold)
  unsigned long long* const esum = opaque_ptr(a.E.sum[cp]);
  // the batch's records through buffer descriptors built once (not pointers
  // re-loaded from the kernarg segment on the wave's first dependent chain)
  const __amdgpu_buffer_rsrc_t rec_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int4*>(a.rec + a.start), 0, a.count * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t rec1_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int*>(a.rec_n1 + a.start), 0, a.count * 4, 0x00020000);
  int nv = 0;
  const int lo = DP ? a.lo : 0, hi = DP ? a.hi : a.count;
  for (int w = lo + blk_b * wpb + (threadIdx.x >> 6); w < hi; w += nB * wpb) {
    // large batches: positive w adds its relation sums into replica w % reps
    // (k_rel_fold folds them after the launch), spreading the hot rows' atomics
    unsigned long long* const racc = racc0 + (size_t)(w & rmask) * rrep;
    unsigned long long tt[4];
    if (a.trace) tt[0] = now_10ns();
    const u32x4 rx = __builtin_amdgcn_raw_buffer_load_b128(rec_rs, w * 16, 0, 0);
    const int r1 = (int)__builtin_amdgcn_raw_buffer_load_b32(rec1_rs, w * 4, 0, 0);
    const int4 r4 = make_int4((int)rx.x, (int)rx.y, (int)rx.z, (int)rx.w);
    // both record loads in one memory round trip (left alone, the scheduler
    // may put the first load's wait before the second load)
    __builtin_amdgcn_sched_barrier(0);
    const int s = __builtin_amdgcn_readfirstlane(r4.x);
    const int o = __builtin_amdgcn_readfirstlane(r4.y);
    const int p = __builtin_amdgcn_readfirstlane(r4.z);
    const int neg0 = __builtin_amdgcn_readfirstlane(r4.w);
    const int neg1 = __builtin_amdgcn_readfirstlane(r1);
    const int n0r = neg0 >= 0 ? neg0 : s, n1r = neg1 >= 0 ? neg1 : o;
    // entity rows as of the launch start (plain loads), their pending marks,
    // and the relation row this batch scores with
    float4 es[KQ], eo[KQ], rp[KQ], fs[KQ], fo[KQ];
    load_row4<KQ>(a.E.P, s, d, es);
    load_row4<KQ>(a.E.P, o, d, eo);
    load_row4<KQ>(a.E.P, n0r, d, fs);
    load_row4<KQ>(a.E.P, n1r, d, fo);
    // pending marks and the rows' done words in the same round trip: a pending
    // row whose update is already published needs only the re-read below (at
    // nb = 2 every row is pending; one done check per row in sequence had cost
    // ~1.9 us per wave)
    int mark = 0, dn = 0, hx = -1;
    if (l < 4) {
      const int rr = sel4(l, s, o, n0r, n1r);
      mark = a.E.pend[pp][rr];
      dn = __hip_atomic_load(a.E.done + rr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (HOT) hx = a.E.hot[rr];
    }
    {
      float4 ra[KQ];
      int c;
      rel_row<KQ, W32>(a.R, p, d, rd, ra_prev, rp, ra, c);
    }
    const uint64_t pend = __ballot(mark == gp) & 0xfull;
    const uint64_t unpub = pend & ~__ballot(dn == gp);   // pending and not yet published
    if (a.trace) tt[1] = now_10ns();
    if (pend) {   // some entity rows have an update of batch b-1 outstanding
      // one (not unrolled) copy of the claim/apply/wait code keeps registers low
#pragma unroll 1
      for (int k = 0; k < 4; ++k) {
        if (!((unpub >> k) & 1ull)) continue;
        ensure_applied<KQ, E8>(a.E, pp, sel4(k, s, o, n0r, n1r), d, gp, a.err);
      }
      if (pend & 1ull) load_row4_sc1<KQ>(a.E.P, s, d, es);
      if (pend & 2ull) load_row4_sc1<KQ>(a.E.P, o, d, eo);
      if (pend & 4ull) load_row4_sc1<KQ>(a.E.P, n0r, d, fs);
      if (pend & 8ull) load_row4_sc1<KQ>(a.E.P, n1r, d, fo);
    }
    if (HOT) {   // hot rows: the value after batch b-1's update, computed here
      const uint64_t hm = __ballot(hx >= 0) & 0xfull;
#pragma unroll 1
      for (int k = 0; k < 4; ++k) {
        if (!((hm >> k) & 1ull)) continue;
        float4 hv[KQ], ha[KQ];
        hot_value<KQ>(a.E, __builtin_amdgcn_readlane(hx, k), g, d, hv, ha);
#pragma unroll
        for (int m = 0; m < KQ; ++m) {
          if (k == 0) es[m] = hv[m];
          if (k == 1) eo[m] = hv[m];
          if (k == 2) fs[m] = hv[m];
          if (k == 3) fo[m] = hv[m];
        }
      }
    }
    if (a.trace) tt[2] = now_10ns();
    float ps = 0.0f, n0 = 0.0f, n1 = 0.0f;
    float4 gp4[KQ], g0[KQ], g1[KQ];
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
    gp4[m].X = signf_np(-((eo[m].X - rp[m].X) - es[m].X)); /* transe.py:103,115 */    \
    g0[m].X = signf_np((eo[m].X - rp[m].X) - fs[m].X);     /* transe.py:104,117 */    \
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
    const int v0 = (neg0 >= 0 && ns0 + a.margin > pscore) ? 1 : 0;   // strict >, transe.py:73
    const int v1 = (neg1 >= 0 && ns1 + a.margin > pscore) ? 1 : 0;
    if (a.trace) tt[3] = now_10ns();
    if (DP && a.dprec) {   // data-parallel: the positive's record for the other ranks
      uint32_t* out = a.dprec + (size_t)(w - lo) * pipe_dp_record_words(d);
      if (l == 0) out[0] = (uint32_t)(v0 | (v1 << 1));
      if (v0 + v1 > 0) {
#pragma unroll
        for (int m = 0; m < KQ; ++m) {
          const int q = 64 * m + l;
          if (q < nq) out[1 + q] = tern4q(gp4[m]) | (tern4q(g0[m]) << 8) | (tern4q(g1[m]) << 16);
        }
      }
    }
    {
      // counts, touched slots and pending marks of this batch
      const int cE = sel4(l, v0 + 2 * v1, 2 * v0 + v1, v0, v1);
      const int rE = sel4(l, s, o, neg0, neg1);
      if (HOT && l < 4 && hx >= 0) {   // hot row: count into its replica, no slot record
        if (cE > 0) atomicAdd(a.E.hcnt[g % 3] + hx * HOT_REPS + (w & (HOT_REPS - 1)), cE);
        tch_cp[4 * w + l] = -1;
      } else if (l < 4) {
        commit_slot(cnt_cp, tch_cp, rE, cE, 4 * w + l);
        if (cE > 0) {
          pend_cp[rE] = g;
          if (own_cp) own_cp[rE] = 4 * w + l;   // large batches: this slot may own the row
        }
      } else if (l == 4 && v0 + v1 > 0) {
        atomicAdd(racc + (size_t)p * a.R.rw + rcw, (unsigned long long)(2 * (v0 + v1)));
      }
    }
    if (v0 + v1 > 0) {
      nv += v0 + v1;
      const float fv0 = (float)v0, fv1 = (float)v1;
      float4 cs[KQ], co[KQ], c0[KQ], c1[KQ], cr[KQ];
#pragma unroll
      for (int m = 0; m < KQ; ++m) {
#define SKGE_CO(X)                                                   \
  cs[m].X = fv0 * gp4[m].X + fv1 * (gp4[m].X + g1[m].X);             \
  co[m].X = -(fv0 * (gp4[m].X + g0[m].X) + fv1 * gp4[m].X);          \
  c0[m].X = g0[m].X;                                                 \
  c1[m].X = -g1[m].X;                                                \
  cr[m].X = fv0 * (gp4[m].X + g0[m].X) + fv1 * (gp4[m].X + g1[m].X);
        SKGE_CO(x)
        SKGE_CO(y)
        SKGE_CO(z)
        SKGE_CO(w)
#undef SKGE_CO
      }
      if (E8) {   // int8x4 sums: one 32-bit atomic per quad
        unsigned int* es8 = reinterpret_cast<unsigned int*>(esum);
        acc_row4_i8<KQ>(es8, s, cs, d);
        acc_row4_i8<KQ>(es8, o, co, d);
        if (v0) acc_row4_i8<KQ>(es8, neg0, c0, d);
        if (v1) acc_row4_i8<KQ>(es8, neg1, c1, d);
      } else {
        // a hot row's sums go to replica w % HOT_REPS
        auto base = [&](int k, int row) {
          const int h = HOT ? __builtin_amdgcn_readlane(hx, k) : -1;
          return h >= 0 ? a.E.hsum[g % 3] + ((size_t)h * HOT_REPS + (w & (HOT_REPS - 1))) * a.E.hw
                        : esum + (size_t)row * nq;
        };
        add_row4_i16<KQ>(base(0, s), cs, d);
        add_row4_i16<KQ>(base(1, o), co, d);
        if (v0) add_row4_i16<KQ>(base(2, neg0), c0, d);
        if (v1) add_row4_i16<KQ>(base(3, neg1), c1, d);
      }
      // relation sums: rows of rw words; int32x2 (two words per quad) when a
      // hot relation's batch total could pass 16 bits
      unsigned long long* rrow = racc + (size_t)p * a.R.rw;
#pragma unroll
      for (int m = 0; m < KQ; ++m) {
        const int q = 64 * m + l;
        if (q < nq) {
          if (W32) {
            atomicAdd(rrow + 2 * q, pack_i32x2(cr[m].x, cr[m].y));
            atomicAdd(rrow + 2 * q + 1, pack_i32x2(cr[m].z, cr[m].w));
          } else {
            atomicAdd(rrow + q, pack_i16x4(cr[m]));
          }
        }
      }
    }
    if (a.trace) {   // stamp after issue (no drain: the trace must not slow the launch)
      if (l == 0) {
        unsigned long long* tr = a.trace + 2 + 6 * (size_t)w;
        tr[0] = tt[0]; tr[1] = tt[1]; tr[2] = tt[2]; tr[3] = tt[3]; tr[4] = now_10ns();
        tr[5] = pend | ((unsigned long long)(v0 + v1 > 0) << 8);
      }
    }
  }
  if (l == 0 && nv) {
    atomicAdd(shard_of(a.nviol_shards), nv);
    if (a.stats_viol) atomicAdd(shard_of(a.stats_viol), nv);
  }
}

// ---- fused runner (round 5): nothing waits ----
//
// k_pipe_batch gives each launch apply waves for batch b-1's rows (dispatched
// first) and scoring waves that WAIT for any row batch b-1 touched (claim /
// done word / write-through re-read); its per-wave traces put the scoring
// waves' start at ~3.2 us (p50) behind ~1.4k apply workgroups, with ~30% of
// them settling a pending row.  In k_pipe_fused no wave waits:
//
//   * a scoring wave that reads a row batch b-1 touched computes that row's
//     update itself from its pre-update value, state, sums and count
//     (row_update_s, the applier's arithmetic: the same bits) -- the
//     pre-update value stays readable all launch because the applier writes
//     the row's OTHER buffer (FusedTab); the buffer holding a row is its meta
//     word z (launch id and buffer of the last write), loaded with its pending
//     mark in the round trip that loads the row from both buffers;
//   * so the scoring items go first (one per positive), then one item per
//     four slot records of launch g-1 (claimed through the row's meta word,
//     applied into the other buffer) that also zeroes the rows of launch g-2's
//     four slot records (the accumulator copy launch g+1 adds into).
//
// Relation rows as in k_pipe_batch (double-buffered and recomputed by every
// scoring wave; items 0..nR-1 publish them for the next launch).  After a
// runner's epochs k_fused_fin copies rows living in buffer 1 back into the
// caller's tables and clears the meta words.
//
// Measured (WN18, same box): d = 50 on its 64-wide padded tables 10.52 ->
// 10.08 us per launch; d = 200 9.78 vs 8.48 us for k_pipe_batch, which stays
// the default there -- at 800-B rows the second buffer's loads and the
// rotating copies cost more than the waits save (the one-role form, every item
// scoring, applying and zeroing, measured 11.45 us; loading the rows after
// their meta words instead of from both buffers, 10.61 us).

template <int KQ, bool E8>
__device__ __forceinline__ void load_sums_raw(const void* S, int row, int d,
                                              unsigned long long (&sv)[KQ]) {
  const int l = lane_id(), nq = d >> 2;
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l, qc = q < nq ? q : nq - 1;
    if (E8)
      sv[m] = reinterpret_cast<const unsigned int*>(S)[(size_t)row * nq + qc];
    else
      sv[m] = reinterpret_cast<const unsigned long long*>(S)[(size_t)row * nq + qc];
  }
}

// packed sums -> floats (exact small integers), zero past the row
template <int KQ, bool E8>
__device__ __forceinline__ void decode_sums(const unsigned long long (&sv)[KQ], int d,
                                            float4 (&sm)[KQ]) {
  const int l = lane_id(), nq = d >> 2;
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const bool in = 64 * m + l < nq;
    sm[m] = E8 ? unpack_i8x4_sum(in ? (unsigned int)sv[m] : 0u) : unpack_i16x4(in ? sv[m] : 0ull);
  }
}

// P (and A) of a row from buffer b, clamped unconditional loads
template <int KQ>
__device__ __forceinline__ void load_pa(const FusedTab& F, int b, int row, int d,
                                        float4 (&p)[KQ], float4 (&av)[KQ]) {
  const int l = lane_id(), nq = d >> 2;
  const float4* prow = reinterpret_cast<const float4*>(F.P[b] + (size_t)row * d);
  const float4* arow = reinterpret_cast<const float4*>((F.A[0] ? F.A[b] : F.P[b]) + (size_t)row * d);
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l, qc = q < nq ? q : nq - 1;
    p[m] = prow[qc];
    av[m] = F.A[0] ? arow[qc] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
}

template <int KQ, bool E8>
__device__ __forceinline__ void zero_sums_row(void* S, int* cnt, int row, int d) {
  const int l = lane_id(), nq = d >> 2;
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l;
    if (q < nq) {
      if (E8)
        reinterpret_cast<unsigned int*>(S)[(size_t)row * nq + q] = 0u;
      else
        reinterpret_cast<unsigned long long*>(S)[(size_t)row * nq + q] = 0ull;
    }
  }
  if (l == 0) cnt[row] = 0;
}

template <int KQ, bool W32, bool E8>
__global__ __launch_bounds__(SKGE_PIPE_WG) void k_pipe_fused(PipeArgs a) {
  const int wpb = blockDim.x >> 6;
  const int l = lane_id();
  const int d = a.d, nq = d >> 2;
  const int rcw = W32 ? 2 * nq : nq;   // relation accumulator: the count word
  const int g = launch_id(a), gp = g - 1;
  const int k0 = g % 3, k1 = (g + 2) % 3, k2 = (g + 1) % 3;   // copies of launches g, g-1, g-2
  const int rd = a.b & 1;                    // relation buffer holding R_{b-1}
  const int rw = a.b < a.nb1 ? rd ^ 1 : 0;   // ... receiving R_b (the flush: the caller's)
  const int ra_prev = (g - 1) % 3, ra_cur = g % 3, ra_old = (g - 2) % 3;
  const bool flush = a.b == a.nb1;
  const bool ada = a.F.A[0] != nullptr;
  const int nR = a.R.rows;
  const int w0 = (int)blockIdx.x * wpb + (int)(threadIdx.x >> 6);
  const int nwv = (int)gridDim.x * wpb;
  if (flush && w0 == 0) fold_shards(a.nviol_shards, a.nviol_total);   // the epoch's violations
  unsigned long long* const racc0 = opaque_ptr(a.R.acc[ra_cur]);
  const size_t rrep = (size_t)a.R.rows * a.R.rw;   // words per relation replica
  const int rmask = a.R.reps - 1;
  void* const esum = opaque_ptr(a.F.sum[k0]);
  const __amdgpu_buffer_rsrc_t rec_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int4*>(a.rec + a.start), 0, a.count * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t rec1_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int*>(a.rec_n1 + a.start), 0, a.count * 4, 0x00020000);
  int nv = 0, napp = 0;
  for (int item = w0; item < nR + a.nwork; item += nwv) {
    if (item < nR) {   // relation row `item`: R_b for the next launch, old sums cleared
      rel_publish<KQ, W32>(a, item, rd, rw, ra_prev, ra_old);
      continue;
    }
    // the item's positive (the scoring items first: nothing waits for the
    // others, so they need not start early) or slot group (four slot records
    // applied, four zeroed)
    const int w = item - nR < a.count ? item - nR : -1;
    const int wa = item - nR < a.count ? -1 : item - nR - a.count;
    const bool sc = w >= 0 && w < a.count;
    unsigned long long tt[4] = {0ull, 0ull, 0ull, 0ull};
    if (a.trace) tt[0] = now_10ns();
    // ---- round trip 1: the record; slot records 4w..4w+3 of launch g-1 (lanes
    // 0-3: applied here) and of launch g-2 (lanes 4-7: their rows zeroed) ----
    u32x4 rx = {0u, 0u, 0u, 0u};
    int r1v = -1;
    if (sc) {
      rx = __builtin_amdgcn_raw_buffer_load_b128(rec_rs, w * 16, 0, 0);
      r1v = (int)__builtin_amdgcn_raw_buffer_load_b32(rec1_rs, w * 4, 0, 0);
    }
    int sl = -1;
    if (wa >= 0) {
      const int i = 4 * wa + (l & 3);
      const bool lo = l < 4;
      if (lo ? i < a.prev_slots : (l < 8 && i < a.pprev_slots))
        sl = (lo ? a.F.touched[k1] : a.F.touched[k2])[i];
    }
    __builtin_amdgcn_sched_barrier(0);
    const int s = uni((int)rx.x), o = uni((int)rx.y), p = uni((int)rx.z);
    const int neg0 = uni((int)rx.w), neg1 = uni(r1v);
    const int n0r = neg0 >= 0 ? neg0 : s, n1r = neg1 >= 0 ? neg1 : o;
    // launch g-2's rows: zero their sums and counts (copy k2: read by nobody in
    // this launch, added into by the next)
#pragma unroll
    for (int j = 4; j < 8; ++j) {
      const int v = __builtin_amdgcn_readlane(sl, j);
      if (v >= 0) zero_sums_row<KQ, E8>(a.F.sum[k2], a.F.cnt[k2], v & (SLOT_BUF - 1), d);
    }
    // ---- round trip 2: the scoring rows from both buffers, their meta words,
    // launch g-1's rows named by this item's slots (claim, value, state, sums,
    // count) and the relation row ----
    float4 x0[4][KQ], x1[4][KQ];
    int4 mt = make_int4(0, 0, 0, 0);
    if (sc) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int r = sel4(k, s, o, n0r, n1r);
        load_row4<KQ>(a.F.P[0], r, d, x0[k]);
        load_row4<KQ>(a.F.P[1], r, d, x1[k]);
      }
      if (l < 4) mt = a.F.meta[sel4(l, s, o, n0r, n1r)];
    }
    int won = 0, cl = 0;
    if (l < 4 && sl >= 0) {
      const int r = sl & (SLOT_BUF - 1);
      won = atomicExch(&a.F.meta[r].w, g) != g;   // the first of its slots to get here applies it
      cl = a.F.cnt[k1][r];
    }
    float4 ap[4][KQ], aa[4][KQ];
    unsigned long long asv[4][KQ];
    int arow[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      arow[j] = __builtin_amdgcn_readlane(sl, j);
      if (arow[j] >= 0) {
        const int r = arow[j] & (SLOT_BUF - 1), b = arow[j] >> 30;
        load_pa<KQ>(a.F, b, r, d, ap[j], aa[j]);
        load_sums_raw<KQ, E8>(a.F.sum[k1], r, d, asv[j]);
      }
    }
    float4 rp[KQ];
    if (sc) {
      float4 ra[KQ];
      int c;
      rel_row<KQ, W32>(a.R, p, d, rd, ra_prev, rp, ra, c);
    }
    if (a.trace) tt[1] = now_10ns();
    // where each scoring row lives, and which batch b-1 touched (lanes 0-3)
    const int pw = (gp & 1) ? mt.y : mt.x;
    const unsigned cur = (unsigned)mt.z;
    const int bn = ((int)(cur >> 1) == g) ? (int)((cur & 1u) ^ 1u) : (int)(cur & 1u);
    const uint64_t pend = sc ? (__ballot(l < 4 && pw == gp) & 0xfull) : 0ull;
    const uint64_t inb1 = __ballot(l < 4 && bn == 1) & 0xfull;
    float4 e[4][KQ];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int m = 0; m < KQ; ++m) e[k][m] = ((inb1 >> k) & 1ull) ? x1[k][m] : x0[k][m];
    // ---- round trip 3 (only rows batch b-1 touched): their state, sums, count ----
    float4 pa[4][KQ];
    unsigned long long psv[4][KQ];
    int pc = 0;
    if (pend) {
      if (l < 4 && ((pend >> l) & 1ull)) pc = a.F.cnt[k1][sel4(l, s, o, n0r, n1r)];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (!((pend >> k) & 1ull)) continue;
        const int r = sel4(k, s, o, n0r, n1r), b = (int)((inb1 >> k) & 1ull);
        if (ada) {
          const float4* arow = reinterpret_cast<const float4*>(a.F.A[b] + (size_t)r * d);
#pragma unroll
          for (int m = 0; m < KQ; ++m) {
            const int q = 64 * m + l;
            pa[k][m] = arow[q < nq ? q : nq - 1];
          }
        }
        load_sums_raw<KQ, E8>(a.F.sum[k1], r, d, psv[k]);
      }
    }
    // ---- apply launch g-1's claimed rows (beside round trip 3): into the
    // row's other buffer, then its meta word; nothing waits for them ----
    const uint64_t wonm = __ballot(won != 0) & 0xfull;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!((wonm >> j) & 1ull)) continue;
      const int c = __builtin_amdgcn_readlane(cl, j);
      const int r = arow[j] & (SLOT_BUF - 1), b = arow[j] >> 30;
      if (c > (E8 ? 127 : PACKED_MAX) && l == 0) atomicOr(a.err, ERR_PACKED);
      float4 sm[KQ];
      decode_sums<KQ, E8>(asv[j], d, sm);
      row_update_s<KQ>(a.E.u, c, d, sm, ap[j], aa[j]);
      store_row4<KQ>(a.F.P[b ^ 1], r, d, ap[j]);
      if (ada) store_row4<KQ>(a.F.A[b ^ 1], r, d, aa[j]);
      if (l == 0) a.F.meta[r].z = (g << 1) | (b ^ 1);
      if (flush) zero_sums_row<KQ, E8>(a.F.sum[k1], a.F.cnt[k1], r, d);   // nobody reads them again
      ++napp;
    }
    if (!sc) continue;
    // ---- the pending rows' updates, computed here (the same bits as the
    // applier's): the values batch b scores with ----
    if (pend) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (!((pend >> k) & 1ull)) continue;
        const int c = __builtin_amdgcn_readlane(pc, k);
        float4 sm[KQ], av[KQ];
        decode_sums<KQ, E8>(psv[k], d, sm);
#pragma unroll
        for (int m = 0; m < KQ; ++m) av[m] = ada ? pa[k][m] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        row_update_s<KQ>(a.E.u, c, d, sm, e[k], av);
      }
    }
    if (a.trace) tt[2] = now_10ns();
    float ps = 0.0f, n0 = 0.0f, n1 = 0.0f;
    float4 gp4[KQ], g0[KQ], g1[KQ];
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
#define SKGE_EL(X)                                                                    \
  {                                                                                   \
    const float vp = (e[0][m].X + rp[m].X) - e[1][m].X;   /* transe.py:32 */          \
    const float v0 = (e[2][m].X + rp[m].X) - e[1][m].X;                               \
    const float v1 = (e[0][m].X + rp[m].X) - e[3][m].X;                               \
    ps += fabsf(vp);                                                                  \
    n0 += fabsf(v0);                                                                  \
    n1 += fabsf(v1);                                                                  \
    gp4[m].X = signf_np(-((e[1][m].X - rp[m].X) - e[0][m].X)); /* transe.py:103,115 */ \
    g0[m].X = signf_np((e[1][m].X - rp[m].X) - e[2][m].X);     /* transe.py:104,117 */ \
    g1[m].X = signf_np((e[3][m].X - rp[m].X) - e[0][m].X);                            \
  }
      SKGE_EL(x)
      SKGE_EL(y)
      SKGE_EL(z)
      SKGE_EL(w)
#undef SKGE_EL
    }
    const float pscore = -wave_sum(ps);
    const float ns0 = -wave_sum(n0), ns1 = -wave_sum(n1);
    const int v0 = (neg0 >= 0 && ns0 + a.margin > pscore) ? 1 : 0;   // strict >, transe.py:73
    const int v1 = (neg1 >= 0 && ns1 + a.margin > pscore) ? 1 : 0;
    if (a.trace) tt[3] = now_10ns();
    unsigned long long* const racc = racc0 + (size_t)(w & rmask) * rrep;
    {
      // counts, slot records (with the buffer the row is in after this
      // launch) and pending marks of batch b
      const int cE = sel4(l, v0 + 2 * v1, 2 * v0 + v1, v0, v1);
      const int rE = sel4(l, s, o, neg0, neg1);
      if (l < 4) {
        const int bend = bn ^ (int)((pend >> l) & 1ull);
        a.F.touched[k0][4 * w + l] = cE > 0 ? (rE | (bend << 30)) : -1;
        if (cE > 0) {
          atomicAdd(a.F.cnt[k0] + rE, cE);
          reinterpret_cast<int*>(a.F.meta + rE)[g & 1] = g;
        }
      } else if (l == 4 && v0 + v1 > 0) {
        atomicAdd(racc + (size_t)p * a.R.rw + rcw, (unsigned long long)(2 * (v0 + v1)));
      }
    }
    if (v0 + v1 > 0) {
      nv += v0 + v1;
      const float fv0 = (float)v0, fv1 = (float)v1;
      float4 cs[KQ], co[KQ], c0[KQ], c1[KQ], cr[KQ];
#pragma unroll
      for (int m = 0; m < KQ; ++m) {
#define SKGE_CO(X)                                                   \
  cs[m].X = fv0 * gp4[m].X + fv1 * (gp4[m].X + g1[m].X);             \
  co[m].X = -(fv0 * (gp4[m].X + g0[m].X) + fv1 * gp4[m].X);          \
  c0[m].X = g0[m].X;                                                 \
  c1[m].X = -g1[m].X;                                                \
  cr[m].X = fv0 * (gp4[m].X + g0[m].X) + fv1 * (gp4[m].X + g1[m].X);
        SKGE_CO(x)
        SKGE_CO(y)
        SKGE_CO(z)
        SKGE_CO(w)
#undef SKGE_CO
      }
      if (E8) {
        unsigned int* es8 = reinterpret_cast<unsigned int*>(esum);
        acc_row4_i8<KQ>(es8, s, cs, d);
        acc_row4_i8<KQ>(es8, o, co, d);
        if (v0) acc_row4_i8<KQ>(es8, neg0, c0, d);
        if (v1) acc_row4_i8<KQ>(es8, neg1, c1, d);
      } else {
        Accum aE = {};
        aE.sum = reinterpret_cast<float*>(esum);
        acc_row4_i16<KQ>(aE, s, cs, d);
        acc_row4_i16<KQ>(aE, o, co, d);
        if (v0) acc_row4_i16<KQ>(aE, neg0, c0, d);
        if (v1) acc_row4_i16<KQ>(aE, neg1, c1, d);
      }
      unsigned long long* rrow = racc + (size_t)p * a.R.rw;
#pragma unroll
      for (int m = 0; m < KQ; ++m) {
        const int q = 64 * m + l;
        if (q < nq) {
          if (W32) {
            atomicAdd(rrow + 2 * q, pack_i32x2(cr[m].x, cr[m].y));
            atomicAdd(rrow + 2 * q + 1, pack_i32x2(cr[m].z, cr[m].w));
          } else {
            atomicAdd(rrow + q, pack_i16x4(cr[m]));
          }
        }
      }
    }
    if (a.trace && l == 0) {   // stamp after issue (no drain)
      unsigned long long* tr = a.trace + 2 + 6 * (size_t)w;
      tr[0] = tt[0]; tr[1] = tt[1]; tr[2] = tt[2]; tr[3] = tt[3]; tr[4] = now_10ns();
      tr[5] = pend | ((unsigned long long)(v0 + v1 > 0) << 8);
    }
  }
  if (l == 0) {
    if (nv) {
      atomicAdd(shard_of(a.nviol_shards), nv);
      if (a.stats_viol) atomicAdd(shard_of(a.stats_viol), nv);
    }
    if (napp && a.E.claims) atomicAdd(shard_of(a.E.claims), napp);
  }
}

// after a fused runner's epochs: rows whose current value is in buffer 1
// copied into buffer 0 (the caller's tables); the meta words are then cleared
// (hipMemsetAsync), so between runs every row lives in the caller's tables
__global__ __launch_bounds__(256) void k_fused_fin(FusedTab F, int rows, int d) {
  const int nq = d >> 2;
  const long long n = (long long)rows * nq;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / nq), q = (int)(i - (long long)r * nq);
    if (F.meta[r].z & 1) {
      const size_t off = (size_t)r * nq + q;
      reinterpret_cast<float4*>(F.P[0])[off] = reinterpret_cast<const float4*>(F.P[1])[off];
      if (F.A[0]) reinterpret_cast<float4*>(F.A[0])[off] = reinterpret_cast<const float4*>(F.A[1])[off];
    }
  }
}

__global__ void k_pipe_advance(uint64_t* ek) { *ek += 1; }

// Large TransE batches (RelTab::reps > 1): after batch launch g, fold the
// relation accumulator copy g % 3's replicas 1..reps-1 into replica 0 (the
// only one rel_row / rel_publish read) and zero them.  Packed integer sums
// add exactly in any order, so the result is bitwise the single-copy one.
// At nb = 2 on WN18 the ~25k violating positives of a batch add 1.6 KB each
// into 18 rows; one copy serialised those atomics on ~2k addresses
// (timing-only ablation without them: 0.370 -> 0.300 ms per epoch).
__global__ __launch_bounds__(256) void k_rel_fold(PipeArgs a) {
  const int g = launch_id(a);
  unsigned long long* acc = a.R.acc[g % 3];
  const size_t rrep = (size_t)a.R.rows * a.R.rw;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < rrep;
       i += (size_t)gridDim.x * blockDim.x) {
    unsigned long long s = acc[i];
    for (int k = 1; k < a.R.reps; ++k) {
      s += acc[k * rrep + i];
      acc[k * rrep + i] = 0ull;
    }
    acc[i] = s;
  }
}

// Data-parallel runners (skge_amd/dp.py): after the records of union batch b
// are all-gathered, each rank adds the OTHER ranks' positives -- union
// positions [0, count) outside its own slice [lo, hi), which its launch
// scored and added itself -- into batch b's accumulator copies exactly as a
// scoring wave of k_pipe_batch does (counts, slot records 4w+k, pending marks
// with batch b's launch id, exact packed entity sums, relation sums into
// replica w % reps): the next launch's A role then applies the union batch,
// bitwise as one GPU scoring all of it.  The header (s, o, p, s', o') comes
// from the epoch's records, which every rank draws alike; the record gives
// the violation flags and sign vectors.
template <int KQ, bool W32, bool E8>
__global__ __launch_bounds__(256) void k_pipe_dp_scatter(PipeArgs a, const uint32_t* __restrict__ recs) {
  const int wpb = blockDim.x >> 6;
  const int l = lane_id();
  const int d = a.d, nq = d >> 2;
  const int rcw = W32 ? 2 * nq : nq;
  const int g = launch_id(a);
  const int cp = a.b & 1;
  const int rw = pipe_dp_record_words(d);
  int* const cnt_cp = a.E.cnt[cp];
  int* const tch_cp = a.E.touched[cp];
  int* const pend_cp = a.E.pend[cp];
  int* const own_cp = a.E.own[cp];
  unsigned long long* const esum = a.E.sum[cp];
  unsigned long long* const racc0 = a.R.acc[g % 3];
  const size_t rrep = (size_t)a.R.rows * a.R.rw;
  const int rmask = a.R.reps - 1;
  const int nown = a.hi - a.lo, nrem = a.count - nown;
  for (int i = blockIdx.x * wpb + (threadIdx.x >> 6); i < nrem; i += gridDim.x * wpb) {
    const int w = i < a.lo ? i : i + nown;   // union position, outside [lo, hi)
    const int4 r4 = a.rec[a.start + w];
    const int s = __builtin_amdgcn_readfirstlane(r4.x);
    const int o = __builtin_amdgcn_readfirstlane(r4.y);
    const int p = __builtin_amdgcn_readfirstlane(r4.z);
    const int neg0 = __builtin_amdgcn_readfirstlane(r4.w);
    const int neg1 = __builtin_amdgcn_readfirstlane(a.rec_n1[a.start + w]);
    const uint32_t* in = recs + (size_t)w * rw;
    const int fl = (int)__builtin_amdgcn_readfirstlane(in[0]);
    const int v0 = fl & 1, v1 = (fl >> 1) & 1;
    unsigned long long* const racc = racc0 + (size_t)(w & rmask) * rrep;
    {   // (k_pipe_batch's commit, lanes 0-4)
      const int cE = sel4(l, v0 + 2 * v1, 2 * v0 + v1, v0, v1);
      const int rE = sel4(l, s, o, neg0, neg1);
      if (l < 4) {
        commit_slot(cnt_cp, tch_cp, rE, cE, 4 * w + l);
        if (cE > 0) {
          pend_cp[rE] = g;
          if (own_cp) own_cp[rE] = 4 * w + l;
        }
      } else if (l == 4 && v0 + v1 > 0) {
        atomicAdd(racc + (size_t)p * a.R.rw + rcw, (unsigned long long)(2 * (v0 + v1)));
      }
    }
    if (v0 + v1 == 0) continue;
    const float fv0 = (float)v0, fv1 = (float)v1;
    float4 cs[KQ], co[KQ], c0[KQ], c1[KQ], cr[KQ];
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      const int q = 64 * m + l;
      const uint32_t x = q < nq ? in[1 + q] : 0u;
      const float4 gp4 = untern4q(x & 0xFFu), g0 = untern4q((x >> 8) & 0xFFu),
                   g1 = untern4q((x >> 16) & 0xFFu);
#define SKGE_CO(X)                                             \
  cs[m].X = fv0 * gp4.X + fv1 * (gp4.X + g1.X);                \
  co[m].X = -(fv0 * (gp4.X + g0.X) + fv1 * gp4.X);             \
  c0[m].X = g0.X;                                              \
  c1[m].X = -g1.X;                                             \
  cr[m].X = fv0 * (gp4.X + g0.X) + fv1 * (gp4.X + g1.X);
      SKGE_CO(x)
      SKGE_CO(y)
      SKGE_CO(z)
      SKGE_CO(w)
#undef SKGE_CO
    }
    if (E8) {
      unsigned int* es8 = reinterpret_cast<unsigned int*>(esum);
      acc_row4_i8<KQ>(es8, s, cs, d);
      acc_row4_i8<KQ>(es8, o, co, d);
      if (v0) acc_row4_i8<KQ>(es8, neg0, c0, d);
      if (v1) acc_row4_i8<KQ>(es8, neg1, c1, d);
    } else {
      add_row4_i16<KQ>(esum + (size_t)s * nq, cs, d);
      add_row4_i16<KQ>(esum + (size_t)o * nq, co, d);
      if (v0) add_row4_i16<KQ>(esum + (size_t)neg0 * nq, c0, d);
      if (v1) add_row4_i16<KQ>(esum + (size_t)neg1 * nq, c1, d);
    }
    unsigned long long* rrow = racc + (size_t)p * a.R.rw;
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      const int q = 64 * m + l;
      if (q < nq) {
        if (W32) {
          atomicAdd(rrow + 2 * q, pack_i32x2(cr[m].x, cr[m].y));
          atomicAdd(rrow + 2 * q + 1, pack_i32x2(cr[m].z, cr[m].w));
        } else {
          atomicAdd(rrow + q, pack_i16x4(cr[m]));
        }
      }
    }
  }
}

// draw every negative of the epoch: one thread per positive, the same draws and
// first-accepted-try rule as k_transe_sample_grad (skge/sample.py:41-46).
// err (pipelined runners; nullptr elsewhere): once a launch has set an error
// bit (a wrapped packed sum, a wait that gave up) every later epoch draws no
// negatives -- no pair, no contribution, no row update -- so the tables are
// left as the failing epoch left them and the runner refuses further run()s
// once the error has been read (skge_pipe_runner_error)
__global__ void k_epoch_sample(const int* __restrict__ trip, long long T, int half, uint64_t seed,
                               const uint64_t* ekp, TripleSet set, int n_ent, int ntries,
                               int4* rec, int* rec_n1, const int* err) {
  const uint64_t ek = *ekp;
  if (err && *err) ntries = 0;
  const Perm pm = {(uint64_t)T, half, epoch_perm_key(seed, ek)};
  const uint64_t skey = epoch_sample_key(seed, ek);
  for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x; j < T;
       j += (long long)gridDim.x * blockDim.x) {
    const long long t = (long long)perm_index((uint64_t)j, pm);
    const int s = trip[3 * t], o = trip[3 * t + 1], p = trip[3 * t + 2];
    int neg0 = -1, neg1 = -1;
    for (int tr = 0; tr < ntries; ++tr) {
      const int c = draw(skey, j, 0, tr, n_ent);
      if (!set_contains(set, c, o, p)) {
        neg0 = c;
        break;
      }
    }
    for (int tr = 0; tr < ntries; ++tr) {
      const int c = draw(skey, j, 1, tr, n_ent);
      if (!set_contains(set, s, c, p)) {
        neg1 = c;
        break;
      }
    }
    rec[j] = make_int4(s, o, p, neg0);
    rec_n1[j] = neg1;
  }
}

int launch_epoch_sample(hipStream_t st, const int* trip, long long T, uint64_t seed,
                        const uint64_t* epoch_key, TripleSet set, int n_ent, int ntries,
                        int4* rec, int* rec_n1) {
  long long blocks = (T + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_epoch_sample, dim3((unsigned)blocks), dim3(256), 0, st, trip, T,
                     perm_half(T), seed, epoch_key, set, n_ent, ntries, rec, rec_n1, nullptr);
  SKGE_CHECK_LAUNCH("epoch sample");
  return SKGE_OK;
}

}  // namespace skge

using namespace skge;

// ---- pipelined runner ----
struct skge_pipe_runner {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  std::vector<void*> bufs;
  int* err = nullptr;
  int* stats = nullptr;            // [nlaunch][3] (profile only)
  // the epoch's launches
  const int* trip = nullptr;
  long long T = 0;
  int half = 0, n_ent = 0, ntries = 0, kq = 1;
  uint64_t seed = 0;
  uint64_t* epoch_key = nullptr;
  TripleSet set;
  int4* rec = nullptr;
  int* rec_n1 = nullptr;
  std::vector<PipeArgs> batch;     // nb1 batches + the flush
  std::vector<int> grid;
  bool w32 = false;                // int32x2 relation sums
  bool e8 = false;                 // int8x4 entity sums (SKGE_ACC_I8X4: per-batch counts <= 127)
  bool hole = false;               // HolE pairwise (k_hole_pipe, fp32 sums)
  bool fft = false;                // HolE: correlations in the frequency domain (skge_hole_fft.h)
  bool rfold = false;              // TransE: relation sums in replicas, k_rel_fold after each batch
  size_t lds = 0;                  // HolE: dynamic LDS per workgroup
  bool pair = false;               // HolE FFT, d = 200: two waves per positive (while 2 x B waves fit the chip)
  bool fused = false;              // TransE: k_pipe_fused (nothing waits; d <= 64 by default)
  bool invalid = false;            // an error bit was read or a launch failed: run() refuses
  bool dp = false;                 // data-parallel form (SKGE_PIPE_DP): driven launch by launch
  int n_rows = 0, d = 0;           // fused: the entity table's geometry (k_fused_fin)
  int nlaunch() const { return (int)batch.size() + 2; }
};

static void* dalloc(skge_pipe_runner* r, size_t bytes) {
  void* p = nullptr;
  if (hipMalloc(&p, bytes ? bytes : 4) != hipSuccess) return nullptr;
  r->bufs.push_back(p);
  if (hipMemset(p, 0, bytes ? bytes : 4) != hipSuccess) return nullptr;
  return p;
}

static void pipe_free(skge_pipe_runner* r) {
  (void)hipGetLastError();   // a failed allocation must not poison later launch checks
  if (!r) return;
  if (r->exec) (void)hipGraphExecDestroy(r->exec);
  if (r->graph) (void)hipGraphDestroy(r->graph);
  for (void* p : r->bufs) (void)hipFree(p);
  delete r;
}

static void launch_fused(const skge_pipe_runner* r, dim3 gr, hipStream_t st, const PipeArgs& a) {
  const dim3 bl(SKGE_PIPE_WG);
  if (r->e8) {
    if (r->w32) hipLaunchKernelGGL((k_pipe_fused<1, true, true>), gr, bl, 0, st, a);
    else hipLaunchKernelGGL((k_pipe_fused<1, false, true>), gr, bl, 0, st, a);
  } else {
    if (r->w32) hipLaunchKernelGGL((k_pipe_fused<1, true, false>), gr, bl, 0, st, a);
    else hipLaunchKernelGGL((k_pipe_fused<1, false, false>), gr, bl, 0, st, a);
  }
}

// k_pipe_batch: the instance for this runner's row width, sums and batch size
static void launch_pipe_batch(const skge_pipe_runner* r, dim3 gr, hipStream_t st,
                              const PipeArgs& a) {
#define SKGE_PB(K)                                                                        \
  do {                                                                                    \
    /* own marks: large batches (grouped owner-row apply); nhot: hot-row replicas */     \
    const bool gp_ = a.E.own[0] != nullptr, hot_ = a.E.nhot > 0;                          \
    const dim3 bl(gp_ ? PIPE_WG_GRP : SKGE_PIPE_WG);                      \
    if (r->e8) {                                                                          \
      if (gp_) {                                                                          \
        if (r->w32) hipLaunchKernelGGL((k_pipe_batch<K, true, true, true>), gr, bl, 0, st, a); \
        else hipLaunchKernelGGL((k_pipe_batch<K, false, true, true>), gr, bl, 0, st, a);  \
      } else {                                                                            \
        if (r->w32) hipLaunchKernelGGL((k_pipe_batch<K, true, true>), gr, bl, 0, st, a);  \
        else hipLaunchKernelGGL((k_pipe_batch<K, false, true>), gr, bl, 0, st, a);        \
      }                                                                                   \
    } else if (hot_) {                                                                    \
      if (gp_) {                                                                          \
        if (r->w32) hipLaunchKernelGGL((k_pipe_batch<K, true, false, true, true>), gr, bl, 0, st, a); \
        else hipLaunchKernelGGL((k_pipe_batch<K, false, false, true, true>), gr, bl, 0, st, a); \
      } else {                                                                            \
        if (r->w32) hipLaunchKernelGGL((k_pipe_batch<K, true, false, false, true>), gr, bl, 0, st, a); \
        else hipLaunchKernelGGL((k_pipe_batch<K, false, false, false, true>), gr, bl, 0, st, a); \
      }                                                                                   \
    } else if (gp_) {                                                                     \
      if (r->w32) hipLaunchKernelGGL((k_pipe_batch<K, true, false, true>), gr, bl, 0, st, a); \
      else hipLaunchKernelGGL((k_pipe_batch<K, false, false, true>), gr, bl, 0, st, a);   \
    } else {                                                                              \
      if (r->w32) hipLaunchKernelGGL((k_pipe_batch<K, true, false>), gr, bl, 0, st, a);   \
      else hipLaunchKernelGGL((k_pipe_batch<K, false, false>), gr, bl, 0, st, a);         \
    }                                                                                     \
  } while (0)
// the data-parallel instances (no hot rows in that form)
#define SKGE_PBD(K)                                                                       \
  do {                                                                                    \
    const bool gp_ = a.E.own[0] != nullptr;                                               \
    const dim3 bl(gp_ ? PIPE_WG_GRP : SKGE_PIPE_WG);                                      \
    if (gp_) {                                                                            \
      if (r->e8) {                                                                        \
        if (r->w32) hipLaunchKernelGGL((k_pipe_batch<K, true, true, true, false, true>), gr, bl, 0, st, a); \
        else hipLaunchKernelGGL((k_pipe_batch<K, false, true, true, false, true>), gr, bl, 0, st, a); \
      } else {                                                                            \
        if (r->w32) hipLaunchKernelGGL((k_pipe_batch<K, true, false, true, false, true>), gr, bl, 0, st, a); \
        else hipLaunchKernelGGL((k_pipe_batch<K, false, false, true, false, true>), gr, bl, 0, st, a); \
      }                                                                                   \
    } else {                                                                              \
      if (r->e8) {                                                                        \
        if (r->w32) hipLaunchKernelGGL((k_pipe_batch<K, true, true, false, false, true>), gr, bl, 0, st, a); \
        else hipLaunchKernelGGL((k_pipe_batch<K, false, true, false, false, true>), gr, bl, 0, st, a); \
      } else {                                                                            \
        if (r->w32) hipLaunchKernelGGL((k_pipe_batch<K, true, false, false, false, true>), gr, bl, 0, st, a); \
        else hipLaunchKernelGGL((k_pipe_batch<K, false, false, false, false, true>), gr, bl, 0, st, a); \
      }                                                                                   \
    }                                                                                     \
  } while (0)
  if (r->dp) {
    if (r->kq <= 1) SKGE_PBD(1);
    else if (r->kq <= 2) SKGE_PBD(2);
    else SKGE_PBD(4);
  } else {
    if (r->kq <= 1) SKGE_PB(1);
    else if (r->kq <= 2) SKGE_PB(2);
    else SKGE_PB(4);
  }
#undef SKGE_PBD
#undef SKGE_PB
}

// Enqueue one epoch: draw the negatives, nb1 batch launches, the flush, the
// key advance.  ev (optional, nlaunch + 1 events) brackets every launch;
// stats (optional) collects per-launch claim / violation counts.
static void enqueue_epoch(const skge_pipe_runner* r, hipStream_t st, hipEvent_t* ev, int* stats,
                          int trace_launch = -1, unsigned long long* trace = nullptr) {
  int i = 0;
  if (ev) (void)hipEventRecord(ev[i], st);
  {
    long long blocks = (r->T + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_epoch_sample, dim3((unsigned)blocks), dim3(256), 0, st, r->trip, r->T,
                       r->half, r->seed, (const uint64_t*)r->epoch_key, r->set, r->n_ent,
                       r->ntries, r->rec, r->rec_n1, (const int*)r->err);
  }
  ++i;
  if (ev) (void)hipEventRecord(ev[i], st);
  for (size_t k = 0; k < r->batch.size(); ++k, ++i) {
    PipeArgs a = r->batch[k];
    if (stats) {
      const int sh = NSHARD * SHARD_STRIDE;
      a.E.claims = stats + (3 * i) * sh;
      a.R.updated = stats + (3 * i + 1) * sh;
      a.stats_viol = stats + (3 * i + 2) * sh;
    }
    if (trace && i == trace_launch) a.trace = trace;
    if (r->hole) {
      launch_hole_pipe(km_for(a.d), r->pair, r->fft, dim3(r->grid[k]),
                       dim3(r->pair ? 128 : SKGE_PIPE_WG), r->lds, st, a);
    } else if (r->fused) {
      launch_fused(r, dim3(r->grid[k]), st, a);
    } else {
      launch_pipe_batch(r, dim3(r->grid[k]), st, a);
    }
    if (r->rfold && a.count > 0) {
      const size_t words = (size_t)a.R.rows * a.R.rw;
      if (r->hole)   // fp32 sums + an int count per row
        launch_rel_fold_f(dim3((unsigned)std::min<size_t>((2 * words + 255) / 256, 4096)), st, a);
      else
        hipLaunchKernelGGL(k_rel_fold, dim3((unsigned)std::min<size_t>((words + 255) / 256, 4096)),
                           dim3(256), 0, st, a);
    }
    if (ev) (void)hipEventRecord(ev[i + 1], st);
  }
  hipLaunchKernelGGL(k_pipe_advance, dim3(1), dim3(1), 0, st, r->epoch_key);
  if (ev) (void)hipEventRecord(ev[i + 1], st);
}

// Hot rows around a run: before the first launch g0 (from the epoch key) the
// caller's rows into hP / hA[(g0 - 1) & 1]; after the last (the flush, id
// g0 - 1 of the next epoch key) hP / hA[that & 1] back into the caller's
// tables and every replica copy cleared, so a run may start at any key.
__global__ __launch_bounds__(256) void k_hot_io(PipeTab t, int nb1, const uint64_t* ek, int d,
                                                int back) {
  const int g0 = (int)(*ek * (uint64_t)(nb1 + 1)) + 2;   // launch_id of batch 0
  const int b = (g0 - 1) & 1;
  const long long n = (long long)t.nhot * d;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int h = (int)(i / d), e = (int)(i - (long long)h * d);
    const size_t off = (size_t)t.hot_rows[h] * d + e;
    if (back) {
      t.P[off] = t.hP[b][i];
      if (t.A) t.A[off] = t.hA[b][i];
    } else {
      t.hP[b][i] = t.P[off];
      if (t.A) t.hA[b][i] = t.A[off];
    }
  }
  if (back) {
    const long long nw = (long long)t.nhot * HOT_REPS * t.hw, nc = (long long)t.nhot * HOT_REPS;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nw;
         i += (long long)gridDim.x * blockDim.x) {
      for (int k = 0; k < 3; ++k) t.hsum[k][i] = 0ull;
      if (i < nc)
        for (int k = 0; k < 3; ++k) t.hcnt[k][i] = 0;
    }
  }
}

static void hot_io(const skge_pipe_runner* r, hipStream_t st, bool back) {
  if (r->batch.empty() || r->batch[0].E.nhot == 0) return;
  const PipeArgs& a = r->batch[0];
  hipLaunchKernelGGL(k_hot_io, dim3(64), dim3(256), 0, st, a.E, a.nb1, a.epoch_key, a.d,
                     back ? 1 : 0);
}

// fused runner: every row back into the caller's tables (buffer 0), meta cleared
static void fused_finalize(const skge_pipe_runner* r, hipStream_t st) {
  if (!r->fused) return;
  const FusedTab& F = r->batch[0].F;
  const long long n = (long long)r->n_rows * (r->d / 4);
  const unsigned blocks = (unsigned)std::max(1ll, std::min((n + 255) / 256, 8192ll));
  hipLaunchKernelGGL(k_fused_fin, dim3(blocks), dim3(256), 0, st, F, r->n_rows, r->d);
  (void)hipMemsetAsync(F.meta, 0, (size_t)r->n_rows * sizeof(int4), st);
}

// Hot rows (PipeTab::hot): entities whose subject / object occurrences in the
// KG put them in >= HOT_MIN slots of an average batch and >= HOT_REL times the
// average row's -- the hubs of a skewed KG, pending for most scoring waves and
// whose per-batch atomics otherwise serialise on one row.  The HOT_MAX most
// frequent get replicated sums.  Returns false on an allocation failure.
__global__ void k_ent_occ(const int* __restrict__ trip, long long T, int* occ) {
  for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x; j < T;
       j += (long long)gridDim.x * blockDim.x) {
    atomicAdd(occ + trip[3 * j], 1);
    atomicAdd(occ + trip[3 * j + 1], 1);
  }
}

static bool find_hot_rows(skge_pipe_runner* r, hipStream_t st, PipeTab& t, const int* trip,
                          long long T, int nb1, int N, int d, int row_words) {
  t.hot = t.hot_rows = nullptr;
  t.nhot = 0;
  int* occ = nullptr;
  if (hipMalloc(&occ, (size_t)N * 4) != hipSuccess) return false;
  std::vector<int> h(N);
  const unsigned blocks = (unsigned)std::max(1ll, std::min((T + 255) / 256, 4096ll));
  bool ok = hipMemsetAsync(occ, 0, (size_t)N * 4, st) == hipSuccess;
  hipLaunchKernelGGL(k_ent_occ, dim3(blocks), dim3(256), 0, st, trip, T, occ);
  ok = ok && hipMemcpyAsync(h.data(), occ, (size_t)N * 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipStreamSynchronize(st) == hipSuccess;
  (void)hipFree(occ);
  if (!ok) return false;
  // expected slots per batch = occurrences / nb1; the average row's: 2T / N / nb1
  const double bar = std::max((double)HOT_MIN * nb1, (double)HOT_REL * 2.0 * (double)T / N);
  std::vector<std::pair<int, int>> cand;   // (occurrences, row)
  for (int i = 0; i < N; ++i)
    if ((double)h[i] >= bar) cand.push_back({h[i], i});
  if (cand.empty()) return true;
  std::sort(cand.begin(), cand.end(), [](const std::pair<int, int>& x, const std::pair<int, int>& y) {
    return x.first != y.first ? x.first > y.first : x.second < y.second;
  });
  if ((int)cand.size() > HOT_MAX) cand.resize(HOT_MAX);
  const int nh = (int)cand.size();
  std::fill(h.begin(), h.end(), -1);
  std::vector<int> rows(nh);
  for (int j = 0; j < nh; ++j) {
    rows[j] = cand[j].second;
    h[rows[j]] = j;
  }
  t.hw = (row_words + 15) / 16 * 16;   // 8-B words per replica row: whole 128-B lines
  int* dh = (int*)dalloc(r, (size_t)N * 4);
  int* dr = (int*)dalloc(r, (size_t)nh * 4);
  bool got = dh && dr;
  for (int k = 0; k < 3; ++k) {
    t.hsum[k] = (unsigned long long*)dalloc(r, (size_t)nh * HOT_REPS * t.hw * 8);
    t.hcnt[k] = (int*)dalloc(r, (size_t)nh * HOT_REPS * 4);
    got = got && t.hsum[k] && t.hcnt[k];
  }
  for (int k = 0; k < 2; ++k) {
    t.hP[k] = (float*)dalloc(r, (size_t)nh * d * 4);
    t.hA[k] = t.A ? (float*)dalloc(r, (size_t)nh * d * 4) : nullptr;
    got = got && t.hP[k] && (!t.A || t.hA[k]);
  }
  if (!got ||
      hipMemcpy(dh, h.data(), (size_t)N * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dr, rows.data(), (size_t)nh * 4, hipMemcpyHostToDevice) != hipSuccess)
    return false;
  t.hot = dh;
  t.hot_rows = dr;
  t.nhot = nh;
  return true;
}

static skge_pipe_runner_t* pipe_create(void* stream, const skge_table_t* ent,
                                       const skge_table_t* rel, int d, const int* trip, int64_t T,
                                       const void* set, int64_t set_capacity, int nbatches,
                                       uint64_t seed, uint64_t* epoch_key, float margin,
                                       int ntries, int* nviol_total, int flags, bool hole, int af) {
  if (flags & ~SKGE_PIPE_DP) {
    set_error("pipelined runner: unknown flags %d", flags);
    return nullptr;
  }
  const bool dp = (flags & SKGE_PIPE_DP) != 0;
  if (dp && hole) {
    set_error("pipelined runner: the data-parallel form is TransE-L1 only");
    return nullptr;
  }
  if (!ent || !rel) {
    set_error("pipelined runner: NULL table");
    return nullptr;
  }
  skge_table_t relc = *rel;   // the relation encoding is the runner's own (checked below)
  if (relc.acc_mode == SKGE_ACC_I32X2) relc.acc_mode = SKGE_ACC_I16X4;
  skge_table_t entc = *ent;   // int8x4 entity sums: the runner's own encoding too
  if (entc.acc_mode == SKGE_ACC_I8X4) entc.acc_mode = SKGE_ACC_I16X4;
  if (check_table(&entc, "ent", true) || check_table(&relc, "rel", true)) return nullptr;
  if (hole) {   // HolE: fp32 sums, quad rows (d % 4 == 0, d <= 256)
    if (ent->acc_mode != SKGE_ACC_F32 || rel->acc_mode != SKGE_ACC_F32 || d % 4 || d < 4 ||
        d > 256 || ent->width != d || rel->width != d || ent->acc_touched == nullptr ||
        rel->acc_touched != nullptr || rel->acc_replicas > 1 || ent->acc_replicas > 1 ||
        ent->gate || rel->gate || af < 0 || af > 3) {
      set_error("pipelined HolE runner: needs fp32 accumulators (entity table with slot "
                "records, dense single-copy relation table), d %% 4 == 0, 4 <= d <= 256, no "
                "gates");
      return nullptr;
    }
  } else if ((ent->acc_mode != SKGE_ACC_I16X4 && ent->acc_mode != SKGE_ACC_I8X4) ||
      (rel->acc_mode != SKGE_ACC_I16X4 && rel->acc_mode != SKGE_ACC_I32X2) || d % 4 || d > 1024 ||
      ent->width != d || rel->width != d || ent->acc_touched == nullptr ||
      rel->acc_touched != nullptr || rel->acc_replicas > 1 || ent->acc_replicas > 1 ||
      ent->gate || rel->gate) {
    set_error("pipelined runner: needs a packed (SKGE_ACC_I16X4) entity table with slot "
              "records, a dense single-copy SKGE_ACC_I16X4 / SKGE_ACC_I32X2 relation table, "
              "d %% 4 == 0, no gates");
    return nullptr;
  }
  if (!trip || !set || !epoch_key || T <= 0 || nbatches < 1 || nbatches > T || !stream ||
      set_capacity < 4 || (set_capacity & (set_capacity - 1)) || ntries < 1) {
    set_error("pipelined runner: bad arguments");
    return nullptr;
  }
  // batch geometry of StochasticTrainer._optim (skge/base.py:1246-1268)
  const int64_t bs = T / nbatches;
  if (4 * bs > ent->touched_cap || 4 * bs > (1ll << 30)) {
    set_error("pipelined runner: batch too large for the slot capacity");
    return nullptr;
  }
  std::vector<std::pair<int64_t, int64_t>> batches;
  for (int64_t s0 = 0; s0 < T; s0 += bs) batches.push_back({s0, (s0 + bs <= T) ? bs : T - s0});
  const int nb1 = (int)batches.size();
  skge_pipe_runner* r = new skge_pipe_runner();
  r->hole = hole;
  r->dp = dp;
  // HolE at d = 200 in the FFT form: two waves per positive (the pair form)
  // while the batch's 2 x B scoring waves fit the chip's 4-wave-per-SIMD
  // residency.  WN18 d = 200, same box: nb = 100 93.7 -> 106.7 M triples/s
  // (14.6 -> 12.8 us per launch); nb = 2 (70k positives per launch) 157 ->
  // 142 M, so off there
  int64_t maxb = 0;
  for (const auto& bt : batches) maxb = std::max(maxb, bt.second);
  const bool hole_pair = hole && hole_use_fft(d) && d == 200 && 2 * maxb <= 4 * 4 * 256;
  r->e8 = !hole && ent->acc_mode == SKGE_ACC_I8X4;
  const int nq = d / 4;
  const int N = ent->rows;
  // large batches (more than 16k slot records): owner marks, k_pipe_batch's A
  // role scans its slots 64 at a time
  const bool grouped = !hole && 4 * bs > 4 * 4096;
  // TransE below that: k_pipe_fused for rows of up to 64 floats (WN18 d = 50
  // on its 64-wide padded tables: 10.52 -> 10.08 us per launch, same box),
  // k_pipe_batch above (d = 200: 8.48 vs 9.78 us -- at 800-B rows the fused
  // kernel's second-buffer loads and rotating copies cost more than its
  // waits save).  SKGE_PIPE_FUSED=0 / 1 forces either (d <= 256).
  {
    const char* fe = getenv("SKGE_PIPE_FUSED");
    const bool ok = !hole && !grouped && nq <= 64 && (long long)N < SLOT_BUF;
    r->fused = ok && !dp && (fe ? atoi(fe) != 0 : nq <= 16);
  }
  PipeArgs a = {};
  auto upd = [](const skge_table_t* s) {
    UpdParams u;
    u.opt = s->opt;
    u.post = s->post;
    u.lr = s->lr;
    u.rin = s->rin;
    u.rout = s->rout;
    u.fdiv = s->fixed_div;
    return u;
  };
  bool ok = true;
  {
    PipeTab& t = a.E;
    t.P = ent->param;
    t.A = ent->opt == SKGE_ADAGRAD ? ent->state : nullptr;
    t.u = upd(ent);
    t.claims = nullptr;
    t.err = nullptr;   // set below, once r->err exists
    t.sum[0] = reinterpret_cast<unsigned long long*>(ent->acc_sum);
    t.cnt[0] = ent->acc_cnt;
    t.touched[0] = ent->acc_touched;
    if (r->fused) {
      // the second row buffer, the other two accumulator copies, the meta words
      FusedTab& F = a.F;
      const size_t sb = (size_t)N * nq * (r->e8 ? 4 : 8);
      F.P[0] = ent->param;
      F.P[1] = (float*)dalloc(r, (size_t)N * d * 4);
      F.A[0] = t.A;
      F.A[1] = F.A[0] ? (float*)dalloc(r, (size_t)N * d * 4) : nullptr;
      F.sum[0] = ent->acc_sum;
      F.cnt[0] = ent->acc_cnt;
      F.touched[0] = ent->acc_touched;
      for (int k = 1; k < 3; ++k) {
        F.sum[k] = dalloc(r, sb);
        F.cnt[k] = (int*)dalloc(r, (size_t)N * 4);
        F.touched[k] = (int*)dalloc(r, (size_t)4 * bs * 4);
        ok = ok && F.sum[k] && F.cnt[k] && F.touched[k];
      }
      F.meta = (int4*)dalloc(r, (size_t)N * sizeof(int4));
      ok = ok && F.P[1] && (!F.A[0] || F.A[1]) && F.meta;
      r->n_rows = N;
      r->d = d;
    } else {
      // a second accumulator copy, slot records, batch marks, done words
      t.done = (int*)dalloc(r, (size_t)N * 4);
      t.sum[1] = (unsigned long long*)dalloc(r, (size_t)N * nq * (hole ? 16 : (r->e8 ? 4 : 8)));
      t.cnt[1] = (int*)dalloc(r, (size_t)N * 4);
      t.touched[1] = (int*)dalloc(r, (size_t)4 * bs * 4);
      t.pend[0] = (int*)dalloc(r, (size_t)N * 4);
      t.pend[1] = (int*)dalloc(r, (size_t)N * 4);
      ok = ok && t.done && t.sum[1] && t.cnt[1] && t.touched[1] && t.pend[0] && t.pend[1];
      if (grouped) {
        t.own[0] = (int*)dalloc(r, (size_t)N * 4);
        t.own[1] = (int*)dalloc(r, (size_t)N * 4);
        ok = ok && t.own[0] && t.own[1];
      }
      // (the data-parallel form keeps every row in the tables: no hot rows;
      // HolE: the pair form only, fp32 sums of d floats per replica row)
      if (ok && !r->e8 && !dp && (!hole || (hole_pair && SKGE_HPIPE_HOT)))
        ok = find_hot_rows(r, as_stream(stream), t, trip, T, nb1, N, d, hole ? d / 2 : nq);
    }
    RelTab& q = a.R;
    const int M = rel->rows;
    const bool ada = rel->opt == SKGE_ADAGRAD;
    q.rows = M;
    // HolE (fp32 sums, float atomics): at large batches every relation row
    // takes thousands of adds per launch, which serialise on its addresses;
    // spread them over replicas (one per ~2k positives, <= 32; 1 at nb = 100)
    q.reps = 1;
    if (hole)
      while (q.reps < 32 && (long long)q.reps * 2048 < bs) q.reps *= 2;
    if (hole && getenv("SKGE_HPIPE_RREPS")) q.reps = std::max(1, atoi(getenv("SKGE_HPIPE_RREPS")));
    // TransE, large batches (the A role's owner-mark regime): the same spread,
    // one replica per ~256 expected adds into a row (bs / M), <= 16, folded by
    // k_rel_fold after every batch launch (WN18 nb = 2: 16; nb = 100: 1)
    if (grouped) {
      const long long per_row = bs / std::max(1, M);
      while (q.reps < 16 && (long long)q.reps * 256 < per_row) q.reps *= 2;
    }
    r->rfold = q.reps > 1;
    q.folded = r->rfold ? 1 : 0;
    r->w32 = rel->acc_mode == SKGE_ACC_I32X2;
    // 8-B words per relation row: sums + count, whole 128-B lines (HolE: d
    // floats, then the count as an int)
    q.rw = hole ? ((d + 2) / 2 + 15) / 16 * 16 : ((r->w32 ? 2 * nq : nq) + 1 + 15) / 16 * 16;
    q.u = upd(rel);
    q.updated = nullptr;
    q.P[0] = rel->param;
    q.P[1] = (float*)dalloc(r, (size_t)M * d * 4);
    q.A[0] = ada ? rel->state : nullptr;
    q.A[1] = ada ? (float*)dalloc(r, (size_t)M * d * 4) : nullptr;
    for (int k = 0; k < 3; ++k)
      q.acc[k] = (unsigned long long*)dalloc(r, (size_t)q.reps * M * q.rw * 8);
    ok = ok && q.P[1] && (!ada || q.A[1]) && q.acc[0] && q.acc[1] && q.acc[2];
  }
  r->rec = (int4*)dalloc(r, (size_t)T * sizeof(int4));
  r->rec_n1 = (int*)dalloc(r, (size_t)T * 4);
  r->err = (int*)dalloc(r, 4);
  r->stats = (int*)dalloc(r, (size_t)(nb1 + 3) * 3 * NSHARD * SHARD_STRIDE * 4);
  int* vsh = (int*)dalloc(r, (size_t)NSHARD * SHARD_STRIDE * 4);
  if (!ok || !r->rec || !r->rec_n1 || !r->err || !r->stats || !vsh) {
    set_error("pipelined runner: device allocation failed");
    pipe_free(r);
    return nullptr;
  }
  r->trip = trip;
  r->T = T;
  r->half = perm_half(T);
  r->n_ent = N;
  r->ntries = ntries;
  r->seed = seed;
  r->epoch_key = epoch_key;
  r->set.slots = (const int4*)set;
  r->set.filter = (const uint32_t*)((const int4*)set + set_capacity);
  r->set.mask = (uint64_t)(set_capacity - 1);
  r->set.fmask = (uint64_t)(8 * set_capacity - 1);
  r->kq = (nq + 63) / 64;
  a.rec = r->rec;
  a.rec_n1 = r->rec_n1;
  a.nb1 = nb1;
  a.epoch_key = epoch_key;
  a.d = d;
  a.margin = margin;
  a.nviol_total = nviol_total;
  a.nviol_shards = vsh;
  a.stats_viol = nullptr;
  a.trace = nullptr;
  a.err = r->err;
  a.E.err = r->err;
  a.af = af;
  r->fft = hole && hole_use_fft(d);
  {
    r->pair = hole_pair;
    // the relation row's loads and update on wave 1 (3 rows each; same box,
    // two rounds: 103.8 -> 104.6 M triples/s)
    a.pair_r1 = 1;
  }
  a.tw = r->fft ? hole_fft_table(d) : nullptr;
  if (r->fft && !a.tw) {
    set_error("pipelined runner: HolE FFT twiddle table allocation failed");
    pipe_free(r);
    return nullptr;
  }
  r->lds = !hole ? 0
           : r->pair ? hole_fft_lds_bytes(d, 1)
           : r->fft ? hole_fft_lds_bytes(d, SKGE_PIPE_WG / 64)
                    : (size_t)(SKGE_PIPE_WG / 64) * hole_pos_lds_floats(d) * sizeof(float);
  const int WPB = r->pair ? 2 : (grouped ? PIPE_WG_GRP : SKGE_PIPE_WG) / 64;
  for (int b = 0; b <= nb1; ++b) {   // b == nb1: flush of the last batch (no scoring)
    a.b = b;
    a.start = b < nb1 ? batches[b].first : 0;
    a.count = b < nb1 ? (int)batches[b].second : 0;
    a.lo = 0;
    a.hi = a.count;
    a.dprec = nullptr;
    const int cprev = b >= 1 ? (int)batches[b - 1].second : 0;
    a.prev_slots = 4 * cprev;
    if (r->fused) {
      // one kind of wave: relation rows, then max(this, the previous and the
      // pre-previous batch's positives) work items.  The epoch starts clean (the
      // flush zeroes both copies it leaves), so the first two launches have no
      // pre-previous slots to zero
      const int cpp = b >= 2 ? (int)batches[b - 2].second : 0;
      a.pprev_slots = 4 * cpp;
      a.nwork = a.count + std::max(cprev, cpp);   // scoring items, then slot groups
      a.nA = 0;
      r->batch.push_back(a);
      r->grid.push_back(std::max(1, (rel->rows + a.nwork + WPB - 1) / WPB));
      continue;
    }
    // A role: every relation row, then the previous batch's entity slots
    // (owner marks: 64-slot groups)
    const int a_items = rel->rows + a.E.nhot +
                        (hole ? 4 * cprev
                         : grouped ? (4 * cprev + 63) / 64 : 4 * cprev);
    // HolE: the apply waves loop over their items within the residency the
    // scoring waves leave (direct form: 2 waves per SIMD at ~180 VGPRs; FFT: 4
    // -- caps 150 / 250 / 400 / 600 / 800 / 1100 on WN18 d = 200: 74.7 / 77.6 /
    // 80.5 / 81.7 / 75.4 / 70.5 M triples/s; the flush has the chip to itself)
    // (pair: two waves per positive, one positive per workgroup)
    auto nBwaves = [&](long long cnt) { return r->pair ? 2 * cnt : (cnt + WPB - 1) / WPB * WPB; };
    const int occ = r->pair ? std::max(4, HPIPE_OCC) : r->fft ? 4 : HPIPE_OCC;
    int a_cap = hole && b < nb1 ? std::max(1, (occ * 4 * 256 - (int)nBwaves(batches[b].second)) / WPB - 8) : 16384;
    // (large batches: more scoring waves than the chip holds -- they run in
    // rounds anyway -- so the apply waves get a fixed share instead of the
    // residency left over, which would be none: nb = 2 on WN18 had 4 apply
    // waves for 283k slot records, 42 ms per epoch)
    if (hole && b < nb1 && (long long)nBwaves(batches[b].second) > occ * 4 * 256)
      a_cap = std::max(a_cap, 256);
    a.nA = std::max(1, std::min((a_items + WPB - 1) / WPB, std::min(a_cap, 16384)));
    const int nBb = r->pair ? std::max(1, std::min(a.count, 2 * 16384))
                            : std::max(1, std::min((a.count + WPB - 1) / WPB, 16384));
    r->batch.push_back(a);
    r->grid.push_back(a.nA + (a.count > 0 ? nBb : 0));
  }
  hipStream_t st = as_stream(stream);
  if (dp) {   // driven launch by launch by the caller (skge_pipe_runner_dp_*), no graph
    if (hipStreamSynchronize(st) != hipSuccess) {
      set_error("hipStreamSynchronize failed");
      pipe_free(r);
      return nullptr;
    }
    return r;
  }
  if (hipStreamSynchronize(st) != hipSuccess ||
      hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    set_error("hipStreamBeginCapture failed");
    pipe_free(r);
    return nullptr;
  }
  enqueue_epoch(r, st, nullptr, nullptr);
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(st, &g);
  if (e != hipSuccess || hipGetLastError() != hipSuccess) {
    set_error("pipelined runner capture failed: %s", hipGetErrorString(e));
    if (g) (void)hipGraphDestroy(g);
    pipe_free(r);
    return nullptr;
  }
  r->graph = g;
  if (hipGraphInstantiate(&r->exec, g, nullptr, nullptr, 0) != hipSuccess) {
    set_error("hipGraphInstantiate failed");
    pipe_free(r);
    return nullptr;
  }
  return r;
}

extern "C" skge_pipe_runner_t* skge_pipe_runner_create_ex(
    void* stream, const skge_table_t* ent, const skge_table_t* rel, int d, const int* trip,
    int64_t T, const void* set, int64_t set_capacity, int nbatches, uint64_t seed,
    uint64_t* epoch_key, float margin, int ntries, int* nviol_total, int flags) {
  return pipe_create(stream, ent, rel, d, trip, T, set, set_capacity, nbatches, seed, epoch_key,
                     margin, ntries, nviol_total, flags, false, 0);
}

extern "C" skge_pipe_runner_t* skge_hole_pipe_runner_create(
    void* stream, int af, const skge_table_t* ent, const skge_table_t* rel, int d,
    const int* trip, int64_t T, const void* set, int64_t set_capacity, int nbatches,
    uint64_t seed, uint64_t* epoch_key, float margin, int ntries, int* nviol_total) {
  return pipe_create(stream, ent, rel, d, trip, T, set, set_capacity, nbatches, seed, epoch_key,
                     margin, ntries, nviol_total, 0, true, af);
}

extern "C" skge_pipe_runner_t* skge_pipe_runner_create(void* stream, const skge_table_t* ent,
                                                       const skge_table_t* rel, int d,
                                                       const int* trip, int64_t T, const void* set,
                                                       int64_t set_capacity, int nbatches,
                                                       uint64_t seed, uint64_t* epoch_key,
                                                       float margin, int ntries,
                                                       int* nviol_total) {
  return skge_pipe_runner_create_ex(stream, ent, rel, d, trip, T, set, set_capacity, nbatches,
                                    seed, epoch_key, margin, ntries, nviol_total, 0);
}

// A runner whose error word was found set (skge_pipe_runner_error), or whose
// epoch launch failed, is invalid: the caller's tables hold whatever the
// failing epoch left (a wrapped sum applied, a row scored stale), and every
// later run() / profile() is refused.  (Epochs already queued behind the
// failing one draw no negatives, so they change nothing: k_epoch_sample.)
static int refuse_invalid(const skge_pipe_runner* r) {
  set_error("pipelined runner: an earlier epoch failed (error word set or launch failed); the "
            "tables hold that epoch's partial updates and the runner refuses further runs -- "
            "restore the parameters and build a new runner");
  (void)r;
  return SKGE_EINVAL;
}

extern "C" int skge_pipe_runner_run(skge_pipe_runner_t* r, void* stream, int nepochs) {
  SKGE_CHECK_ARG(r && (r->exec || r->dp), "bad runner");
  SKGE_CHECK_ARG(!r->dp, "data-parallel runner: drive it with skge_pipe_runner_dp_*");
  if (r->invalid) return refuse_invalid(r);
  hipStream_t st = as_stream(stream);
  hot_io(r, st, false);
  hipError_t e = hipSuccess;
  for (int i = 0; i < nepochs && e == hipSuccess; ++i) e = hipGraphLaunch(r->exec, st);
  // the epilogue runs even after a failed launch: hub rows and the fused
  // kernel's second-buffer rows go back to the caller's tables either way
  hot_io(r, st, true);
  fused_finalize(r, st);
  if (e != hipSuccess) {
    r->invalid = true;
    set_error("pipelined runner: hipGraphLaunch failed: %s (runner now invalid)",
              hipGetErrorString(e));
    return SKGE_EHIP;
  }
  SKGE_CHECK_LAUNCH("pipelined runner finalize");
  return SKGE_OK;
}

extern "C" int skge_pipe_runner_profile(skge_pipe_runner_t* r, void* stream, float* us_out,
                                        int* stats_out, int n, int trace_launch,
                                        uint64_t* trace_out, int64_t trace_len) {
  SKGE_CHECK_ARG(r && us_out && stats_out, "NULL argument");
  SKGE_CHECK_ARG(!r->dp, "profile(): not for the data-parallel form");
  if (r->invalid) return refuse_invalid(r);
  const int nl = r->nlaunch();
  SKGE_CHECK_ARG(n >= nl, "output arrays need nlaunches entries");
  hipStream_t st = as_stream(stream);
  std::vector<hipEvent_t> ev(nl + 1, nullptr);
  int rc = SKGE_OK;
  for (auto& e : ev)
    if (hipEventCreate(&e) != hipSuccess) rc = SKGE_EHIP;
  const size_t sh = (size_t)NSHARD * SHARD_STRIDE;
  if (rc == SKGE_OK && hipMemsetAsync(r->stats, 0, (size_t)nl * 3 * sh * 4, st) != hipSuccess)
    rc = SKGE_EHIP;
  unsigned long long* dtrace = nullptr;
  if (rc == SKGE_OK && trace_out && trace_launch >= 1 && trace_launch <= (int)r->batch.size()) {
    const PipeArgs& tb = r->batch[trace_launch - 1];
    const int64_t need = 2 + 6 * (int64_t)tb.count + 2 * 4 * (int64_t)tb.nA;
    if (trace_len < need) {
      set_error("trace buffer needs %lld entries", (long long)need);
      rc = SKGE_EINVAL;
    } else if (hipMalloc(&dtrace, need * 8) != hipSuccess ||
               hipMemsetAsync(dtrace, 0, need * 8, st) != hipSuccess) {
      rc = SKGE_EHIP;
    } else {
      const unsigned long long hdr[2] = {(unsigned long long)tb.count, 4ull * tb.nA};
      if (hipMemcpyAsync(dtrace, hdr, 16, hipMemcpyHostToDevice, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess)   // ordered after the memset, on st
        rc = SKGE_EHIP;
    }
  }
  if (rc == SKGE_OK) {
    hot_io(r, st, false);
    enqueue_epoch(r, st, ev.data(), r->stats, trace_launch, dtrace);
    hot_io(r, st, true);
    fused_finalize(r, st);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) rc = SKGE_EHIP;
  }
  if (rc == SKGE_OK) {
    for (int i = 0; i < nl; ++i) {
      float ms = 0.0f;
      if (hipEventElapsedTime(&ms, ev[i], ev[i + 1]) != hipSuccess) rc = SKGE_EHIP;
      us_out[i] = 1e3f * ms;
    }
    std::vector<int> h((size_t)nl * 3 * sh);
    if (hipMemcpy(h.data(), r->stats, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
      rc = SKGE_EHIP;
    for (int k = 0; k < 3 * nl; ++k) {
      int v = 0;
      for (int q = 0; q < NSHARD; ++q) v += h[(size_t)k * sh + (size_t)q * SHARD_STRIDE];
      stats_out[k] = v;
    }
    if (dtrace) {
      const PipeArgs& tb = r->batch[trace_launch - 1];
      const int64_t need = 2 + 6 * (int64_t)tb.count + 2 * 4 * (int64_t)tb.nA;
      if (hipMemcpy(trace_out, dtrace, need * 8, hipMemcpyDeviceToHost) != hipSuccess)
        rc = SKGE_EHIP;
    }
  }
  if (dtrace) (void)hipFree(dtrace);
  for (auto& e : ev)
    if (e) (void)hipEventDestroy(e);
  if (rc != SKGE_OK) set_error("pipelined runner profile failed");
  return rc;
}

// ---- data-parallel form (SKGE_PIPE_DP): the caller's per-epoch sequence is
// dp_begin, then for every batch b: dp_batch(b, own slice) -> all-gather of
// the slice records -> dp_scatter(b, gathered records), then dp_batch(nb1)
// (the flush) and dp_end.  Every call is stream-ordered and capturable. ----
static void rel_fold_launch(const skge_pipe_runner* r, hipStream_t st, const PipeArgs& a) {
  if (!r->rfold || a.count <= 0) return;
  const size_t words = (size_t)a.R.rows * a.R.rw;
  hipLaunchKernelGGL(k_rel_fold, dim3((unsigned)std::min<size_t>((words + 255) / 256, 4096)),
                     dim3(256), 0, st, a);
}

extern "C" size_t skge_pipe_dp_record_bytes(int d) {
  return d > 0 && d % 4 == 0 ? 4 * (size_t)pipe_dp_record_words(d) : 0;
}

extern "C" int skge_pipe_runner_nbatches(const skge_pipe_runner_t* r) {
  return r ? (int)r->batch.size() - 1 : -1;
}

extern "C" int skge_pipe_runner_dp_begin(skge_pipe_runner_t* r, void* stream) {
  SKGE_CHECK_ARG(r && r->dp, "not a data-parallel pipelined runner");
  if (r->invalid) return refuse_invalid(r);
  long long blocks = (r->T + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_epoch_sample, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                     r->trip, r->T, r->half, r->seed, (const uint64_t*)r->epoch_key, r->set,
                     r->n_ent, r->ntries, r->rec, r->rec_n1, (const int*)r->err);
  SKGE_CHECK_LAUNCH("dp epoch sample");
  return SKGE_OK;
}

extern "C" int skge_pipe_runner_dp_batch(skge_pipe_runner_t* r, void* stream, int b, int lo,
                                         int hi, void* rec_out, int fold) {
  SKGE_CHECK_ARG(r && r->dp, "not a data-parallel pipelined runner");
  if (r->invalid) return refuse_invalid(r);
  const int nb1 = (int)r->batch.size() - 1;
  SKGE_CHECK_ARG(b >= 0 && b <= nb1, "batch %d out of [0, %d]", b, nb1);
  PipeArgs a = r->batch[b];
  SKGE_CHECK_ARG(0 <= lo && lo <= hi && hi <= a.count, "slice [%d, %d) out of the batch", lo, hi);
  SKGE_CHECK_ARG(rec_out || lo == hi, "NULL record buffer");
  a.lo = lo;
  a.hi = hi;
  a.dprec = (uint32_t*)rec_out;
  const int wpb = (a.E.own[0] ? PIPE_WG_GRP : SKGE_PIPE_WG) / 64;
  const int nBb = hi > lo ? std::min((hi - lo + wpb - 1) / wpb, 16384) : 0;
  hipStream_t st = as_stream(stream);
  launch_pipe_batch(r, dim3((unsigned)(a.nA + nBb)), st, a);
  if (fold) rel_fold_launch(r, st, a);
  SKGE_CHECK_LAUNCH("dp batch");
  return SKGE_OK;
}

extern "C" int skge_pipe_runner_dp_scatter(skge_pipe_runner_t* r, void* stream, int b,
                                           const void* recs, int lo, int hi) {
  SKGE_CHECK_ARG(r && r->dp, "not a data-parallel pipelined runner");
  if (r->invalid) return refuse_invalid(r);
  const int nb1 = (int)r->batch.size() - 1;
  SKGE_CHECK_ARG(b >= 0 && b < nb1, "batch %d out of [0, %d)", b, nb1);
  PipeArgs a = r->batch[b];
  SKGE_CHECK_ARG(0 <= lo && lo <= hi && hi <= a.count, "slice [%d, %d) out of the batch", lo, hi);
  const int nrem = a.count - (hi - lo);
  SKGE_CHECK_ARG(recs || nrem == 0, "NULL records");
  a.lo = lo;
  a.hi = hi;
  hipStream_t st = as_stream(stream);
  if (nrem > 0) {
    const dim3 gr((unsigned)std::max(1, std::min((nrem + 3) / 4, 16384))), bl(256);
    const uint32_t* rc = (const uint32_t*)recs;
#define SKGE_DS(K)                                                                              \
  do {                                                                                          \
    if (r->e8) {                                                                                \
      if (r->w32) hipLaunchKernelGGL((k_pipe_dp_scatter<K, true, true>), gr, bl, 0, st, a, rc);  \
      else hipLaunchKernelGGL((k_pipe_dp_scatter<K, false, true>), gr, bl, 0, st, a, rc);        \
    } else {                                                                                    \
      if (r->w32) hipLaunchKernelGGL((k_pipe_dp_scatter<K, true, false>), gr, bl, 0, st, a, rc); \
      else hipLaunchKernelGGL((k_pipe_dp_scatter<K, false, false>), gr, bl, 0, st, a, rc);       \
    }                                                                                           \
  } while (0)
    if (r->kq <= 1) SKGE_DS(1);
    else if (r->kq <= 2) SKGE_DS(2);
    else SKGE_DS(4);
#undef SKGE_DS
  }
  rel_fold_launch(r, st, a);
  SKGE_CHECK_LAUNCH("dp scatter");
  return SKGE_OK;
}

extern "C" int skge_pipe_runner_dp_end(skge_pipe_runner_t* r, void* stream) {
  SKGE_CHECK_ARG(r && r->dp, "not a data-parallel pipelined runner");
  hipLaunchKernelGGL(k_pipe_advance, dim3(1), dim3(1), 0, as_stream(stream), r->epoch_key);
  SKGE_CHECK_LAUNCH("dp end");
  return SKGE_OK;
}

extern "C" int skge_pipe_runner_error(skge_pipe_runner_t* r, void* stream) {
  SKGE_CHECK_ARG(r, "bad runner");
  int v = 0;
  SKGE_CHECK_HIP(hipStreamSynchronize(as_stream(stream)));
  SKGE_CHECK_HIP(hipMemcpy(&v, r->err, 4, hipMemcpyDeviceToHost));
  if (v) r->invalid = true;   // sticky: later run()s are refused
  return v;
}

extern "C" int skge_pipe_runner_nlaunches(const skge_pipe_runner_t* r) {
  return r ? r->nlaunch() : -1;
}

extern "C" int skge_pipe_runner_kernel(const skge_pipe_runner_t* r) {
  return r ? (r->hole ? 2 : (r->fused ? 1 : 0)) : -1;
}

extern "C" int skge_pipe_runner_hot_rows(const skge_pipe_runner_t* r) {
  return r ? (r->batch.empty() ? 0 : r->batch[0].E.nhot) : -1;
}

extern "C" void skge_pipe_runner_destroy(skge_pipe_runner_t* r) { pipe_free(r); }
