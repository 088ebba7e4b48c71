// Pipelined HolE pairwise runner kernels (skge/hole.py:44-100): the launch
// structure of skge_pipeline.hip's k_pipe_batch with fp32 sums; driven by
// the same runner host code (skge_hole_pipe_runner_create).
#include "skge_hole.h"
#include "skge_hole_fft.h"
#include "skge_pipe.h"

namespace skge {

// ======================== HolE pairwise, pipelined ========================
//
// The launch structure of k_pipe_batch for HolE (skge/hole.py:44-100, the
// pairwise gradients, E post normless1): launch g scores batch b -- one wave
// per positive, both of its pairs, k_hole_pos's seven correlations and exact
// arithmetic -- while other workgroups apply batch b-1's rows (claim,
// write-through publish, done word; a scoring wave reading a row batch b-1
// touched applies it itself or waits).  Sums are fp32 (HolE contributions are
// not small integers): entity sums [rows][d] double-buffered by batch parity,
// relation sums [rows][rw words] (floats 0..d-1, count as an int at float d)
// triple-buffered by launch id, one copy (every scoring wave recomputes
// R_b[p] from R_{b-1}[p] and batch b-1's sums, as k_pipe_batch does).  Float
// atomics add in any order, so the result equals the two-launch HolE loop to
// fp32 rounding, not bit for bit.  Scoring workgroups are dispatched first
// (their correlations are the launch's long pole): the apply waves then run
// beside them.

// One row's update from fp32 sums (zero past the row); row_update's arithmetic
template <int KQ>
__device__ __forceinline__ void row_update_f(const UpdParams& t, int c, int d,
                                             const float4 (&sm)[KQ], float4 (&p)[KQ],
                                             float4 (&a)[KQ]) {
  const int l = lane_id(), nq = d >> 2;
  const bool ada = t.opt == OPT_ADAGRAD;
  const float div = t.fdiv > 0.0f ? t.fdiv : (float)c;
  float ss = 0.0f;
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const bool in = 64 * m + l < nq;
#define SKGE_UP(X)                                                      \
  {                                                                     \
    const float g = (sm[m].X + t.rin * p[m].X) / div + t.rout * p[m].X; \
    float pv = p[m].X;                                                  \
    if (ada) {                                                          \
      a[m].X = a[m].X + g * g;                        /* param.py:147 */\
      pv = pv - (t.lr * g) / fmaxf(sqrtf(a[m].X), 1e-7f); /* 152-155 */ \
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
    const float nrm = t.post == POST_NORMALIZE ? sqrtf(ss) : (ss < 1.0f ? 1.0f : ss);
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      p[m].x = p[m].x / nrm;
      p[m].y = p[m].y / nrm;
      p[m].z = p[m].z / nrm;
      p[m].w = p[m].w / nrm;
    }
  }
}

// P, A (P again when A is null: discarded) and fp32 sums of one quad-layout
// row, unconditional 16-B loads; sums zero past the row
template <int KQ>
__device__ __forceinline__ void load_f32_row(const float* P, const float* A, const float* S,
                                             int row, int d, float4 (&p)[KQ], float4 (&a)[KQ],
                                             float4 (&sm)[KQ]) {
  const int l = lane_id(), nq = d >> 2;
  const float4* prow = reinterpret_cast<const float4*>(P + (size_t)row * d);
  const float4* arow = reinterpret_cast<const float4*>((A ? A : P) + (size_t)row * d);
  const float4* srow = reinterpret_cast<const float4*>(S + (size_t)row * d);
  const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l, qc = q < nq ? q : nq - 1;
    const float4 sv = srow[qc];
    p[m] = prow[qc];
    a[m] = arow[qc];
    sm[m] = q < nq ? sv : z;
  }
}

template <int KQ>
__device__ __forceinline__ void claim_and_apply_f(const PipeTab& t, int pp, int row, int d,
                                                  int gp) {
  const int l = lane_id(), nq = d >> 2;
  int c = 0;
  if (l == 0) c = atomicExch(t.cnt[pp] + row, 0);
  float* S = reinterpret_cast<float*>(t.sum[pp]);
  float4 sm[KQ], p[KQ], a[KQ];
  load_f32_row<KQ>(t.P, t.A, S, row, d, p, a, sm);
  c = __builtin_amdgcn_readfirstlane(c);
  if (c == 0) return;   // another wave owns the row
  row_update_f<KQ>(t.u, c, d, sm, p, a);
  float4* srow = reinterpret_cast<float4*>(S + (size_t)row * d);
#pragma unroll
  for (int m = 0; m < KQ; ++m)
    if (64 * m + l < nq) srow[64 * m + l] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  store_row4_sc1<KQ>(t.P, row, d, p);
  if (t.A) store_row4_sc1<KQ>(t.A, row, d, a);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every store of this wave has landed
  if (l == 0) __hip_atomic_store(t.done + row, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t.claims && l == 0) atomicAdd(shard_of(t.claims), 1);
}

// The HolE launch's A role over its share of the slot records: slots k0,
// k0 + ks, ... < ns.  The slot ids come in one vector load per 64 slots (empty
// slots cost nothing more), and each touched row's claim and loads are issued
// while the previous row is updated and published, so a wave's rows overlap
// instead of paying a dependent slot load + claim round trip each.
template <int KQ>
__device__ __forceinline__ void apply_slots_f(const PipeTab& t, int pp, int k0, int ks, int ns,
                                              int d, int gp) {
  const int l = lane_id(), nq = d >> 2;
  float* S = reinterpret_cast<float*>(t.sum[pp]);
  for (int base = k0; base < ns; base += 64 * ks) {
    const int k = base + l * ks;
    const int rowl = k < ns ? t.touched[pp][k] : -1;
    uint64_t m = __ballot(rowl >= 0);
    if (!m) continue;
    int i = __builtin_ctzll(m);
    m &= m - 1;
    int r = __builtin_amdgcn_readlane(rowl, i), c = 0;
    float4 sm[KQ], p[KQ], a[KQ];
    if (l == 0) c = atomicExch(t.cnt[pp] + r, 0);
    load_f32_row<KQ>(t.P, t.A, S, r, d, p, a, sm);
    int nclaim = 0;
    while (true) {
      int rn = -1, cn = 0;
      float4 smn[KQ], pn[KQ], an[KQ];
      if (m) {   // the next row's claim and loads in flight behind this row
        i = __builtin_ctzll(m);
        m &= m - 1;
        rn = __builtin_amdgcn_readlane(rowl, i);
        if (l == 0) cn = atomicExch(t.cnt[pp] + rn, 0);
        load_f32_row<KQ>(t.P, t.A, S, rn, d, pn, an, smn);
      }
      c = __builtin_amdgcn_readfirstlane(c);
      if (c != 0) {   // this wave owns the row
        row_update_f<KQ>(t.u, c, d, sm, p, a);
        float4* srow = reinterpret_cast<float4*>(S + (size_t)r * d);
#pragma unroll
        for (int q = 0; q < KQ; ++q)
          if (64 * q + l < nq) srow[64 * q + l] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        store_row4_sc1<KQ>(t.P, r, d, p);
        if (t.A) store_row4_sc1<KQ>(t.A, r, d, a);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every store of this wave has landed
        if (l == 0) __hip_atomic_store(t.done + r, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ++nclaim;
      }
      if (rn < 0) break;
      r = rn;
      c = cn;
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        sm[q] = smn[q];
        p[q] = pn[q];
        a[q] = an[q];
      }
    }
    if (t.claims && l == 0 && nclaim) atomicAdd(shard_of(t.claims), nclaim);
  }
}

template <int KQ>
__device__ __forceinline__ void ensure_applied_f(const PipeTab& t, int pp, int row, int d, int gp,
                                                 int* err) {
  if (__hip_atomic_load(t.done + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gp) return;
  claim_and_apply_f<KQ>(t, pp, row, d, gp);
  unsigned spins = 0;
  while (__hip_atomic_load(t.done + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gp) {
    __builtin_amdgcn_s_sleep(2);
    if (++spins > (1u << 22)) {   // ~0.5 s: never hang the GPU; report instead
      if (lane_id() == 0) atomicOr(err, ERR_WAIT);
      break;
    }
    if ((spins & 1023u) == 0 &&
        __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      break;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the re-read below the poll
}

// Hot entity rows (PipeTab::hot; the pair form on skewed KGs), fp32 sums: the
// scheme of TransE's hot_value / apply_hot (skge_pipe.h).  A hub's sums and
// count go to replica w % HOT_REPS of three rotating copies (launch g adds
// into copy g % 3); its value after launch g lives in hP[g & 1].  A scoring
// wave of launch g that reads a hub computes the value batch b scores with --
// the previous value hP[(g-1) & 1] updated with copy (g-1) % 3, inputs nobody
// writes during launch g -- itself, with the replicas added in index order
// and the applier's arithmetic (row_update_f): every reader and the A-role
// item get the same bits, and nobody waits on a hub.  Float atomics make the
// replica sums themselves order-dependent (as every HolE sum is), so the
// runner equals the two-launch loop to fp32 rounding.  Replica rows hold
// 2 * hw floats.
template <int KQ>
__device__ __forceinline__ int hot_value_f(const PipeTab& t, int h, int g, int d, float4 (&p)[KQ],
                                           float4 (&a)[KQ]) {
  const int l = lane_id(), nq = d >> 2, hwf = 2 * t.hw;
  const int src = (g - 1) & 1, cp = (g - 1) % 3;
  const float4* prow = reinterpret_cast<const float4*>(t.hP[src] + (size_t)h * d);
  const float4* arow = reinterpret_cast<const float4*>((t.hA[src] ? t.hA[src] : t.hP[src]) +
                                                       (size_t)h * d);
  const float* hrow = reinterpret_cast<const float*>(t.hsum[cp]) + (size_t)h * HOT_REPS * hwf;
  const int cl = l < HOT_REPS ? t.hcnt[cp][h * HOT_REPS + l] : 0;
  const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  float4 x[HOT_REPS][KQ], sm[KQ];
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l, qc = q < nq ? q : nq - 1;
    p[m] = prow[qc];
    a[m] = t.hA[src] ? arow[qc] : z;
#pragma unroll
    for (int k = 0; k < HOT_REPS; ++k) {
      const float4 v = reinterpret_cast<const float4*>(hrow + (size_t)k * hwf)[qc];
      x[k][m] = q < nq ? v : z;
    }
  }
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    sm[m] = x[0][m];
#pragma unroll
    for (int k = 1; k < HOT_REPS; ++k) {
      sm[m].x += x[k][m].x;
      sm[m].y += x[k][m].y;
      sm[m].z += x[k][m].z;
      sm[m].w += x[k][m].w;
    }
  }
  const int c = wave_sum_int(cl);
  if (c) {
    row_update_f<KQ>(t.u, c, d, sm, p, a);
  } else {
#pragma unroll
    for (int m = 0; m < KQ; ++m)
      if (64 * m + l >= nq) p[m] = z;
  }
  return c;
}

// launch g's item for hot row h: its value after the launch into hP[g & 1]
// (plain stores: read by later launches only), the replica copy launch g + 1
// adds into ((g - 2) % 3) zeroed
template <int KQ>
__device__ __forceinline__ void apply_hot_f(const PipeTab& t, int h, int g, int d) {
  const int l = lane_id(), nq = d >> 2, hwf = 2 * t.hw;
  float4 p[KQ], a[KQ];
  const int c = hot_value_f<KQ>(t, h, g, d, p, a);
  store_row4<KQ>(t.hP[g & 1], h, d, p);
  if (t.hA[0]) store_row4<KQ>(t.hA[g & 1], h, d, a);
  const int old = (g - 2) % 3;
  float* hrow = reinterpret_cast<float*>(t.hsum[old]) + (size_t)h * HOT_REPS * hwf;
#pragma unroll
  for (int k = 0; k < HOT_REPS; ++k)
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      const int q = 64 * m + l;
      if (q < nq)
        reinterpret_cast<float4*>(hrow + (size_t)k * hwf)[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
  if (l < HOT_REPS) t.hcnt[old][h * HOT_REPS + l] = 0;
  if (c && t.claims && l == 0) atomicAdd(shard_of(t.claims), 1);
}

// relation row R_b[row] from R_{b-1} (buffer rd) and batch b-1's fp32 sums
// (copy ra: floats [0, d), count at float d); zero past the row
template <int KQ>
__device__ __forceinline__ void rel_row_f(const RelTab& t, int row, int d, int rd, int ra,
                                          float4 (&p)[KQ], float4 (&a)[KQ], int& c) {
  const int l = lane_id(), nq = d >> 2;
  const float* acc = reinterpret_cast<const float*>(t.acc[ra] + (size_t)row * t.rw);
  float4 sm[KQ];
  load_f32_row<KQ>(t.P[rd] + (size_t)row * d, t.A[rd] ? t.A[rd] + (size_t)row * d : nullptr,
                   acc, 0, d, p, a, sm);
  c = __builtin_amdgcn_readfirstlane(__float_as_int(acc[d]));
  const int nrep = t.folded ? 1 : t.reps;   // folded: replica 0 holds the sum
  for (int k = 1; k < nrep; ++k) {   // large batches: the replicas, in a fixed order
    const float* ak = reinterpret_cast<const float*>(t.acc[ra] +
                                                     ((size_t)k * t.rows + row) * t.rw);
    const float4* ak4 = reinterpret_cast<const float4*>(ak);
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      const int q = 64 * m + l;
      const float4 v = ak4[q < nq ? q : nq - 1];
      if (q < nq) {
        sm[m].x += v.x;
        sm[m].y += v.y;
        sm[m].z += v.z;
        sm[m].w += v.w;
      }
    }
    c += __builtin_amdgcn_readfirstlane(__float_as_int(ak[d]));
  }
  if (c) {
    row_update_f<KQ>(t.u, c, d, sm, p, a);
  } else {
#pragma unroll
    for (int m = 0; m < KQ; ++m)
      if (64 * m + l >= nq) p[m] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
}

template <int KQ>
__device__ __forceinline__ void rel_publish_f(const PipeArgs& a, int w, int rd, int rw,
                                              int ra_prev, int ra_old) {
  const int l = lane_id(), d = a.d, nq = d >> 2;
  float4 p[KQ], av[KQ];
  int c;
  rel_row_f<KQ>(a.R, w, d, rd, ra_prev, p, av, c);
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
  for (int k = 0; k < a.R.reps; ++k) {   // rw 8-B words: the sums and the count
    const size_t ko = (size_t)k * a.R.rows * a.R.rw;
    for (int q = l; q < a.R.rw; q += 64) {
      old[ko + q] = 0ull;
      if (flush) prev[ko + q] = 0ull;
    }
  }
  if (c && a.R.updated && l == 0) atomicAdd(shard_of(a.R.updated), 1);
}


// PAIR (round 4, SKGE_HPIPE_PAIR; FFT at d = 200): 128-thread
// workgroups, and a scoring workgroup's two waves score ONE positive together
// -- each loads and settles two of its rows, the transforms' stage passes are
// split between them (fft_run_c2: the same butterflies, the same bits), both
// compute the spectra and scores (identical values), and each issues half of
// the contribution rows' atomics -- so a positive's serial chain is shorter.
template <int KM, bool HOT>
__device__ __forceinline__ void hole_pipe_score_pair(const PipeArgs& a, float* smem, int blk_b,
                                                     int nB) {
  const int hw = (int)(threadIdx.x >> 6);   // the wave's half of the pair
  const int l = lane_id();
  const int d = a.d;
  const int g = launch_id(a), gp = g - 1;
  const int cp = a.b & 1, pp = cp ^ 1;
  const int rd = a.b & 1;
  const int ra_prev = (g - 1) % 3, ra_cur = g % 3;
  float2* const tw = reinterpret_cast<float2*>(smem);
  // the twiddle table into LDS before the loop (its load overlapped with the
  // first record's round trip measured no faster: not on the critical path)
  fft_twiddles(tw, a.tw, d);
  float* const wb = smem + 2 * d;   // the pair's two transform buffers
  float2* const b0 = reinterpret_cast<float2*>(wb);
  float2* const b1 = b0 + 5 * 100;
  Accum aE = {};
  aE.sum = reinterpret_cast<float*>(a.E.sum[cp]);
  aE.width = d;
  const int rstride = 2 * a.R.rw;
  int nv = 0;
  for (int w = blk_b; w < a.count; w += nB) {
    float* const racc = reinterpret_cast<float*>(a.R.acc[ra_cur]) +
                        (size_t)(w % a.R.reps) * a.R.rows * rstride;
    unsigned long long tt[4] = {0ull, 0ull, 0ull, 0ull};   // diagnostics: wave 0's phases
    if (a.trace) tt[0] = now_10ns();
    const long long j = a.start + w;
    const int4 r4 = a.rec[j];
    const int r1 = a.rec_n1[j];
    __builtin_amdgcn_sched_barrier(0);
    const int s = uni(r4.x), o = uni(r4.y), p = uni(r4.z), neg0 = uni(r4.w);
    const int neg1 = uni(r1);
    const int n0r = neg0 >= 0 ? neg0 : s, n1r = neg1 >= 0 ? neg1 : o;
    // wave 0: E[s], E[s'] (signals 1, 2); wave 1: E[o], E[o'] (3, 4); R[p] (0)
    // on wave pair_r1
    const int ra_row = hw ? o : s, rb_row = hw ? n1r : n0r;
    float4 xa[1], xb[1], xr[1] = {};
    load_row4<1>(a.E.P, ra_row, d, xa);
    load_row4<1>(a.E.P, rb_row, d, xb);
    int mark = 0, hxl = -1;
    if (l < 2) mark = a.E.pend[pp][l ? rb_row : ra_row];
    if (HOT && l < 4) hxl = a.E.hot[sel4(l, s, o, n0r, n1r)];   // hub rows: no marks, no waits
    if (hw == a.pair_r1) {
      float4 rav[1];
      int c;
      rel_row_f<1>(a.R, p, d, rd, ra_prev, xr, rav, c);
    }
    const uint64_t pend = __ballot(mark == gp) & 0x3ull;
    if (a.trace) tt[1] = now_10ns();
    if (pend) {
      if (pend & 1ull) ensure_applied_f<1>(a.E, pp, ra_row, d, gp, a.err);
      if (pend & 2ull) ensure_applied_f<1>(a.E, pp, rb_row, d, gp, a.err);
      if (pend & 1ull) load_row4_sc1<1>(a.E.P, ra_row, d, xa);
      if (pend & 2ull) load_row4_sc1<1>(a.E.P, rb_row, d, xb);
    }
    if (HOT) {   // this wave's hub rows: the value after batch b-1, computed here
      const int ha = __builtin_amdgcn_readlane(hxl, hw ? 1 : 0);
      const int hb = __builtin_amdgcn_readlane(hxl, hw ? 3 : 2);
      float4 hv[1], hav[1];
      if (ha >= 0) {
        hot_value_f<1>(a.E, ha, g, d, hv, hav);
        xa[0] = hv[0];
      }
      if (hb >= 0) {
        hot_value_f<1>(a.E, hb, g, d, hv, hav);
        xb[0] = hv[0];
      }
    }
    if (a.trace) tt[2] = now_10ns();
    __syncthreads();   // the previous positive's buffers are free, the twiddles in place
    if (hw == a.pair_r1) fft_put_row(b0, 100, 0, xr[0], d);
    if (hw == 0) {
      fft_put_row(b0, 100, 1, xa[0], d);
      fft_put_row(b0, 100, 2, xb[0], d);
    } else {
      fft_put_row(b0, 100, 3, xa[0], d);
      fft_put_row(b0, 100, 4, xb[0], d);
    }
    __syncthreads();
    const float2* Z = fft_run_c2<100, 5, false>(b0, b1, tw, hw);
    float praw, raw0, raw1;
    const HoleSpec hs = hole_fft_spectra(Z, tw, d, praw, raw0, raw1);
    const float pf = af_f(a.af, praw), f0 = af_f(a.af, raw0), f1 = af_f(a.af, raw1);
    const int v0 = uni((neg0 >= 0 && f0 + a.margin > pf) ? 1 : 0);   // hole.py:56
    const int v1 = uni((neg1 >= 0 && f1 + a.margin > pf) ? 1 : 0);
    if (a.trace) tt[3] = now_10ns();
    // trace record of positive w (wave 0, lane 0): stamps, then the flags word
    // (bits 0-1: wave 0's pending rows s, s'; 8 violating; 9 v0; 10 v1; 16+:
    // the inverse phase in 10 ns ticks)
    auto stamp = [&](unsigned long long flags) {
      if (a.trace && hw == 0 && l == 0) {
        unsigned long long* tr = a.trace + 2 + 6 * (size_t)w;
        tr[0] = tt[0]; tr[1] = tt[1]; tr[2] = tt[2]; tr[3] = tt[3]; tr[4] = now_10ns();
        tr[5] = flags;
      }
    };
    if (hw == 0) {
      const int cE = sel4(l, v0 + 2 * v1, 2 * v0 + v1, v0, v1);
      const int rE = sel4(l, s, o, neg0, neg1);
      if (HOT && l < 4 && hxl >= 0) {   // hub: count into its replica, no slot record
        if (cE > 0) atomicAdd(a.E.hcnt[g % 3] + hxl * HOT_REPS + (w & (HOT_REPS - 1)), cE);
        a.E.touched[cp][4 * w + l] = -1;
      } else if (l < 4) {
        commit_slot(a.E.cnt[cp], a.E.touched[cp], rE, cE, 4 * w + l);
        if (cE > 0) a.E.pend[cp][rE] = g;
      } else if (l == 4 && v0 + v1 > 0) {
        atomicAdd(reinterpret_cast<int*>(racc + (size_t)p * rstride + d), 2 * (v0 + v1));
      }
      nv += v0 + v1;
    }
    if (v0 + v1 == 0) {   // (the same in both waves)
      stamp(pend);
      continue;
    }
    const float gpf = -af_g_given_f(a.af, pf);   // hole.py:66
    const float g0 = af_g_given_f(a.af, f0), g1 = af_g_given_f(a.af, f1);   // hole.py:67
    const float* z = hole_fft_rows_pair(wb, tw, hs, v0, v1, gpf, g0, g1, hw);
    const unsigned long long inv_dt = a.trace ? now_10ns() - tt[3] : 0ull;
    // an entity row's target: its sums, or a hub's replica w % HOT_REPS
    auto ent_row = [&](int k, int row, int t) {
      const int h = HOT ? __builtin_amdgcn_readlane(hxl, k) : -1;
      if (h >= 0) {
        Accum aH = {};
        aH.sum = reinterpret_cast<float*>(a.E.hsum[g % 3]) +
                 ((size_t)h * HOT_REPS + (w & (HOT_REPS - 1))) * (2 * a.E.hw);
        aH.width = d;
        acc_fft_row<KM>(aH, 0, z, t, d);
      } else {
        acc_fft_row<KM>(aE, row, z, t, d);
      }
    };
    if (hw == 0) {
      Accum aR = {};
      aR.sum = racc + (size_t)p * rstride;
      aR.width = d;
      acc_fft_row<KM>(aR, 0, z, 2, d);
      ent_row(0, s, 0);
    } else {
      ent_row(1, o, 1);
      if (v0) ent_row(2, neg0, 3);
      if (v1) ent_row(3, neg1, 3 + v0);
    }
    __builtin_amdgcn_wave_barrier();
    stamp(pend | (1ull << 8) | ((unsigned long long)v0 << 9) | ((unsigned long long)v1 << 10) |
          (inv_dt << 16));
  }
  if (l == 0 && nv) {
    atomicAdd(shard_of(a.nviol_shards), nv);
    if (a.stats_viol) atomicAdd(shard_of(a.stats_viol), nv);
  }
}

template <int KM, bool FFT, bool PAIR = false, bool HOT = false>
__global__ __launch_bounds__(SKGE_PIPE_WG) void k_hole_pipe(PipeArgs a) {
  static_assert(!PAIR || FFT, "the pair form is the FFT form's");
  static_assert(!HOT || PAIR, "hot rows: the pair form only");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wpb = blockDim.x >> 6, wave = threadIdx.x >> 6;
  const int l = lane_id();
  const int d = a.d;
  const int g = launch_id(a), gp = g - 1;
  const int cp = a.b & 1, pp = cp ^ 1;
  const int rd = a.b & 1;
  const int rw = a.b < a.nb1 ? rd ^ 1 : 0;
  const int ra_prev = (g - 1) % 3, ra_cur = g % 3, ra_old = (g - 2) % 3;
  const int nB = gridDim.x - a.nA;
  const int blk = (int)blockIdx.x;
  if (blk < a.nA) {
    // ---- A role: write R_b, then apply the previous batch's entity rows ----
    const int blk_a = blk;
    const int nR = a.R.rows;
    const int wa = blk_a * wpb + wave;
    const unsigned long long ta0 = a.trace ? now_10ns() : 0ull;
    if (a.b == a.nb1 && wa == 0) fold_shards(a.nviol_shards, a.nviol_total);
    // items w = wa, wa + S, ...: relation rows w < nR, hot rows, then entity
    // slots w - nR - nH
    const int S = a.nA * wpb;
    const int nRH = nR + a.E.nhot;
    for (int w = wa; w < nRH; w += S) {
      if (w < nR) rel_publish_f<1>(a, w, rd, rw, ra_prev, ra_old);
      else if (HOT) apply_hot_f<1>(a.E, w - nR, g, d);
    }
    const int k0 = wa >= nRH ? wa - nRH : wa - nRH + ((nRH - wa + S - 1) / S) * S;
    apply_slots_f<1>(a.E, pp, k0, S, a.prev_slots, d, gp);
    if (a.trace && l == 0) {   // diagnostics (skge_pipe_runner_profile, tools/hole_trace.py)
      unsigned long long* tr = a.trace + 2 + 6 * (size_t)a.count + 2 * (size_t)wa;
      tr[0] = ta0;
      tr[1] = now_10ns();
    }
    return;
  }
  // ---- B role: score batch b (k_hole_pos's arithmetic), scatter into cp / ra_cur ----
  const int blk_b = blk - a.nA;
  if constexpr (PAIR) {
    hole_pipe_score_pair<KM, HOT>(a, smem, blk_b, nB);
    return;
  }
  // FFT: the workgroup's twiddle table, then per wave two transform buffers
  float2* const tw = reinterpret_cast<float2*>(smem);
  if constexpr (FFT) {
    fft_twiddles(tw, a.tw, d);
    __syncthreads();
  }
  float* const wb = FFT ? smem + 2 * d + wave * hole_fft_wave_floats(d) : nullptr;
  const HolePosLds L(FFT ? smem : smem + wave * hole_pos_lds_floats(d), d);
  Accum aE = {};   // mode ACC_F32 (0), one copy
  aE.sum = reinterpret_cast<float*>(a.E.sum[cp]);
  aE.width = d;
  const int rstride = 2 * a.R.rw;   // floats per relation accumulator row
  int nv = 0;
  for (int w = blk_b * wpb + wave; w < a.count; w += nB * wpb) {
    float* const racc = reinterpret_cast<float*>(a.R.acc[ra_cur]) +
                        (size_t)(w % a.R.reps) * a.R.rows * rstride;
    unsigned long long tt[4] = {0ull, 0ull, 0ull, 0ull};
    if (a.trace) tt[0] = now_10ns();
    const long long j = a.start + w;
    const int4 r4 = a.rec[j];
    const int r1 = a.rec_n1[j];
    __builtin_amdgcn_sched_barrier(0);
    const int s = uni(r4.x), o = uni(r4.y), p = uni(r4.z), neg0 = uni(r4.w);
    const int neg1 = uni(r1);
    const int n0r = neg0 >= 0 ? neg0 : s, n1r = neg1 >= 0 ? neg1 : o;
    float4 es[1], eo[1], rp[1], fs[1], fo[1];
    load_row4<1>(a.E.P, s, d, es);
    load_row4<1>(a.E.P, o, d, eo);
    load_row4<1>(a.E.P, n0r, d, fs);
    load_row4<1>(a.E.P, n1r, d, fo);
    int mark = 0;
    if (l < 4) mark = a.E.pend[pp][sel4(l, s, o, n0r, n1r)];
    {
      float4 ra[1];
      int c;
      rel_row_f<1>(a.R, p, d, rd, ra_prev, rp, ra, c);
    }
    const uint64_t pend = __ballot(mark == gp) & 0xfull;
    if (a.trace) tt[1] = now_10ns();
    if (pend) {
#pragma unroll 1
      for (int k = 0; k < 4; ++k) {
        if (!((pend >> k) & 1ull)) continue;
        ensure_applied_f<1>(a.E, pp, sel4(k, s, o, n0r, n1r), d, gp, a.err);
      }
      if (pend & 1ull) load_row4_sc1<1>(a.E.P, s, d, es);
      if (pend & 2ull) load_row4_sc1<1>(a.E.P, o, d, eo);
      if (pend & 4ull) load_row4_sc1<1>(a.E.P, n0r, d, fs);
      if (pend & 8ull) load_row4_sc1<1>(a.E.P, n1r, d, fo);
    }
    if (a.trace) tt[2] = now_10ns();
    float praw, raw0, raw1;
    float4 A = {}, B = {};
    HoleSpec hs;
    if constexpr (FFT) {
      hs = hole_fft_forward(wb, tw, d, rp[0], es[0], fs[0], eo[0], fo[0], praw, raw0, raw1);
    } else {
      q_lds_dbl(L.R2, rp[0], d);
      q_lds_dbl(L.O2, eo[0], d);
      q_lds_dbl(L.Q2, fo[0], d);
      __builtin_amdgcn_wave_barrier();
      float4 AB[2];
      {
        const float* const b2[2] = {L.O2, L.Q2};
        corr_quad_b<2>(L.R2, b2, d, AB);
      }
      A = AB[0];
      B = AB[1];
      praw = hole_score_q(es[0], A);
      raw0 = hole_score_q(fs[0], A);
      raw1 = hole_score_q(es[0], B);
    }
    const float pf = af_f(a.af, praw), f0 = af_f(a.af, raw0), f1 = af_f(a.af, raw1);
    const int v0 = uni((neg0 >= 0 && f0 + a.margin > pf) ? 1 : 0);   // hole.py:56
    const int v1 = uni((neg1 >= 0 && f1 + a.margin > pf) ? 1 : 0);
    if (a.trace) tt[3] = now_10ns();
    {
      const int cE = sel4(l, v0 + 2 * v1, 2 * v0 + v1, v0, v1);
      const int rE = sel4(l, s, o, neg0, neg1);
      if (l < 4) {
        commit_slot(a.E.cnt[cp], a.E.touched[cp], rE, cE, 4 * w + l);
        if (cE > 0) a.E.pend[cp][rE] = g;
      } else if (l == 4 && v0 + v1 > 0) {
        atomicAdd(reinterpret_cast<int*>(racc + (size_t)p * rstride + d), 2 * (v0 + v1));
      }
    }
    if (a.trace && l == 0 && v0 + v1 == 0) {
      unsigned long long* tr = a.trace + 2 + 6 * (size_t)w;
      tr[0] = tt[0]; tr[1] = tt[1]; tr[2] = tt[2]; tr[3] = tt[3]; tr[4] = now_10ns();
      tr[5] = pend;
    }
    if (v0 + v1 == 0) continue;
    nv += v0 + v1;
    unsigned long long inv_dt = 0ull;            // diagnostics: the inverse-transform phase
    const float gpf = -af_g_given_f(a.af, pf);   // hole.py:66
    const float g0 = af_g_given_f(a.af, f0), g1 = af_g_given_f(a.af, f1);   // hole.py:67
    Accum aR = {};   // mode ACC_F32 (0), one copy
    aR.sum = racc + (size_t)p * rstride;
    aR.width = d;
    if constexpr (FFT) {
      const float* z = hole_fft_rows(wb, tw, d, hs, v0, v1, gpf, g0, g1);
      if (a.trace) {   // diagnostics: the inverse transforms done (LDS results waited for)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        inv_dt = now_10ns() - tt[3];   // (reported in the flags word's high bits)
      }
      acc_fft_row<KM>(aR, 0, z, 2, d);
      acc_fft_row<KM>(aE, s, z, 0, d);
      acc_fft_row<KM>(aE, o, z, 1, d);
      if (v0) acc_fft_row<KM>(aE, neg0, z, 3, d);
      if (v1) acc_fft_row<KM>(aE, neg1, z, 3 + v0, d);
    } else {
      const HoleRows h = hole_pos_rows(L, d, es[0], fs[0], A, B, v0, v1, gpf, g0, g1);
      acc_q<KM>(aR, 0, h.cr, d, L.U);
      acc_q<KM>(aE, s, h.cs, d, L.U);
      acc_q<KM>(aE, o, h.co, d, L.U);
      if (v0) acc_q<KM>(aE, neg0, h.c0, d, L.U);
      if (v1) acc_q<KM>(aE, neg1, h.cq, d, L.U);
    }
    __builtin_amdgcn_wave_barrier();
    if (a.trace && l == 0) {   // stamp after issue (no drain)
      unsigned long long* tr = a.trace + 2 + 6 * (size_t)w;
      tr[0] = tt[0]; tr[1] = tt[1]; tr[2] = tt[2]; tr[3] = tt[3]; tr[4] = now_10ns();
      tr[5] = pend | (1ull << 8) | ((unsigned long long)v0 << 9) | ((unsigned long long)v1 << 10) |
              (inv_dt << 16);
    }
  }
  if (l == 0 && nv) {
    atomicAdd(shard_of(a.nviol_shards), nv);
    if (a.stats_viol) atomicAdd(shard_of(a.stats_viol), nv);
  }
}


// HolE, large batches: the fp32 form of k_rel_fold -- float e of row p summed
// over the replicas in index order (the order rel_row_f's readers used, so the
// same bits), the count word (float index d of the row) as an int; replicas
// 1..reps-1 zeroed.  The readers then load replica 0 alone instead of every
// replica (nb = 2: 16-32 replicas of 800 B per scoring wave).
__global__ __launch_bounds__(256) void k_rel_fold_f(PipeArgs a) {
  const int g = launch_id(a);
  float* acc = reinterpret_cast<float*>(a.R.acc[g % 3]);
  const int rstride = 2 * a.R.rw, d = a.d;
  const size_t rrep = (size_t)a.R.rows * rstride;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < rrep;
       i += (size_t)gridDim.x * blockDim.x) {
    if ((int)(i % rstride) == d) {   // the count
      int* ai = reinterpret_cast<int*>(acc);
      int c = ai[i];
      for (int k = 1; k < a.R.reps; ++k) {
        c += ai[k * rrep + i];
        ai[k * rrep + i] = 0;
      }
      ai[i] = c;
    } else {
      float v = acc[i];
      for (int k = 1; k < a.R.reps; ++k) {
        v += acc[k * rrep + i];
        acc[k * rrep + i] = 0.0f;
      }
      acc[i] = v;
    }
  }
}

void launch_hole_pipe(int km, bool pair, bool fft, dim3 gr, dim3 bl, size_t lds, hipStream_t st,
                      const PipeArgs& a) {
#define SKGE_HPIPE(K)                                                          \
  if (pair && a.E.nhot > 0)                                                    \
    hipLaunchKernelGGL((k_hole_pipe<K, true, true, true>), gr, bl, lds, st, a); \
  else if (pair)                                                               \
    hipLaunchKernelGGL((k_hole_pipe<K, true, true>), gr, bl, lds, st, a);      \
  else if (fft)                                                                \
    hipLaunchKernelGGL((k_hole_pipe<K, true>), gr, bl, lds, st, a);            \
  else                                                                         \
    hipLaunchKernelGGL((k_hole_pipe<K, false>), gr, bl, lds, st, a);
  switch (km) {
    case 1: SKGE_HPIPE(1) break;
    case 2: SKGE_HPIPE(2) break;
    case 3: SKGE_HPIPE(3) break;
    default: SKGE_HPIPE(4) break;
  }
#undef SKGE_HPIPE
}

void launch_rel_fold_f(dim3 gr, hipStream_t st, const PipeArgs& a) {
  hipLaunchKernelGGL(k_rel_fold_f, gr, dim3(256), 0, st, a);
}

}  // namespace skge
