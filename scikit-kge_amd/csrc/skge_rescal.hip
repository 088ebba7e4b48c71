// RESCAL pairwise training step on the matrix cores (fp32 MFMA).
//
// The reference scores and differentiates RESCAL one pair at a time with
// GEMVs against the pair's d x d relation matrix (skge/rescal.py:78-139):
// per pair W[p] E[o] and E[s] W[p] for the positive and the negative, and per
// relation the sum of outer products E[s] (x) E[o] for dW.  Reading W[p]
// (160 KB at d=200) once per GEMV makes that path L2-bound.  Here the batch's
// triples (positives and negatives) are grouped by relation, and per relation
// the three contractions become small GEMMs on v_mfma_f32_16x16x4_f32 (exact
// fp32: a k-ordered fmaf chain, MI355X_MICROARCH.md "Matrix cores"):
//   WE^T = E_o W[p]^T      [items x d]   (WE_i = W[p] E[o_i],  rescal.py:261)
//   EW   = E_s W[p]        [items x d]   (EW_i = E[s_i] W[p],  rescal.py:262)
//   dW[p] = E_s^T diag(coef) E_o  [d x d] (rescal.py:113-125, all pairs)
// with score_i = E[s_i] . WE_i.  Kernels:
//   k_rs_count/scan/scatter  stable counting sort of the 2P triples by
//                     relation (per-64-item-chunk ballot ranks), 16-item tiles
//   k_rescal_gemm     one workgroup per (64-triple tile, 64-column block,
//                     product): LDS-tiled, double-buffered fp32 MFMA GEMM;
//                     writes WE^T / EW rows and partial scores
//   k_rescal_scatter  one wave per pair: activation, strict margin test, the
//                     entity contributions (gp WE_p, gn WE_n over s; gp EW_p,
//                     gn EW_n over o) into the entity accumulator, coef
//   k_rescal_wgrad_mfma  one workgroup per (relation, 16-row strip, 64-col
//                     group): dW[p] tiles written with plain stores
// Scores, WE, EW and dW have fixed summation orders (stable buckets, fixed
// MFMA k order, fixed cross-wave reduction order), so the relation gradient
// is bitwise reproducible; the entity sums use float atomics, as elsewhere.
#include "skge_host.h"

namespace skge {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int RT_ITEMS = 64;    // triples per GEMM tile
constexpr int GC = 64;          // output columns per GEMM tile
constexpr int KS = 16;          // k per staged step
constexpr int RS_MAX_D = 1024;  // d of the MFMA path
constexpr int RS_MAX_M = 8192;  // relations (k_rs_scan keeps 2M+1 ints in LDS)

static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct RescalWs {
  int* chunk;       // [nchunks][M] per-chunk counts, then offsets
  int* rel_off;     // [M+1]
  int* items;       // [n] triple ids grouped by relation, stable
  int* tile_rel;    // [tmax]
  int* tile_start;  // [tmax]
  int* tile_cnt;    // [tmax]
  int* ntiles;      // [1]
  int* sorted_s;    // [n] E row of s / o of items[i] (bucket order)
  int* sorted_o;
  int* bpos;        // [n] bucket position of triple k (items[bpos[k]] == k)
  float* spart;     // [n][ceil(d/64)] partial scores of the WE column blocks
  float* coef;      // [n] dW coefficient of items[i] (bucket order)
  float* WE;        // [n][d]
  float* EW;        // [n][d]
};

static int rs_tmax(int n, int M) { return n / RT_ITEMS + M + 1; }

// carve the workspace (base may be null: size only)
// n: triples in the batch (2P for pairs: positives then negatives; T for
// labelled triples)
static size_t rescal_ws_layout(int n, int M, int d, void* base, RescalWs* ws) {
  const int nchunks = (n + 63) / 64, tmax = rs_tmax(n, M);
  size_t off = 0;
  char* b = (char*)base;
  auto take = [&](size_t bytes) {
    char* p = b ? b + off : nullptr;
    off += al256(bytes);
    return p;
  };
  RescalWs w;
  w.chunk = (int*)take((size_t)nchunks * M * 4);
  w.rel_off = (int*)take((size_t)(M + 1) * 4);
  w.items = (int*)take((size_t)n * 4);
  w.tile_rel = (int*)take((size_t)tmax * 4);
  w.tile_start = (int*)take((size_t)tmax * 4);
  w.tile_cnt = (int*)take((size_t)tmax * 4);
  w.ntiles = (int*)take(4);
  w.sorted_s = (int*)take((size_t)n * 4);
  w.sorted_o = (int*)take((size_t)n * 4);
  w.bpos = (int*)take((size_t)n * 4);
  w.spart = (float*)take((size_t)n * ((d + GC - 1) / GC) * 4);
  w.coef = (float*)take((size_t)n * 4);
  w.WE = (float*)take((size_t)n * d * 4);
  w.EW = (float*)take((size_t)n * d * 4);
  if (ws) *ws = w;
  return off;
}

// triple k of the batch: list a (na triples: the positives), then list b
__device__ __forceinline__ const int* item_trip(const int* a, const int* b, int na, int k) {
  return k < na ? a + 3 * (size_t)k : b + 3 * (size_t)(k - na);
}

// ---------------------------------------------------------------------------
// stable counting sort by relation, in three small launches:
//   k_rs_count    one wave per 64-triple chunk: per-relation counts (ballot
//                 "match" loop; the table is zeroed by a memset before)
//   k_rs_scan     one workgroup: per relation, wave-parallel exclusive scan
//                 over the chunks; relation offsets; the 16-triple tile list
//   k_rs_scatter  one wave per chunk: ranks again, writes the grouped lists
// ---------------------------------------------------------------------------
__device__ __forceinline__ int wave_incl_scan(int v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o, 64);
    if (l >= o) v += t;
  }
  return v;
}

__global__ __launch_bounds__(256) void k_rs_count(const int* __restrict__ pos,
                                                  const int* __restrict__ neg, int P, int n,
                                                  int M, RescalWs ws) {
  const int nchunks = (n + 63) / 64, l = lane_id();
  const int c = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  const int k = c * 64 + l;
  const int b = k < n ? item_trip(pos, neg, P, k)[2] : -1;
  uint64_t act = __ballot(b >= 0);
  while (act) {
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int bl = __builtin_amdgcn_readlane(b, leader);
    const uint64_t m = __ballot(b == bl) & act;
    if (l == leader) ws.chunk[(size_t)c * M + bl] = __popcll(m);
    act &= ~m;
  }
}

__global__ __launch_bounds__(1024) void k_rs_scan(int n, int M, RescalWs ws) {
  extern __shared__ int lds[];   // cnt[M], tile_base[M+1]
  int* cnt = lds;
  int* tbase = lds + M;
  const int nchunks = (n + 63) / 64;
  const int tid = threadIdx.x, l = lane_id(), wave = tid >> 6, nw = blockDim.x >> 6;
  for (int p = wave; p < M; p += nw) {   // exclusive scan of relation p over the chunks
    int carry = 0;
    for (int c0 = 0; c0 < nchunks; c0 += 64) {
      const int c = c0 + l;
      const int v = c < nchunks ? ws.chunk[(size_t)c * M + p] : 0;
      const int inc = wave_incl_scan(v);
      if (c < nchunks) ws.chunk[(size_t)c * M + p] = carry + inc - v;
      carry += __shfl(inc, 63, 64);
    }
    if (l == 0) cnt[p] = carry;
  }
  __syncthreads();
  if (wave == 0) {   // relation offsets and tile bases (exclusive scans over p)
    int off = 0, toff = 0;
    for (int p0 = 0; p0 < M; p0 += 64) {
      const int p = p0 + l;
      const int v = p < M ? cnt[p] : 0, tv = (v + RT_ITEMS - 1) / RT_ITEMS;
      const int inc = wave_incl_scan(v), tinc = wave_incl_scan(tv);
      if (p < M) {
        ws.rel_off[p] = off + inc - v;
        tbase[p] = toff + tinc - tv;
      }
      off += __shfl(inc, 63, 64);
      toff += __shfl(tinc, 63, 64);
    }
    if (l == 0) {
      ws.rel_off[M] = off;
      tbase[M] = toff;
      *ws.ntiles = toff;
    }
  }
  __syncthreads();
  const int nt = tbase[M];
  for (int t = tid; t < nt; t += blockDim.x) {   // tile t: relation p with tbase[p] <= t
    int lo = 0, hi = M - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tbase[mid] <= t) lo = mid; else hi = mid - 1;
    }
    const int p = lo, s = (t - tbase[p]) * RT_ITEMS;
    int off = 0;   // rel_off[p] again: prefix of cnt (cheap: read back)
    off = ws.rel_off[p];
    ws.tile_rel[t] = p;
    ws.tile_start[t] = off + s;
    ws.tile_cnt[t] = min(RT_ITEMS, cnt[p] - s);
  }
}

__global__ __launch_bounds__(256) void k_rs_scatter(const int* __restrict__ pos,
                                                    const int* __restrict__ neg, int P, int n,
                                                    int M, RescalWs ws) {
  const int nchunks = (n + 63) / 64, l = lane_id();
  const int c = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  const int k = c * 64 + l;
  const int* tr = item_trip(pos, neg, P, k < n ? k : 0);
  const int ts = tr[0], to = tr[1], b = k < n ? tr[2] : -1;
  uint64_t act = __ballot(b >= 0);
  while (act) {
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int bl = __builtin_amdgcn_readlane(b, leader);
    const uint64_t m = __ballot(b == bl) & act;
    if (b == bl) {
      const int at = ws.rel_off[bl] + ws.chunk[(size_t)c * M + bl] +
                     __popcll(m & ((1ull << l) - 1ull));
      ws.items[at] = k;
      ws.sorted_s[at] = ts;
      ws.sorted_o[at] = to;
      ws.bpos[k] = at;
    }
    act &= ~m;
  }
}

// ---------------------------------------------------------------------------
// Relation-grouped GEMMs, one workgroup per (64-triple tile, 64-column block,
// product):  WE^T[i][r] = sum_k Eo[i][k] W[r][k]   (product 0)
//            EW[i][j]   = sum_k Es[i][k] W[k][j]   (product 1)
// K advances 16 at a time through double-buffered LDS tiles (A: 64 triples x
// 16, B: 16 x 64 columns), the next step's global loads in flight while the
// current step's MFMAs run.  Wave w owns triples 16w..16w+15 and four 16x16
// accumulators (independent chains hide the MFMA latency).  Product-0 blocks
// also write each triple's partial score E[s_i] . WE_i over their 64 columns.
// ---------------------------------------------------------------------------
constexpr int PF = 6;   // k-steps of global loads kept in flight (registers)

template <bool VEC>
__global__ __launch_bounds__(256) void k_rescal_gemm(const float* __restrict__ E,
                                                     const float* __restrict__ W, int d,
                                                     RescalWs ws) {
  const int ncb = (d + GC - 1) / GC;
  const int t = blockIdx.x / (2 * ncb);
  if (t >= *ws.ntiles) return;
  const int rem = blockIdx.x - t * 2 * ncb;
  const int prod = rem / ncb, cb = rem - (rem / ncb) * ncb;
  const int tid = threadIdx.x, l = lane_id(), wave = tid >> 6;
  const int p = ws.tile_rel[t], s0 = ws.tile_start[t], cnt = ws.tile_cnt[t];
  const int c0 = cb * GC;
  __shared__ float sA[2][RT_ITEMS][KS + 4];
  __shared__ float sB[2][KS][GC + 4];
  __shared__ int s_row[RT_ITEMS], s_gid[RT_ITEMS], s_es[RT_ITEMS];
  if (tid < RT_ITEMS) {
    const bool ok = tid < cnt;
    const int at = s0 + (ok ? tid : 0);
    s_row[tid] = prod == 0 ? ws.sorted_o[at] : ws.sorted_s[at];   // A rows: E[o] or E[s]
    s_es[tid] = ws.sorted_s[at];
    s_gid[tid] = ok ? ws.items[at] : -1;
  }
  __syncthreads();
  const float* Wp = W + (size_t)p * d * d;
  const int nk = (d + KS - 1) / KS;
  // staging map: thread -> one float4 of A and one float4 of B per k-step
  const int ai = tid >> 2, ak = (tid & 3) * 4;            // A[ai][ak..ak+3]
  const float* arow = E + (size_t)s_row[ai] * d;
  const bool a_ok = ai < cnt;
  // B for product 0: W[c0 + bi][k..k+3] (stored transposed); product 1: W[k + bk][c0 + bj..+3]
  const int bi = tid >> 2, bk = (tid & 3) * 4;            // product 0
  const int bkr = tid >> 4, bj = (tid & 15) * 4;          // product 1
  auto load_step = [&](int ks, float4& av, float4& bv) {
    const int k = ks * KS;
#ifdef SKGE_RS_ABL_NOLOADW   // timing-only ablation builds (tools/ablate.sh)
    av = make_float4(k, k, k, k);
    bv = av;
    return;
#endif
    if (VEC) {   // d % 4 == 0: every 4-float group is inside or outside together
      const int kk = k + ak;
      const float4 x = *reinterpret_cast<const float4*>(arow + (kk < d ? kk : 0));
      av = (a_ok && kk < d) ? x : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      if (prod == 0) {
        const int r = c0 + bi, kb2 = k + bk;
        const float4 y = *reinterpret_cast<const float4*>(
            Wp + (size_t)(r < d ? r : 0) * d + (kb2 < d ? kb2 : 0));
        bv = (r < d && kb2 < d) ? y : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      } else {
        const int kr = k + bkr, j = c0 + bj;
        const float4 y = *reinterpret_cast<const float4*>(
            Wp + (size_t)(kr < d ? kr : 0) * d + (j < d ? j : 0));
        bv = (kr < d && j < d) ? y : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      }
      return;
    }
    {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kk = k + ak + u;
        const float x = arow[kk < d ? kk : 0];
        v[u] = (a_ok && kk < d) ? x : 0.0f;
      }
      av = make_float4(v[0], v[1], v[2], v[3]);
    }
    float v[4];
    if (prod == 0) {
      const int r = c0 + bi, rc = r < d ? r : 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kk = k + bk + u;
        const float x = Wp[(size_t)rc * d + (kk < d ? kk : 0)];
        v[u] = (r < d && kk < d) ? x : 0.0f;
      }
    } else {
      const int kk = k + bkr, kc = kk < d ? kk : 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = c0 + bj + u;
        const float x = Wp[(size_t)kc * d + (j < d ? j : 0)];
        v[u] = (kk < d && j < d) ? x : 0.0f;
      }
    }
    bv = make_float4(v[0], v[1], v[2], v[3]);
  };
  auto store_step = [&](int buf, const float4& av, const float4& bv) {
    *reinterpret_cast<float4*>(&sA[buf][ai][ak]) = av;
    if (prod == 0) {   // B[k][r] = W[r][k]
      sB[buf][bk + 0][bi] = bv.x;
      sB[buf][bk + 1][bi] = bv.y;
      sB[buf][bk + 2][bi] = bv.z;
      sB[buf][bk + 3][bi] = bv.w;
    } else {
      *reinterpret_cast<float4*>(&sB[buf][bkr][bj]) = bv;
    }
  };
  f32x4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  // PF steps of loads in flight: regs[u] holds step ks0 + u until it is staged
  float4 ra[PF], rb[PF];
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < nk) load_step(u, ra[u], rb[u]);
  const int row = wave * 16 + (l & 15), kq = l >> 4;
  for (int ks0 = 0; ks0 < nk; ks0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int ks = ks0 + u;
      if (ks >= nk) break;
      const int buf = ks & 1;
      store_step(buf, ra[u], rb[u]);
      __syncthreads();
      if (ks + PF < nk) load_step(ks + PF, ra[u], rb[u]);
#ifndef SKGE_RS_ABL_NOMFMA
#pragma unroll
      for (int k4 = 0; k4 < KS; k4 += 4) {
        const float a = sA[buf][row][k4 + kq];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, sB[buf][k4 + kq][q * 16 + (l & 15)],
                                                        acc[q], 0, 0, 0);
      }
#else
      acc[0][0] += sA[buf][row][kq] + sB[buf][kq][l & 15];
#endif
    }
  }
  // epilogue: D[row 4g + reg][col] of accumulator q -> triple 16w + 4g + reg, column c0 + 16q + c
#ifdef SKGE_RS_ABL_NOEPI
  if (acc[0][0] == 12345.0f) ws.WE[0] = acc[1][1] + acc[2][2] + acc[3][3];
  return;
#endif
  float* out = prod == 0 ? ws.WE : ws.EW;
  const int g = l >> 4, c = l & 15;
  float ps[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int col = c0 + q * 16 + c;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int it = wave * 16 + 4 * g + reg;
      if (it < cnt && col < d) out[(size_t)s_gid[it] * d + col] = acc[q][reg];
      if (prod == 0) {
        const float e = E[(size_t)s_es[it] * d + (col < d ? col : 0)];
        ps[reg] += (col < d) ? acc[q][reg] * e : 0.0f;
      }
    }
  }
  if (prod == 0) {
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      float v = ps[reg];
      v += __shfl_xor(v, 8, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 1, 64);
      const int it = wave * 16 + 4 * g + reg;
      if (c == 0 && it < cnt) ws.spart[(size_t)s_gid[it] * ncb + cb] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// margin test + entity contributions, one wave per pair (rescal.py:264-302)
// ---------------------------------------------------------------------------
template <int KM>
__global__ __launch_bounds__(256) void k_rescal_scatter(const int* __restrict__ pos,
                                                        const int* __restrict__ neg, int P, int d,
                                                        int af, float margin, RescalWs ws,
                                                        Accum accE, float* pscore, float* nscore,
                                                        int* nviol) {
  const int wpb = blockDim.x >> 6;
  int nv = 0;
  for (int i = blockIdx.x * wpb + (threadIdx.x >> 6); i < P; i += gridDim.x * wpb) {
    const int ix[6] = {__builtin_amdgcn_readfirstlane(pos[3 * i]),
                       __builtin_amdgcn_readfirstlane(pos[3 * i + 1]),
                       __builtin_amdgcn_readfirstlane(pos[3 * i + 2]),
                       __builtin_amdgcn_readfirstlane(neg[3 * i]),
                       __builtin_amdgcn_readfirstlane(neg[3 * i + 1]),
                       __builtin_amdgcn_readfirstlane(neg[3 * i + 2])};
    if (ix[2] < 0) {   // skipped pair: never bucketed (relation -1), no contribution
      commit_pair(accE, nullptr, false, ix, i);
      continue;
    }
    const int ncb = (d + GC - 1) / GC;
    float praw = 0.0f, nraw = 0.0f;
    for (int q = 0; q < ncb; ++q) {   // fixed order: deterministic
      praw += ws.spart[(size_t)i * ncb + q];
      nraw += ws.spart[(size_t)(P + i) * ncb + q];
    }
    const float pf = af_f(af, praw), nf = af_f(af, nraw);
    const float gp = -af_g_given_f(af, pf);   // rescal.py:275 (all pairs)
    const float gn = af_g_given_f(af, nf);
    if (lane_id() == 0) {
      if (pscore) pscore[i] = praw;
      if (nscore) nscore[i] = nraw;
      ws.coef[ws.bpos[i]] = gp;
      ws.coef[ws.bpos[P + i]] = gn;
    }
    const bool viol = nf + margin > pf;   // rescal.py:269
    commit_pair(accE, nullptr, viol, ix, i);
    if (!viol) continue;
    ++nv;
    float wep[KM], wen[KM], ewp[KM], ewn[KM], x[KM], y[KM];
    load_row<KM>(ws.WE, i, d, wep);
    load_row<KM>(ws.WE, P + i, d, wen);
    load_row<KM>(ws.EW, i, d, ewp);
    load_row<KM>(ws.EW, P + i, d, ewn);
    // (sp, sn) <- (gp WEp, gn WEn)                    rescal.py:299-300
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      x[k] = gp * wep[k];
      y[k] = gn * wen[k];
    }
    acc_two<KM>(accE, ix[0], x, ix[3], y, d);
    // (op, on) <- (gp EWp, gn EWn)                    rescal.py:296-301
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      x[k] = gp * ewp[k];
      y[k] = gn * ewn[k];
    }
    acc_two<KM>(accE, ix[1], x, ix[4], y, d);
  }
  __shared__ int lds_nv;
  if (nviol) block_count_add(nviol, nv, &lds_nv);
}

// ---------------------------------------------------------------------------
// logistic loss + entity contributions, one wave per labelled triple
// (rescal.py:37-76): fs = -y sigmoid(-y f); E[s] += fs WE, E[o] += fs EW
// ---------------------------------------------------------------------------
template <int KM>
__global__ __launch_bounds__(256) void k_rescal_logistic(const int* __restrict__ trip,
                                                         const float* __restrict__ ys, int T,
                                                         int d, RescalWs ws, Accum accE,
                                                         float* score_out, float* loss) {
  const int wpb = blockDim.x >> 6, ncb = (d + GC - 1) / GC;
  float lsum = 0.0f;
  for (int i = blockIdx.x * wpb + (threadIdx.x >> 6); i < T; i += gridDim.x * wpb) {
    const int s = __builtin_amdgcn_readfirstlane(trip[3 * i]);
    const int o = __builtin_amdgcn_readfirstlane(trip[3 * i + 1]);
    float score = 0.0f;
    for (int q = 0; q < ncb; ++q) score += ws.spart[(size_t)i * ncb + q];   // fixed order
    const float y = ys[i];
    const float ysc = y * score;
    const float li = fmaxf(-ysc, 0.0f) + log1pf(expf(-fabsf(ysc)));   // logaddexp(0, -ys)
    const float fs = -(y * (1.0f / (1.0f + expf(ysc))));                 // -(y sigmoid(-ys))
    if (lane_id() == 0) {
      if (score_out) score_out[i] = score;
      ws.coef[ws.bpos[i]] = fs;
    }
    {
      const int l = lane_id();   // entity occurrences (s, o): slots 2i, 2i+1
      if (l < 2) commit_slot(accE, l == 0 ? s : o, s == o ? (l == 0 ? 2 : 0) : 1, 2 * i + l);
    }
    float we[KM], ew[KM], x[KM], yv[KM];
    load_row<KM>(ws.WE, i, d, we);
    load_row<KM>(ws.EW, i, d, ew);
#pragma unroll
    for (int k = 0; k < KM; ++k) {   // rescal.py:65-66 (fs WE over ss, fs EW over os)
      x[k] = fs * we[k];
      yv[k] = fs * ew[k];
    }
    acc_two<KM>(accE, s, x, o, yv, d);
    lsum += li;
  }
  __shared__ float lds_loss;
  if (loss) block_sum_add(loss, lsum, &lds_loss);
}

// ---------------------------------------------------------------------------
// dW[p] = sum_items coef_i E[s_i] (x) E[o_i]: one workgroup per (relation,
// 16-row strip, 4 x 16-column tiles); K = the relation's triples in bucket order
// ---------------------------------------------------------------------------
constexpr int WG_CHUNK = 128;

__global__ __launch_bounds__(256) void k_rescal_wgrad_mfma(const float* __restrict__ E, int d,
                                                           RescalWs ws, Accum accW) {
  const int dp = (d + 15) & ~15, ntd = dp / 16, ngrp = (ntd + 3) / 4;
  const int blk = blockIdx.x;
  const int p = blk / (ntd * ngrp);
  const int rem = blk - p * ntd * ngrp;
  const int rt = rem / ngrp, cg = rem - (rem / ngrp) * ngrp;
  const int tid = threadIdx.x, l = lane_id(), wave = tid >> 6;
  const int off = ws.rel_off[p], cnt = ws.rel_off[p + 1] - off;
  if (rem == 0 && tid == 0) {   // slot p (skge_hip.h slot map)
    if (accW.touched) accW.touched[p] = cnt > 0 ? p : -1;
    accW.cnt[p] = cnt;
  }
  if (cnt == 0) return;
  __shared__ float sEs[WG_CHUNK][16];
  __shared__ float sEo[WG_CHUNK][64 + 4];
  __shared__ int s_s[WG_CHUNK], s_o[WG_CHUNK];
  __shared__ float s_c[WG_CHUNK];
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  const int r0 = rt * 16, c0 = cg * 64;
  for (int b0 = 0; b0 < cnt; b0 += WG_CHUNK) {
    const int m = min(WG_CHUNK, cnt - b0);
    if (tid < WG_CHUNK) {
      const int at = off + b0 + (tid < m ? tid : 0);
      s_s[tid] = ws.sorted_s[at];
      s_o[tid] = ws.sorted_o[at];
      s_c[tid] = tid < m ? ws.coef[at] : 0.0f;
    }
    __syncthreads();
    {   // every gather of this thread issued before the LDS stores wait on them
      float vs[WG_CHUNK * 16 / 256], vo[WG_CHUNK * 64 / 256];
#pragma unroll
      for (int u = 0; u < WG_CHUNK * 16 / 256; ++u) {
        const int q = tid + u * 256, i = q >> 4, cc = q & 15;
        vs[u] = E[(size_t)s_s[i] * d + (r0 + cc < d ? r0 + cc : 0)];
      }
#pragma unroll
      for (int u = 0; u < WG_CHUNK * 64 / 256; ++u) {
        const int q = tid + u * 256, i = q >> 6, cc = q & 63;
        vo[u] = E[(size_t)s_o[i] * d + (c0 + cc < d ? c0 + cc : 0)];
      }
#pragma unroll
      for (int u = 0; u < WG_CHUNK * 16 / 256; ++u) {
        const int q = tid + u * 256, i = q >> 4, cc = q & 15;
        sEs[i][cc] = (i < m && r0 + cc < d) ? s_c[i] * vs[u] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < WG_CHUNK * 64 / 256; ++u) {
        const int q = tid + u * 256, i = q >> 6, cc = q & 63;
        sEo[i][cc] = (i < m && c0 + cc < d) ? vo[u] : 0.0f;
      }
    }
    __syncthreads();
    // A[row r][k = item] = coef Es[item][r], B[k = item][col] = Eo[item][col]
    for (int k0 = 0; k0 < m; k0 += 4) {
      const int it = k0 + (l >> 4);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(sEs[it][l & 15], sEo[it][wave * 16 + (l & 15)],
                                                  acc, 0, 0, 0);
    }
    __syncthreads();
  }
  const int ct = cg * 4 + wave;
  if (ct >= ntd) return;
  float* out = accW.sum + (size_t)p * d * d;
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) {   // D[row 4g + reg][col]
    const int r = r0 + 4 * (l >> 4) + reg, cc = ct * 16 + (l & 15);
    if (r < d && cc < d) out[(size_t)r * d + cc] = acc[reg];
  }
}

}  // namespace skge

using namespace skge;

size_t skge_rescal_mfma_ws_bytes(int n, int M, int d) {
  return rescal_ws_layout(n, M, d, nullptr, nullptr);
}

bool skge_rescal_mfma_ok(int d, int M) {
  return d >= 1 && d <= RS_MAX_D && M >= 1 && M <= RS_MAX_M;
}

// bucket the n = na + nb triples (list a, then list b) by relation and run the
// two GEMMs (WE^T, EW, partial scores)
static int rescal_front(hipStream_t st, const skge_table_t* ent, const skge_table_t* rel, int d,
                        const int* a, int na, const int* b, int n, const RescalWs& ws) {
  const int M = rel->rows;
  const int nchunks = (n + 63) / 64;
  SKGE_CHECK_HIP(hipMemsetAsync(ws.chunk, 0, (size_t)nchunks * M * sizeof(int), st));
  const int cblocks = (nchunks + 3) / 4;
  hipLaunchKernelGGL(k_rs_count, dim3(cblocks), dim3(256), 0, st, a, b, na, n, M, ws);
  hipLaunchKernelGGL(k_rs_scan, dim3(1), dim3(1024), (size_t)(2 * M + 1) * sizeof(int), st, n, M,
                     ws);
  hipLaunchKernelGGL(k_rs_scatter, dim3(cblocks), dim3(256), 0, st, a, b, na, n, M, ws);
  const int ncb = (d + GC - 1) / GC;
  const dim3 ggrid((unsigned)(rs_tmax(n, M) * 2 * ncb));
  if ((d & 3) == 0)
    hipLaunchKernelGGL((k_rescal_gemm<true>), ggrid, dim3(256), 0, st, ent->param, rel->param, d,
                       ws);
  else
    hipLaunchKernelGGL((k_rescal_gemm<false>), ggrid, dim3(256), 0, st, ent->param, rel->param,
                       d, ws);
  SKGE_CHECK_LAUNCH("rescal mfma front");
  return SKGE_OK;
}

static void rescal_wgrad_launch(hipStream_t st, const skge_table_t* ent,
                                const skge_table_t* rel, int d, const RescalWs& ws) {
  const int dp = (d + 15) & ~15, ntd = dp / 16, ngrp = (ntd + 3) / 4;
  hipLaunchKernelGGL(k_rescal_wgrad_mfma, dim3((unsigned)((long long)rel->rows * ntd * ngrp)),
                     dim3(256), 0, st, ent->param, d, ws, accum_of(rel));
}

#define SKGE_KM_SWITCH(KERNEL, ...)                                             \
  switch (km_for(d)) {                                                          \
    case 1: hipLaunchKernelGGL((KERNEL<1>), __VA_ARGS__); break;                \
    case 2: hipLaunchKernelGGL((KERNEL<2>), __VA_ARGS__); break;                \
    case 3: hipLaunchKernelGGL((KERNEL<3>), __VA_ARGS__); break;                \
    case 4: hipLaunchKernelGGL((KERNEL<4>), __VA_ARGS__); break;                \
    case 8: hipLaunchKernelGGL((KERNEL<8>), __VA_ARGS__); break;                \
    case 16: hipLaunchKernelGGL((KERNEL<16>), __VA_ARGS__); break;              \
    default: set_error("d=%d unsupported on the MFMA path", d); return SKGE_ENOTSUP; \
  }

// the RESCAL pairwise gradient (entity accumulator, W accumulator) on MFMA
int skge_rescal_pair_grad_mfma(hipStream_t st, int af, const skge_table_t* ent,
                               const skge_table_t* rel, int d, const int* pos, const int* neg,
                               int P, float margin, void* workspace, size_t ws_bytes,
                               float* pscore, float* nscore, int* nviol) {
  RescalWs ws;
  const size_t need = rescal_ws_layout(2 * P, rel->rows, d, workspace, &ws);
  SKGE_CHECK_ARG(workspace && ws_bytes >= need, "RESCAL workspace needs %zu bytes", need);
  SKGE_CHECK_ARG(rel->acc_sum && rel->acc_cnt, "W accumulator missing");
  int rc = rescal_front(st, ent, rel, d, pos, P, neg, 2 * P, ws);
  if (rc) return rc;
  const int blocks = std::max(1, std::min((P + 3) / 4, 16384));
  const Accum aE = accum_of(ent);
  SKGE_KM_SWITCH(k_rescal_scatter, dim3(blocks), dim3(256), 0, st, pos, neg, P, d, af, margin, ws,
                 aE, pscore, nscore, nviol)
  rescal_wgrad_launch(st, ent, rel, d, ws);
  SKGE_CHECK_LAUNCH("rescal mfma pair grad");
  return SKGE_OK;
}

// the RESCAL logistic gradient (rescal.py:37-76) on MFMA
int skge_rescal_triple_grad_mfma(hipStream_t st, const skge_table_t* ent,
                                 const skge_table_t* rel, int d, const int* trip,
                                 const float* ys, int T, void* workspace, size_t ws_bytes,
                                 float* score, float* loss) {
  RescalWs ws;
  const size_t need = rescal_ws_layout(T, rel->rows, d, workspace, &ws);
  SKGE_CHECK_ARG(workspace && ws_bytes >= need, "RESCAL workspace needs %zu bytes", need);
  SKGE_CHECK_ARG(rel->acc_sum && rel->acc_cnt, "W accumulator missing");
  int rc = rescal_front(st, ent, rel, d, trip, T, trip, T, ws);
  if (rc) return rc;
  const int blocks = std::max(1, std::min((T + 3) / 4, 16384));
  const Accum aE = accum_of(ent);
  SKGE_KM_SWITCH(k_rescal_logistic, dim3(blocks), dim3(256), 0, st, trip, ys, T, d, ws, aE, score,
                 loss)
  rescal_wgrad_launch(st, ent, rel, d, ws);
  SKGE_CHECK_LAUNCH("rescal mfma triple grad");
  return SKGE_OK;
}
