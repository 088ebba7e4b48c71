// Filtered link-prediction ranks on the device.
//
// The reference's FilteredRankingEval.positions (skge/base.py:913-1031), with
// TransEEval (skge/run_transe.py:15-29) or HolEEval (skge/run_hole.py:12-19),
// scores every entity as the tail of (s, p, ?) and as the head of (?, p, o)
// for each test triple, sorts, and takes the position of the true entity;
// the filtered variant first sets the scores of the other known answers to
// -inf.  Here:
//   k_rank_query   one wave per test triple: the tail and head query vectors
//                  and the true entities' scores.  Every model's score over
//                  all entities is a distance or a dot product with one vector:
//                    TransE  -sum|q - E_j|   q_tail = E_s + R_p, q_head = E_o - R_p
//                            (the reference's eval uses the L1 form for both norms)
//                    HolE    E_j . q         q_tail = cconv(R_p, E_s), q_head = ccorr(R_p, E_o)
//                    RESCAL  E_j . q         q_tail = E_s W_p,        q_head = W_p E_o
//   k_rank_count   one workgroup per 64 query vectors, streaming every entity
//                  through LDS tiles; each thread scores a 4 x 4 (entity x
//                  query) micro-tile and counts the entities scoring strictly
//                  above the true one (raw), skipping known triples for the
//                  filtered count (triple-set lookups, skge_epoch.hip).
// rank = 1 + #{entities scoring strictly higher}: ties go the true entity's
// way (the reference's order among exact ties is that of numpy's unstable
// argsort, reversed).
#include <algorithm>

#include "skge_host.h"

namespace skge {

constexpr int QB = 64;    // query vectors per workgroup
constexpr int EB = 64;    // entities per LDS tile
constexpr int KC = 32;    // dims per LDS chunk

struct RankArgs {
  const float* E;
  const float* R;      // TransE / HolE: [M][d]; RESCAL: W [M][d][d]
  int N, d, model, nq;
  const int* queries;  // [nq][3] (s, o, p)
  TripleSet set;
  int has_set;
  float* Q;            // workspace [2 nq][d]: vector 2i = tail query of triple i, 2i+1 = head
  float* tgt;          // workspace [2 nq]: the true entity's score
  int* ranks;          // [nq][4]: tail raw, tail filtered, head raw, head filtered
};

// ---- query vectors and true scores: one wave per test triple ----
// The true entity's score is recomputed by lane 0 with exactly the counting
// kernel's arithmetic (sequential k, the same fma / abs expression on the
// same stored query vector), so the true entity never outranks itself.
__global__ __launch_bounds__(128) void k_rank_query(RankArgs a) {
  const int wpb = blockDim.x >> 6, l = lane_id(), d = a.d;
  extern __shared__ float sm[];
  float* sw = sm + (threadIdx.x >> 6) * 5 * d;   // E_s, E_o, R_p, q_tail, q_head
  for (int i = blockIdx.x * wpb + (threadIdx.x >> 6); i < a.nq; i += gridDim.x * wpb) {
    const int s = __builtin_amdgcn_readfirstlane(a.queries[3 * i]);
    const int o = __builtin_amdgcn_readfirstlane(a.queries[3 * i + 1]);
    const int p = __builtin_amdgcn_readfirstlane(a.queries[3 * i + 2]);
    float* es = sw;
    float* eo = sw + d;
    float* rp = sw + 2 * d;
    float* lqt = sw + 3 * d;
    float* lqh = sw + 4 * d;
    for (int k = l; k < d; k += 64) {
      es[k] = a.E[(size_t)s * d + k];
      eo[k] = a.E[(size_t)o * d + k];
      if (a.model != SKGE_RESCAL) rp[k] = a.R[(size_t)p * d + k];
    }
    __builtin_amdgcn_wave_barrier();
    float* qt = a.Q + (size_t)(2 * i) * d;
    float* qh = a.Q + (size_t)(2 * i + 1) * d;
    const float* W = a.R + (size_t)p * d * d;
    const bool l1 = a.model == SKGE_TRANSE_L1 || a.model == SKGE_TRANSE_L2;
    for (int k = l; k < d; k += 64) {
      float vt, vh;
      if (l1) {
        vt = es[k] + rp[k];
        vh = eo[k] - rp[k];
      } else if (a.model == SKGE_HOLE) {
        // cconv(R, E_s)_k = sum_j R_j E_s[(k-j) mod d]; ccorr(R, E_o)_k = sum_j R_j E_o[(j+k) mod d]
        float ct = 0.0f, ch = 0.0f;
        for (int j = 0; j < d; ++j) {
          int im = k - j;
          im += im < 0 ? d : 0;
          int ip = j + k;
          ip -= ip >= d ? d : 0;
          ct = fmaf(rp[j], es[im], ct);
          ch = fmaf(rp[j], eo[ip], ch);
        }
        vt = ct;
        vh = ch;
      } else {   // RESCAL: (E_s W)_k = sum_j E_s[j] W[j][k]; (W E_o)_k = sum_j W[k][j] E_o[j]
        float ct = 0.0f, ch = 0.0f;
        for (int j = 0; j < d; ++j) {
          ct = fmaf(es[j], W[(size_t)j * d + k], ct);
          ch = fmaf(W[(size_t)k * d + j], eo[j], ch);
        }
        vt = ct;
        vh = ch;
      }
      qt[k] = vt;
      qh[k] = vh;
      lqt[k] = vt;
      lqh[k] = vh;
    }
    __builtin_amdgcn_wave_barrier();
    if (l == 0) {   // tail: entity o under q_tail; head: entity s under q_head
      float st = 0.0f, sh = 0.0f;
      for (int k = 0; k < d; ++k) {
        if (l1) {
          st = st - fabsf(lqt[k] - eo[k]);
          sh = sh - fabsf(lqh[k] - es[k]);
        } else {
          st = fmaf(eo[k], lqt[k], st);
          sh = fmaf(es[k], lqh[k], sh);
        }
      }
      a.tgt[2 * i] = st;
      a.tgt[2 * i + 1] = sh;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ---- counting pass: 64 query vectors per workgroup, all entities ----
template <bool L1>
__global__ __launch_bounds__(256) void k_rank_count(RankArgs a) {
  __shared__ float sQ[KC][QB + 1];
  __shared__ float sE[KC][EB + 1];
  __shared__ int s_raw[QB], s_filt[QB];
  __shared__ int s_qs[QB], s_qo[QB], s_qp[QB], s_qt[QB];
  __shared__ float s_tgt[QB];
  const int tid = threadIdx.x, d = a.d;
  const int v0 = blockIdx.x * QB, nv = 2 * a.nq;
  if (tid < QB) {
    const int v = v0 + tid;
    const bool ok = v < nv;
    const int qi = ok ? v >> 1 : 0;
    s_qs[tid] = a.queries[3 * qi];
    s_qo[tid] = a.queries[3 * qi + 1];
    s_qp[tid] = a.queries[3 * qi + 2];
    s_qt[tid] = ok ? ((v & 1) ? s_qs[tid] : s_qo[tid]) : -1;   // the true entity
    s_tgt[tid] = ok ? a.tgt[v] : INFINITY;
    s_raw[tid] = 0;
    s_filt[tid] = 0;
  }
  __syncthreads();
  const int te = (tid & 15) * 4, tq = (tid >> 4) * 4;   // this thread's 4 entities x 4 queries
  int raw[4] = {0, 0, 0, 0}, filt[4] = {0, 0, 0, 0};
  for (int e0 = 0; e0 < a.N; e0 += EB) {
    float acc[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[x][y] = 0.0f;
    for (int k0 = 0; k0 < d; k0 += KC) {
      __syncthreads();
      for (int q = tid; q < KC * QB; q += 256) {   // [k][vector]: coalesced along k
        const int vv = q / KC, k = q - vv * KC;
        const int v = v0 + vv;
        const bool ok = v < nv && k0 + k < d;
        sQ[k][vv] = ok ? a.Q[(size_t)v * d + k0 + k] : 0.0f;
      }
      for (int q = tid; q < KC * EB; q += 256) {
        const int ee = q / KC, k = q - ee * KC;
        const int e = e0 + ee;
        const bool ok = e < a.N && k0 + k < d;
        sE[k][ee] = ok ? a.E[(size_t)e * d + k0 + k] : 0.0f;
      }
      __syncthreads();
      const int kn = min(KC, d - k0);
      for (int k = 0; k < kn; ++k) {
        float ev[4], qv[4];
#pragma unroll
        for (int x = 0; x < 4; ++x) ev[x] = sE[k][te + x];
#pragma unroll
        for (int y = 0; y < 4; ++y) qv[y] = sQ[k][tq + y];
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < 4; ++y)
            acc[x][y] = L1 ? acc[x][y] - fabsf(qv[y] - ev[x]) : fmaf(ev[x], qv[y], acc[x][y]);
      }
    }
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      const int vv = tq + y;
      const float t = s_tgt[vv];
      const int dir = (v0 + vv) & 1;   // 0: tail (vary o), 1: head (vary s)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int e = e0 + te + x;
        if (e < a.N && acc[x][y] > t) {
          ++raw[y];
          const bool known = a.has_set && e != s_qt[vv] &&
                             (dir == 0 ? set_contains(a.set, s_qs[vv], e, s_qp[vv])
                                       : set_contains(a.set, e, s_qo[vv], s_qp[vv]));
          if (!known) ++filt[y];
        }
      }
    }
  }
#pragma unroll
  for (int y = 0; y < 4; ++y) {
    atomicAdd(&s_raw[tq + y], raw[y]);
    atomicAdd(&s_filt[tq + y], filt[y]);
  }
  __syncthreads();
  if (tid < QB) {
    const int v = v0 + tid;
    if (v < nv) {
      const int qi = v >> 1, dir = v & 1;
      a.ranks[4 * qi + 2 * dir] = 1 + s_raw[tid];
      a.ranks[4 * qi + 2 * dir + 1] = 1 + s_filt[tid];
    }
  }
}

// ---- round 2: raw counts over entity slices + filtered counts from the
// queries' known answers ----
// rank_filtered = rank_raw - #{known answers of the query, other than the
// true entity, scoring strictly above it}: the counting pass needs no
// triple-set lookups (at random parameters half the entities score above the
// true one, so the lookups were most of the pass), and the known answers --
// a handful per query -- are scored by their own small kernel with the
// counting pass's arithmetic (sequential k).
constexpr int QB2 = 64;    // query vectors per workgroup
constexpr int EB2 = 128;   // entities per LDS tile
constexpr int KC2 = 32;    // dims per LDS chunk
constexpr int PADQ = QB2 + 4, PADE = EB2 + 4;   // rows stay 16-B aligned

struct RankArgs2 {
  const float* E;
  int N, d, nv;        // nv = 2 nq query vectors
  int eslice;          // entities per workgroup slice (multiple of EB2)
  const float* Q;      // [nv][d]
  const float* tgt;    // [nv]
  int* raw;            // [nv] entities scoring strictly higher (atomics over the slices)
};

// one workgroup: QB2 query vectors x one entity slice; thread: 8 entities x 4
// queries, every accumulator a sequential-k chain (the true score's arithmetic)
template <bool L1>
__global__ __launch_bounds__(256) void k_rank_count2(RankArgs2 a) {
  __shared__ __attribute__((aligned(16))) float sQ[KC2][PADQ];
  __shared__ __attribute__((aligned(16))) float sE[KC2][PADE];
  __shared__ int s_raw[QB2];
  __shared__ float s_tgt[QB2];
  const int tid = threadIdx.x, d = a.d;
  const int v0 = blockIdx.x * QB2;
  const int ebeg = blockIdx.y * a.eslice, eend = min(a.N, ebeg + a.eslice);
  if (tid < QB2) {
    const int v = v0 + tid;
    s_tgt[tid] = v < a.nv ? a.tgt[v] : INFINITY;
    s_raw[tid] = 0;
  }
  const int te = (tid & 15) * 8, tq = (tid >> 4) * 4;
  int raw[4] = {0, 0, 0, 0};
  // staging maps: Q chunk = 64 vectors x 8 float4 (2 per thread), E chunk =
  // 128 entities x 8 float4 (4 per thread); k fastest in global memory
  const int sq_v = tid >> 2, sq_k = (tid & 3) * 4;          // + 16 for the second float4
  const int se_e = tid >> 1, se_k = (tid & 1) * 4;          // + 8, 16, 24
  for (int e0 = ebeg; e0 < eend; e0 += EB2) {
    float acc[8][4];
#pragma unroll
    for (int x = 0; x < 8; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[x][y] = 0.0f;
    for (int k0 = 0; k0 < d; k0 += KC2) {
      float4 qa[2], ea[4];
      {
        const int v = v0 + sq_v;
        const float* qrow = a.Q + (size_t)(v < a.nv ? v : 0) * d;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int k = k0 + sq_k + 16 * u;
          float4 x = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
          if (v < a.nv) {
            if ((d & 3) == 0 && k + 3 < d) {
              x = *reinterpret_cast<const float4*>(qrow + k);
            } else {
              x.x = k < d ? qrow[k] : 0.0f;
              x.y = k + 1 < d ? qrow[k + 1] : 0.0f;
              x.z = k + 2 < d ? qrow[k + 2] : 0.0f;
              x.w = k + 3 < d ? qrow[k + 3] : 0.0f;
            }
          }
          qa[u] = x;
        }
        const int e = e0 + se_e;
        const float* erow = a.E + (size_t)(e < eend ? e : ebeg) * d;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int k = k0 + se_k + 8 * u;
          float4 x = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
          if (e < eend) {
            if ((d & 3) == 0 && k + 3 < d) {
              x = *reinterpret_cast<const float4*>(erow + k);
            } else {
              x.x = k < d ? erow[k] : 0.0f;
              x.y = k + 1 < d ? erow[k + 1] : 0.0f;
              x.z = k + 2 < d ? erow[k + 2] : 0.0f;
              x.w = k + 3 < d ? erow[k + 3] : 0.0f;
            }
          }
          ea[u] = x;
        }
      }
      __syncthreads();   // the previous chunk's reads are done
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int k = sq_k + 16 * u;
        sQ[k][sq_v] = qa[u].x;
        sQ[k + 1][sq_v] = qa[u].y;
        sQ[k + 2][sq_v] = qa[u].z;
        sQ[k + 3][sq_v] = qa[u].w;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = se_k + 8 * u;
        sE[k][se_e] = ea[u].x;
        sE[k + 1][se_e] = ea[u].y;
        sE[k + 2][se_e] = ea[u].z;
        sE[k + 3][se_e] = ea[u].w;
      }
      __syncthreads();
      const int kn = min(KC2, d - k0);
      for (int k = 0; k < kn; ++k) {
        const float4 e4a = *reinterpret_cast<const float4*>(&sE[k][te]);
        const float4 e4b = *reinterpret_cast<const float4*>(&sE[k][te + 4]);
        const float4 q4 = *reinterpret_cast<const float4*>(&sQ[k][tq]);
        const float ev[8] = {e4a.x, e4a.y, e4a.z, e4a.w, e4b.x, e4b.y, e4b.z, e4b.w};
        const float qv[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
        for (int x = 0; x < 8; ++x)
#pragma unroll
          for (int y = 0; y < 4; ++y)
            acc[x][y] = L1 ? acc[x][y] - fabsf(qv[y] - ev[x]) : fmaf(ev[x], qv[y], acc[x][y]);
      }
    }
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      const float t = s_tgt[tq + y];
#pragma unroll
      for (int x = 0; x < 8; ++x)
        if (e0 + te + x < eend && acc[x][y] > t) ++raw[y];
    }
  }
#pragma unroll
  for (int y = 0; y < 4; ++y)
    if (raw[y]) atomicAdd(&s_raw[tq + y], raw[y]);
  __syncthreads();
  if (tid < QB2) {
    const int v = v0 + tid;
    if (v < a.nv && s_raw[tid]) atomicAdd(a.raw + v, s_raw[tid]);
  }
}

// filtered correction + the ranks: one thread per query vector, its known
// answers (CSR, the true entity excluded by the caller) scored with the
// counting pass's arithmetic (sequential k)
template <bool L1>
__global__ __launch_bounds__(256) void k_rank_known(const float* __restrict__ E, int d, int nq,
                                                    const float* __restrict__ Q,
                                                    const float* __restrict__ tgt,
                                                    const int* __restrict__ raw,
                                                    const int* __restrict__ tail_off,
                                                    const int* __restrict__ tail_ent,
                                                    const int* __restrict__ head_off,
                                                    const int* __restrict__ head_ent,
                                                    int* __restrict__ ranks) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= 2 * nq) return;
  const int qi = v >> 1, dir = v & 1;   // 0: tail (vary o), 1: head (vary s)
  const int* off = dir ? head_off : tail_off;
  const int* ent = dir ? head_ent : tail_ent;
  const float* q = Q + (size_t)v * d;
  const float t = tgt[v];
  int dec = 0;
  for (int i = off[qi]; i < off[qi + 1]; ++i) {
    const float* e = E + (size_t)ent[i] * d;
    float acc = 0.0f;
    for (int k = 0; k < d; ++k) acc = L1 ? acc - fabsf(q[k] - e[k]) : fmaf(e[k], q[k], acc);
    if (acc > t) ++dec;
  }
  ranks[4 * qi + 2 * dir] = 1 + raw[v];
  ranks[4 * qi + 2 * dir + 1] = 1 + raw[v] - dec;
}

}  // namespace skge

using namespace skge;

extern "C" size_t skge_rank_known_workspace_bytes(int nq, int d) {
  return (size_t)2 * nq * d * sizeof(float) + (size_t)2 * nq * (sizeof(float) + sizeof(int)) + 512;
}

extern "C" int skge_rank_known(void* stream, int model, const float* E, const float* R, int N,
                               int d, const int* queries, int nq, const int* tail_off,
                               const int* tail_ent, const int* head_off, const int* head_ent,
                               void* workspace, size_t ws_bytes, int* ranks_out) {
  SKGE_CHECK_ARG(E && R && queries && ranks_out && tail_off && head_off, "NULL argument");
  SKGE_CHECK_ARG(model >= 0 && model <= 3, "unknown model %d", model);
  SKGE_CHECK_ARG(N > 0 && d > 0 && d <= 1024 && nq >= 0, "bad sizes (d <= 1024)");
  if (nq == 0) return SKGE_OK;
  SKGE_CHECK_ARG(workspace && ws_bytes >= skge_rank_known_workspace_bytes(nq, d),
                 "rank workspace needs %zu bytes", skge_rank_known_workspace_bytes(nq, d));
  RankArgs a = {};
  a.E = E;
  a.R = R;
  a.N = N;
  a.d = d;
  a.model = model;
  a.nq = nq;
  a.queries = queries;
  a.has_set = 0;
  a.Q = (float*)workspace;
  a.tgt = a.Q + (size_t)2 * nq * d;
  int* raw = (int*)(a.tgt + 2 * (size_t)nq);
  a.ranks = ranks_out;
  hipStream_t st = as_stream(stream);
  SKGE_CHECK_HIP(hipMemsetAsync(raw, 0, (size_t)2 * nq * sizeof(int), st));
  const int qblocks = std::max(1, std::min((nq + 1) / 2, 16384));
  hipLaunchKernelGGL(k_rank_query, dim3(qblocks), dim3(128), (size_t)2 * 5 * d * sizeof(float), st,
                     a);
  RankArgs2 b;
  b.E = E;
  b.N = N;
  b.d = d;
  b.nv = 2 * nq;
  b.Q = a.Q;
  b.tgt = a.tgt;
  b.raw = raw;
  // enough workgroups to fill the chip: query blocks x entity slices
  const int qb = (2 * nq + QB2 - 1) / QB2;
  const int tiles = (N + EB2 - 1) / EB2;
  const int want = std::max(1, std::min(tiles, (2048 + qb - 1) / qb));
  const int per = (tiles + want - 1) / want;
  b.eslice = per * EB2;
  const int ns = (tiles + per - 1) / per;
  const bool l1 = model == SKGE_TRANSE_L1 || model == SKGE_TRANSE_L2;
  if (l1)
    hipLaunchKernelGGL((k_rank_count2<true>), dim3(qb, ns), dim3(256), 0, st, b);
  else
    hipLaunchKernelGGL((k_rank_count2<false>), dim3(qb, ns), dim3(256), 0, st, b);
  const int kb = (2 * nq + 255) / 256;
  if (l1)
    hipLaunchKernelGGL((k_rank_known<true>), dim3(kb), dim3(256), 0, st, E, d, nq, a.Q, a.tgt, raw,
                       tail_off, tail_ent, head_off, head_ent, ranks_out);
  else
    hipLaunchKernelGGL((k_rank_known<false>), dim3(kb), dim3(256), 0, st, E, d, nq, a.Q, a.tgt,
                       raw, tail_off, tail_ent, head_off, head_ent, ranks_out);
  SKGE_CHECK_LAUNCH("rank (known answers)");
  return SKGE_OK;
}

extern "C" size_t skge_rank_workspace_bytes(int nq, int d) {
  return (size_t)2 * nq * d * sizeof(float) + (size_t)2 * nq * sizeof(float) + 256;
}

extern "C" int skge_rank(void* stream, int model, const float* E, const float* R, int N, int d,
                         const int* queries, int nq, const void* set, int64_t set_capacity,
                         void* workspace, size_t ws_bytes, int* ranks_out) {
  SKGE_CHECK_ARG(E && R && queries && ranks_out, "NULL argument");
  SKGE_CHECK_ARG(model >= 0 && model <= 3, "unknown model %d", model);
  SKGE_CHECK_ARG(N > 0 && d > 0 && d <= 1024 && nq >= 0, "bad sizes (d <= 1024)");
  if (nq == 0) return SKGE_OK;
  SKGE_CHECK_ARG(workspace && ws_bytes >= skge_rank_workspace_bytes(nq, d),
                 "rank workspace needs %zu bytes", skge_rank_workspace_bytes(nq, d));
  SKGE_CHECK_ARG(!set || (set_capacity >= 4 && (set_capacity & (set_capacity - 1)) == 0),
                 "set capacity must be a power of 2");
  RankArgs a = {};
  a.E = E;
  a.R = R;
  a.N = N;
  a.d = d;
  a.model = model;
  a.nq = nq;
  a.queries = queries;
  a.has_set = set ? 1 : 0;
  if (set) {
    a.set.slots = (const int4*)set;
    a.set.filter = (const uint32_t*)((const int4*)set + set_capacity);
    a.set.mask = (uint64_t)(set_capacity - 1);
    a.set.fmask = (uint64_t)(8 * set_capacity - 1);
  }
  a.Q = (float*)workspace;
  a.tgt = a.Q + (size_t)2 * nq * d;
  a.ranks = ranks_out;
  hipStream_t st = as_stream(stream);
  const int qblocks = std::max(1, std::min((nq + 1) / 2, 16384));
  hipLaunchKernelGGL(k_rank_query, dim3(qblocks), dim3(128), (size_t)2 * 5 * d * sizeof(float), st,
                     a);
  const int cblocks = (2 * nq + QB - 1) / QB;
  if (model == SKGE_TRANSE_L1 || model == SKGE_TRANSE_L2)
    hipLaunchKernelGGL((k_rank_count<true>), dim3(cblocks), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((k_rank_count<false>), dim3(cblocks), dim3(256), 0, st, a);
  SKGE_CHECK_LAUNCH("rank");
  return SKGE_OK;
}
