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

}  // namespace skge

using namespace skge;

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
