// Row-sharded TransE-L1 training step across G ranks (SURVEY.md 8(e),
// BASELINE configs[4]): the entity table E and its AdaGrad state are split by
// row, rank g owning the rows r with r % G == g at local index r / G; the
// relation table R is replicated.  One mini-batch of the reference's loop
// (skge/base.py:1394-1427: _pairwise_gradients + _batch_step over the union of
// every rank's positives) becomes
//
//   route      requests (s, o, s', o') of the rank's positives, bucketed by owner
//   [exchange] request ids to their owners                       (all-to-all)
//   gather     owners copy the requested rows out of their shard
//   [exchange] rows back to the requesters                        (all-to-all)
//   score      L1 scores of both pairs, strict margin test, the exact sign
//              contributions per request (int8) and into the local R sums
//   [exchange] contributions to the owners                        (all-to-all)
//   accum      owners add them into their exact packed row sums
//   [exchange] R sums and counts                                  (all-reduce)
//   apply      segment mean + AdaGrad + normalize (skge_accum_apply)
//
// The exchanges are the caller's (RCCL through torch.distributed); these
// kernels only touch device buffers.  The contributions of TransE-L1 are
// small integers, so every sum is exact and independent of the order in which
// ranks and atomics add them: a G-rank step gives, bit for bit, the parameters
// one rank would compute for the union batch.
#include "skge_host.h"

namespace skge {

constexpr int SHARD_MAX_RANKS = 64;
constexpr int ROUTE_BLOCK = 256;      // requests per route workgroup (64 positives)

// request k of positive j: 0 = s, 1 = o, 2 = s' (rec.w), 3 = o' (rec_n1); -1 = none
__device__ __forceinline__ int request_id(const int4* __restrict__ rec,
                                          const int* __restrict__ rec_n1, long long j, int k) {
  const int4 r = rec[j];
  return k == 0 ? r.x : (k == 1 ? r.y : (k == 2 ? r.w : rec_n1[j]));
}

// per-workgroup request counts per owner: bcnt[g * nblk + b]
__global__ __launch_bounds__(ROUTE_BLOCK) void k_route_count(const int4* __restrict__ rec,
                                                             const int* __restrict__ rec_n1,
                                                             long long start, int cnt, int G,
                                                             int* __restrict__ bcnt) {
  __shared__ int c[SHARD_MAX_RANKS];
  const int nblk = gridDim.x;
  if (threadIdx.x < G) c[threadIdx.x] = 0;
  __syncthreads();
  const long long i = (long long)blockIdx.x * ROUTE_BLOCK + threadIdx.x;   // request index
  if (i < 4ll * cnt) {
    const int id = request_id(rec, rec_n1, start + (i >> 2), (int)(i & 3));
    if (id >= 0) atomicAdd(&c[id % G], 1);
  }
  __syncthreads();
  if (threadIdx.x < G) bcnt[threadIdx.x * nblk + blockIdx.x] = c[threadIdx.x];
}

// one workgroup: exclusive offsets of every (owner, workgroup) cell in the
// owner-major send buffer, and the bucket sizes (int64, the all-to-all splits)
__global__ __launch_bounds__(256) void k_route_scan(int* __restrict__ bcnt, int nblk, int G,
                                                    long long* __restrict__ counts) {
  __shared__ int part[256];
  int base = 0;
  for (int g = 0; g < G; ++g) {
    int run = base;
    for (int b0 = 0; b0 < nblk; b0 += 256) {
      const int b = b0 + threadIdx.x;
      const int v = b < nblk ? bcnt[g * nblk + b] : 0;
      part[threadIdx.x] = v;
      __syncthreads();
      // Hillis-Steele inclusive scan over the 256 values
      for (int off = 1; off < 256; off <<= 1) {
        const int t = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += t;
        __syncthreads();
      }
      if (b < nblk) bcnt[g * nblk + b] = run + part[threadIdx.x] - v;
      run += part[255];
      __syncthreads();
    }
    if (threadIdx.x == 0) counts[g] = run - base;
    base = run;
  }
}

// stable scatter: request i goes to send slot off (owner-major, request order
// inside a bucket); req_pos[i] = off (-1 for no request)
__global__ __launch_bounds__(ROUTE_BLOCK) void k_route_scatter(
    const int4* __restrict__ rec, const int* __restrict__ rec_n1, long long start, int cnt, int G,
    const int* __restrict__ boff, int* __restrict__ send_ids, int* __restrict__ req_pos) {
  __shared__ int wcnt[ROUTE_BLOCK / 64][SHARD_MAX_RANKS];
  const int nblk = gridDim.x;
  const int l = lane_id(), wv = threadIdx.x >> 6;
  const long long i = (long long)blockIdx.x * ROUTE_BLOCK + threadIdx.x;
  const bool in = i < 4ll * cnt;
  const int id = in ? request_id(rec, rec_n1, start + (i >> 2), (int)(i & 3)) : -1;
  const int owner = id >= 0 ? id % G : -1;
  const uint64_t lt = (1ull << l) - 1ull;
  int rank_in_wave = 0;
  for (int g = 0; g < G; ++g) {
    const uint64_t m = __ballot(owner == g);
    if (owner == g) rank_in_wave = __popcll(m & lt);
    if (l == 0) wcnt[wv][g] = __popcll(m);
  }
  __syncthreads();
  if (!in) return;
  if (owner < 0) {
    req_pos[i] = -1;
    return;
  }
  int off = boff[owner * nblk + blockIdx.x] + rank_in_wave;
  for (int w = 0; w < wv; ++w) off += wcnt[w][owner];
  send_ids[off] = id;
  req_pos[i] = off;
}

// Fixed-capacity layout (graph-capturable step, no host-side split sizes):
// the send buffer holds G buckets of C request slots each, bucket g = owner g,
// request order inside a bucket, unused slots -1.  Offsets inside each bucket:
// the same per-(owner, workgroup) exclusive scan with every bucket starting at
// 0; a bucket past C raises *err (the runner checks it after the epoch).
__global__ __launch_bounds__(256) void k_route_scan_cap(int* __restrict__ bcnt, int nblk, int G) {
  __shared__ int part[256];
  for (int g = 0; g < G; ++g) {
    int run = 0;
    for (int b0 = 0; b0 < nblk; b0 += 256) {
      const int b = b0 + threadIdx.x;
      const int v = b < nblk ? bcnt[g * nblk + b] : 0;
      part[threadIdx.x] = v;
      __syncthreads();
      for (int off = 1; off < 256; off <<= 1) {
        const int t = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += t;
        __syncthreads();
      }
      if (b < nblk) bcnt[g * nblk + b] = run + part[threadIdx.x] - v;
      run += part[255];
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(ROUTE_BLOCK) void k_route_scatter_cap(
    const int4* __restrict__ rec, const int* __restrict__ rec_n1, long long start, int cnt, int G,
    int C, const int* __restrict__ boff, int* __restrict__ send_ids, int* __restrict__ req_pos,
    int* __restrict__ err) {
  __shared__ int wcnt[ROUTE_BLOCK / 64][SHARD_MAX_RANKS];
  const int nblk = gridDim.x;
  const int l = lane_id(), wv = threadIdx.x >> 6;
  const long long i = (long long)blockIdx.x * ROUTE_BLOCK + threadIdx.x;
  const bool in = i < 4ll * cnt;
  const int id = in ? request_id(rec, rec_n1, start + (i >> 2), (int)(i & 3)) : -1;
  const int owner = id >= 0 ? id % G : -1;
  const uint64_t lt = (1ull << l) - 1ull;
  int rank_in_wave = 0;
  for (int g = 0; g < G; ++g) {
    const uint64_t m = __ballot(owner == g);
    if (owner == g) rank_in_wave = __popcll(m & lt);
    if (l == 0) wcnt[wv][g] = __popcll(m);
  }
  __syncthreads();
  if (!in) return;
  if (owner < 0) {
    req_pos[i] = -1;
    return;
  }
  int off = boff[owner * nblk + blockIdx.x] + rank_in_wave;
  for (int w = 0; w < wv; ++w) off += wcnt[w][owner];
  if (off >= C) {            // bucket overflow: flagged, the request dropped
    atomicOr(err, 1);
    req_pos[i] = -1;
    return;
  }
  send_ids[owner * C + off] = id;
  req_pos[i] = owner * C + off;
}

// owner side: rows_out[i] = E_shard[ids[i] / G] (ids[i] < 0: an unused slot,
// nothing written); one wave per row, 16-B lanes
__global__ __launch_bounds__(256) void k_shard_gather(const float* __restrict__ E, int d, int G,
                                                      const int* __restrict__ ids, long long n,
                                                      float* __restrict__ rows_out) {
  const int wpb = blockDim.x >> 6, l = lane_id(), nq = d >> 2;
  for (long long w = (long long)blockIdx.x * wpb + (threadIdx.x >> 6); w < n;
       w += (long long)gridDim.x * wpb) {
    const int id = __builtin_amdgcn_readfirstlane(ids[w]);
    if (id < 0) continue;
    const int row = id / G;
    const float4* src = reinterpret_cast<const float4*>(E + (size_t)row * d);
    float4* dst = reinterpret_cast<float4*>(rows_out + (size_t)w * d);
    for (int q = l; q < nq; q += 64) dst[q] = src[q];
  }
}

// contribution record of one request: int32 count, 12 pad bytes, int8[d]
__host__ __device__ __forceinline__ long long contrib_stride(int d) { return 16 + ((d + 15) & ~15); }

__device__ __forceinline__ uint32_t pack_i8x4(const float4& c) {
  return (uint32_t)(uint8_t)(int8_t)c.x | (uint32_t)(uint8_t)(int8_t)c.y << 8 |
         (uint32_t)(uint8_t)(int8_t)c.z << 16 | (uint32_t)(uint8_t)(int8_t)c.w << 24;
}
__device__ __forceinline__ float4 unpack_i8x4(uint32_t u) {
  return make_float4((float)(int8_t)(u & 0xFF), (float)(int8_t)((u >> 8) & 0xFF),
                     (float)(int8_t)((u >> 16) & 0xFF), (float)(int8_t)(u >> 24));
}

template <int KQ>
__device__ __forceinline__ void store_contrib(uint8_t* __restrict__ C, long long stride, int pos,
                                              int c, const float4 (&v)[KQ], int d) {
  if (pos < 0) return;       // a request dropped on bucket overflow: no record slot
  uint8_t* rec = C + (size_t)pos * stride;
  const int l = lane_id(), nq = d >> 2;
  if (l == 0) *reinterpret_cast<int*>(rec) = c;
  if (c == 0) return;
  uint32_t* pay = reinterpret_cast<uint32_t*>(rec + 16);
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l;
    if (q < nq) pay[q] = pack_i8x4(v[m]);
  }
}

template <int KQ>
__device__ __forceinline__ void load_fetched(const float* __restrict__ F, int pos, int d,
                                             float4 (&v)[KQ]) {
  load_row4<KQ>(F, pos < 0 ? 0 : pos, d, v);
}

struct ShardScoreArgs {
  const int4* rec;
  const int* rec_n1;
  long long start;
  int count, d;
  const float* F;          // fetched rows [n_send][d]
  const int* req_pos;      // [4 * count]
  const float* R;
  Accum accR;              // dense, packed
  uint8_t* C;              // contribution records [n_send][stride]
  long long cstride;
  float margin;
  int* vshards;            // violation shards (NSHARD words, SHARD_STRIDE apart)
};

// One wave per positive: the arithmetic of k_transe_l1_sample_grad_i16
// (skge_epoch.hip; transe.py:25-46, 48-165) on rows fetched from their owners.
template <int KQ>
__global__ __launch_bounds__(256) void k_shard_score(ShardScoreArgs a) {
  const int wpb = blockDim.x >> 6, l = lane_id(), d = a.d;
  int nv = 0;
  for (int w = blockIdx.x * wpb + (threadIdx.x >> 6); w < a.count; w += gridDim.x * wpb) {
    const long long j = a.start + w;
    const int4 r = a.rec[j];
    const int p = __builtin_amdgcn_readfirstlane(r.z);
    const int ps_ = __builtin_amdgcn_readfirstlane(a.req_pos[4 * w + 0]);
    const int po_ = __builtin_amdgcn_readfirstlane(a.req_pos[4 * w + 1]);
    const int p0_ = __builtin_amdgcn_readfirstlane(a.req_pos[4 * w + 2]);
    const int p1_ = __builtin_amdgcn_readfirstlane(a.req_pos[4 * w + 3]);
    // bucket overflow dropped the positive's own s / o row (error flagged by the
    // route kernel): the positive is skipped whole -- no contributions, no
    // relation sums, no violations -- rather than scored against a wrong row
    if (ps_ < 0 || po_ < 0) {
      // the slots this positive still holds carry a zero count (the record
      // buffer is reused across batches: a stale count must not be re-added)
      float4 z[KQ];
#pragma unroll
      for (int m = 0; m < KQ; ++m) z[m] = make_float4(0.f, 0.f, 0.f, 0.f);
      store_contrib<KQ>(a.C, a.cstride, ps_, 0, z, d);
      store_contrib<KQ>(a.C, a.cstride, po_, 0, z, d);
      store_contrib<KQ>(a.C, a.cstride, p0_, 0, z, d);
      store_contrib<KQ>(a.C, a.cstride, p1_, 0, z, d);
      continue;
    }
    float4 es[KQ], eo[KQ], fs[KQ], fo[KQ], rp[KQ];
    load_fetched<KQ>(a.F, ps_, d, es);
    load_fetched<KQ>(a.F, po_, d, eo);
    load_fetched<KQ>(a.F, p0_, d, fs);
    load_fetched<KQ>(a.F, p1_, d, fo);
    load_row4<KQ>(a.R, p, d, rp);
    float ps = 0.0f, n0 = 0.0f, n1 = 0.0f;
    float4 gp[KQ], g0[KQ], g1[KQ];
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
    const int v0 = (p0_ >= 0 && ns0 + a.margin > pscore) ? 1 : 0;   // strict >, transe.py:73
    const int v1 = (p1_ >= 0 && ns1 + a.margin > pscore) ? 1 : 0;
    nv += v0 + v1;
    // pair 0 lists (sp,op,sn,on) = (s,o,s',o), pair 1 = (s,o,s,o'):
    // rows s, o, s', o' receive (cs, co, c0, c1) with counts (v0+2v1, 2v0+v1, v0, v1)
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
    store_contrib<KQ>(a.C, a.cstride, ps_, v0 + 2 * v1, cs, d);
    store_contrib<KQ>(a.C, a.cstride, po_, 2 * v0 + v1, co, d);
    if (p0_ >= 0) store_contrib<KQ>(a.C, a.cstride, p0_, v0, c0, d);
    if (p1_ >= 0) store_contrib<KQ>(a.C, a.cstride, p1_, v1, c1, d);
    if (v0 + v1) {
      const Accum aR = replica(a.accR, j);
      if (l == 0) atomicAdd(aR.cnt + p, 2 * (v0 + v1));
      acc_row4_i16<KQ>(aR, p, cr, d);
    }
  }
  if (l == 0 && nv) atomicAdd(shard_of(a.vshards), nv);
}

// owner side: add received contribution i into the exact packed sums of local
// row ids[i] / G and record it in touched slot i (-1 when it carries nothing)
template <int KQ>
__global__ __launch_bounds__(256) void k_shard_accum(Accum acc, int d, int G,
                                                     const int* __restrict__ ids,
                                                     const uint8_t* __restrict__ C,
                                                     long long cstride, long long n) {
  const int wpb = blockDim.x >> 6, l = lane_id(), nq = d >> 2;
  for (long long w = (long long)blockIdx.x * wpb + (threadIdx.x >> 6); w < n;
       w += (long long)gridDim.x * wpb) {
    const uint8_t* rec = C + (size_t)w * cstride;
    const int id = __builtin_amdgcn_readfirstlane(ids[w]);
    if (id < 0) {              // an unused slot of the fixed-capacity layout
      if (l == 0) acc.touched[w] = -1;
      continue;
    }
    const int c = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const int*>(rec));
    const int row = id / G;
    if (l == 0) commit_slot(acc, row, c, (int)w);
    if (c == 0) continue;
    const uint32_t* pay = reinterpret_cast<const uint32_t*>(rec + 16);
    unsigned long long* base = reinterpret_cast<unsigned long long*>(acc.sum) + (size_t)row * nq;
#pragma unroll
    for (int m = 0; m < KQ; ++m) {
      const int q = 64 * m + l;
      if (q < nq) {
        const uint32_t u = pay[q];
        if (u) atomicAdd(base + q, pack_i16x4(unpack_i8x4(u)));
      }
    }
  }
}

__global__ void k_fold_vshards(int* shards, int* nviol) { fold_shards(shards, nviol); }

static int blocks_for_waves(long long waves) {
  long long b = (waves + 3) / 4;
  if (b < 1) b = 1;
  if (b > 16384) b = 16384;
  return (int)b;
}

}  // namespace skge

using namespace skge;

extern "C" size_t skge_shard_route_workspace_bytes(int count, int G) {
  const long long nblk = (4ll * count + ROUTE_BLOCK - 1) / ROUTE_BLOCK;
  return (size_t)(nblk > 0 ? nblk : 1) * (size_t)G * sizeof(int) + 256;
}

extern "C" long long skge_shard_contrib_stride(int d) { return contrib_stride(d); }

extern "C" int skge_shard_route(void* stream, const int* rec, const int* rec_n1, int64_t start,
                                int count, int G, int* send_ids, int* req_pos,
                                long long* counts, void* workspace, size_t ws_bytes) {
  SKGE_CHECK_ARG(rec && rec_n1 && send_ids && req_pos && counts, "NULL argument");
  SKGE_CHECK_ARG(G >= 1 && G <= SHARD_MAX_RANKS, "G must be 1..%d", SHARD_MAX_RANKS);
  SKGE_CHECK_ARG(count >= 0 && start >= 0, "bad batch range");
  SKGE_CHECK_ARG(workspace && ws_bytes >= skge_shard_route_workspace_bytes(count, G),
                 "workspace too small");
  hipStream_t st = as_stream(stream);
  if (count == 0) {
    SKGE_CHECK_HIP(hipMemsetAsync(counts, 0, sizeof(long long) * G, st));
    return SKGE_OK;
  }
  const long long nblk = (4ll * count + ROUTE_BLOCK - 1) / ROUTE_BLOCK;
  SKGE_CHECK_ARG(nblk <= (1ll << 30), "batch too large");
  int* bcnt = (int*)workspace;
  hipLaunchKernelGGL(k_route_count, dim3((unsigned)nblk), dim3(ROUTE_BLOCK), 0, st,
                     (const int4*)rec, rec_n1, (long long)start, count, G, bcnt);
  hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(256), 0, st, bcnt, (int)nblk, G, counts);
  hipLaunchKernelGGL(k_route_scatter, dim3((unsigned)nblk), dim3(ROUTE_BLOCK), 0, st,
                     (const int4*)rec, rec_n1, (long long)start, count, G, bcnt, send_ids, req_pos);
  SKGE_CHECK_LAUNCH("shard route");
  return SKGE_OK;
}

extern "C" int skge_shard_route_cap(void* stream, const int* rec, const int* rec_n1,
                                    int64_t start, int count, int G, int C, int* send_ids,
                                    int* req_pos, void* workspace, size_t ws_bytes, int* err) {
  SKGE_CHECK_ARG(rec && rec_n1 && send_ids && req_pos && err, "NULL argument");
  SKGE_CHECK_ARG(G >= 1 && G <= SHARD_MAX_RANKS, "G must be 1..%d", SHARD_MAX_RANKS);
  SKGE_CHECK_ARG(count >= 0 && start >= 0 && C >= 1, "bad batch range / capacity");
  SKGE_CHECK_ARG(workspace && ws_bytes >= skge_shard_route_workspace_bytes(count, G),
                 "workspace too small");
  hipStream_t st = as_stream(stream);
  SKGE_CHECK_HIP(hipMemsetAsync(send_ids, 0xFF, sizeof(int) * (size_t)G * C, st));   // -1
  if (count == 0) return SKGE_OK;
  const long long nblk = (4ll * count + ROUTE_BLOCK - 1) / ROUTE_BLOCK;
  SKGE_CHECK_ARG(nblk <= (1ll << 30), "batch too large");
  int* bcnt = (int*)workspace;
  hipLaunchKernelGGL(k_route_count, dim3((unsigned)nblk), dim3(ROUTE_BLOCK), 0, st,
                     (const int4*)rec, rec_n1, (long long)start, count, G, bcnt);
  hipLaunchKernelGGL(k_route_scan_cap, dim3(1), dim3(256), 0, st, bcnt, (int)nblk, G);
  hipLaunchKernelGGL(k_route_scatter_cap, dim3((unsigned)nblk), dim3(ROUTE_BLOCK), 0, st,
                     (const int4*)rec, rec_n1, (long long)start, count, G, C, bcnt, send_ids,
                     req_pos, err);
  SKGE_CHECK_LAUNCH("shard route (fixed capacity)");
  return SKGE_OK;
}

extern "C" int skge_shard_gather(void* stream, const float* E_shard, int d, int G,
                                 const int* ids, int64_t n, float* rows_out) {
  SKGE_CHECK_ARG(G >= 1 && G <= SHARD_MAX_RANKS, "G must be 1..%d", SHARD_MAX_RANKS);
  SKGE_CHECK_ARG(d > 0 && d % 4 == 0, "d must be a positive multiple of 4");
  if (n == 0) return SKGE_OK;
  SKGE_CHECK_ARG(E_shard && ids && rows_out, "NULL argument");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(k_shard_gather, dim3(blocks_for_waves(n)), dim3(256), 0, st, E_shard, d, G,
                     ids, (long long)n, rows_out);
  SKGE_CHECK_LAUNCH("shard gather");
  return SKGE_OK;
}

extern "C" int skge_shard_score(void* stream, const skge_table_t* rel, int d, const int* rec,
                                const int* rec_n1, int64_t start, int count, const float* fetched,
                                const int* req_pos, float margin, void* contrib, int* vshards) {
  int rc;
  if ((rc = check_table(rel, "rel", true))) return rc;
  SKGE_CHECK_ARG(rel->acc_mode == SKGE_ACC_I16X4 && rel->acc_touched == nullptr &&
                     rel->width == d,
                 "rel: dense packed accumulator of width d needed");
  SKGE_CHECK_ARG(d % 4 == 0 && d <= 1024, "d must be a multiple of 4, <= 1024");
  SKGE_CHECK_ARG(count >= 0 && start >= 0, "bad batch range");
  if (count == 0) return SKGE_OK;
  SKGE_CHECK_ARG(rec && rec_n1 && fetched && req_pos && contrib && vshards, "NULL argument");
  hipStream_t st = as_stream(stream);
  ShardScoreArgs a;
  a.rec = (const int4*)rec;
  a.rec_n1 = rec_n1;
  a.start = start;
  a.count = count;
  a.d = d;
  a.F = fetched;
  a.req_pos = req_pos;
  a.R = rel->param;
  a.accR = accum_of(rel);
  a.C = (uint8_t*)contrib;
  a.cstride = contrib_stride(d);
  a.margin = margin;
  a.vshards = vshards;
  const int kq = (d / 4 + 63) / 64;
  const int blocks = blocks_for_waves(count);
  if (kq <= 1) hipLaunchKernelGGL((k_shard_score<1>), dim3(blocks), dim3(256), 0, st, a);
  else if (kq <= 2) hipLaunchKernelGGL((k_shard_score<2>), dim3(blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((k_shard_score<4>), dim3(blocks), dim3(256), 0, st, a);
  SKGE_CHECK_LAUNCH("shard score");
  return SKGE_OK;
}

extern "C" int skge_shard_accum(void* stream, const skge_table_t* ent_shard, int G, const int* ids,
                                const void* contrib, int64_t n) {
  int rc;
  if ((rc = check_table(ent_shard, "ent", true))) return rc;
  SKGE_CHECK_ARG(G >= 1 && G <= SHARD_MAX_RANKS, "G must be 1..%d", SHARD_MAX_RANKS);
  SKGE_CHECK_ARG(ent_shard->acc_mode == SKGE_ACC_I16X4 && ent_shard->acc_touched &&
                     ent_shard->acc_replicas <= 1,
                 "ent: packed single-copy accumulator with slot records needed");
  if ((rc = check_slots(ent_shard, n, "ent"))) return rc;
  if (n == 0) return SKGE_OK;
  SKGE_CHECK_ARG(ids && contrib, "NULL argument");
  hipStream_t st = as_stream(stream);
  const int d = ent_shard->width, kq = (d / 4 + 63) / 64;
  const Accum acc = accum_of(ent_shard);
  const long long cs = contrib_stride(d);
  const int blocks = blocks_for_waves(n);
  if (kq <= 1)
    hipLaunchKernelGGL((k_shard_accum<1>), dim3(blocks), dim3(256), 0, st, acc, d, G, ids,
                       (const uint8_t*)contrib, cs, (long long)n);
  else if (kq <= 2)
    hipLaunchKernelGGL((k_shard_accum<2>), dim3(blocks), dim3(256), 0, st, acc, d, G, ids,
                       (const uint8_t*)contrib, cs, (long long)n);
  else
    hipLaunchKernelGGL((k_shard_accum<4>), dim3(blocks), dim3(256), 0, st, acc, d, G, ids,
                       (const uint8_t*)contrib, cs, (long long)n);
  SKGE_CHECK_LAUNCH("shard accum");
  return SKGE_OK;
}

extern "C" int skge_shard_fold_violations(void* stream, int* vshards, int* nviol_total) {
  SKGE_CHECK_ARG(vshards, "NULL argument");
  hipLaunchKernelGGL(k_fold_vshards, dim3(1), dim3(64), 0, as_stream(stream), vshards, nviol_total);
  SKGE_CHECK_LAUNCH("fold violations");
  return SKGE_OK;
}
