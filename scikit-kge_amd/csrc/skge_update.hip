// Segment mean + updater + projection kernels (skge/param.py:108-174,
// skge/util.py:53-101, StochasticTrainer._batch_step skge/base.py:1306-1316).
//
// Narrow rows (width <= 1024: E, R) are updated by one wavefront per row with
// the row in registers, so the projection's row norm is a wave reduction and
// the row is read and written exactly once.  Wide rows (RESCAL's W, width
// d*d, no projection) are updated elementwise.
#include "skge_host.h"

namespace skge {

struct TableDev {
  float* P;
  float* A;
  Accum acc;
  int rows, width, opt, post;
  float lr, rin, rout, fdiv;
  const int* gate;
};

static TableDev table_dev(const skge_table_t* t) {
  TableDev d;
  d.P = t->param;
  d.A = t->state;
  d.acc = accum_of(t);
  d.rows = t->rows;
  d.width = t->width;
  d.opt = t->opt;
  d.post = t->post;
  d.lr = t->lr;
  d.rin = t->rin;
  d.rout = t->rout;
  d.fdiv = t->fixed_div;
  d.gate = t->gate;
  return d;
}

struct Tables4 {
  TableDev t[4];
  int nslots[4];
  int n;
};

// SGD._update / AdaGrad._update + post projection for one register-resident row
template <int KM>
__device__ __forceinline__ void update_row(const TableDev& t, int row, const float (&g)[KM]) {
  const int l = lane_id();
  const int w = t.width;
  float* prow = t.P + (size_t)row * w;
  float* arow = t.A ? t.A + (size_t)row * w : nullptr;
  float p[KM];
  float ss = 0.0f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    float pv = 0.0f;
    if (e < w) {
      pv = prow[e];
      if (t.opt == OPT_ADAGRAD) {
        const float av = arow[e] + g[k] * g[k];         // p2[idx] += g*g        param.py:147
        arow[e] = av;
        const float h = fmaxf(sqrtf(av), 1e-7f);         // H = max(sqrt(p2),1e-7) param.py:152
        pv = pv - (t.lr * g[k]) / h;                     // P -= lr*g/H           param.py:155
      } else {
        pv = pv - t.lr * g[k];                           // P -= lr*g             param.py:130
      }
    }
    p[k] = pv;
    ss += pv * pv;
  }
  if (t.post != POST_NONE) {
    ss = wave_sum(ss);
    if (t.post == POST_NORMALIZE) {
      const float nrm = sqrtf(ss);                       // param.py:165-166
#pragma unroll
      for (int k = 0; k < KM; ++k) p[k] = p[k] / nrm;
    } else {
      const float nrm = ss < 1.0f ? 1.0f : ss;           // param.py:171-173
#pragma unroll
      for (int k = 0; k < KM; ++k) p[k] = p[k] / nrm;
    }
  }
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    if (e < w) prow[e] = p[k];
  }
}

// g = (sum + rin*P) / div + rout*P; then reset the accumulator row
template <int KM>
__device__ __forceinline__ void mean_row(const TableDev& t, int row, int c, float (&g)[KM]) {
  const int l = lane_id();
  const int w = t.width;
  float* srow = t.acc.sum + (size_t)row * w;
  const float* prow = t.P + (size_t)row * w;
  const float div = t.fdiv > 0.0f ? t.fdiv : (float)c;
  const bool reg = t.rin != 0.0f || t.rout != 0.0f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    float gv = 0.0f;
    if (e < w) {
      const float s = srow[e];
      if (reg) {
        const float pv = prow[e];
        gv = (s + t.rin * pv) / div + t.rout * pv;
      } else {
        gv = s / div;
      }
      srow[e] = 0.0f;
    }
    g[k] = gv;
  }
  if (l == 0) t.acc.cnt[row] = 0;
}

// fused apply: one wavefront per touched slot of any of the tables
template <int KM>
__global__ __launch_bounds__(256) void k_apply(Tables4 ts) {
  const int wpb = blockDim.x >> 6;
  const int w0 = blockIdx.x * wpb + (threadIdx.x >> 6);
  const int nw = gridDim.x * wpb;
  int total = 0;
  for (int i = 0; i < ts.n; ++i) total += ts.nslots[i];
  for (int w = w0; w < total; w += nw) {
    int ti = 0, r = w;
    while (r >= ts.nslots[ti]) {
      r -= ts.nslots[ti];
      ++ti;
    }
    const TableDev& t = ts.t[ti];
    const int row = __builtin_amdgcn_readfirstlane(t.acc.touched[r]);
    if (row < 0) continue;
    const int c = __builtin_amdgcn_readfirstlane(t.acc.cnt[row]);
    if (c == 0) continue;   // stale slot (accumulator already consumed)
    float g[KM];
    mean_row<KM>(t, row, c, g);
    if (t.gate == nullptr || *t.gate != 0) update_row<KM>(t, row, g);
  }
}

// wide rows (RESCAL W): elementwise mean + update, no projection; the counts
// are cleared afterwards by k_zero_counts_slots
__global__ __launch_bounds__(256) void k_apply_wide(TableDev t, int nslots) {
  const int gate = t.gate ? *t.gate : 1;
  const long long w = t.width;
  const long long total = (long long)nslots * w;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const long long ti = idx / w;
    const long long e = idx - ti * w;
    const int row = t.acc.touched[ti];
    if (row < 0) continue;
    const int c = t.acc.cnt[row];
    if (c == 0) continue;
    const size_t off = (size_t)row * w + e;
    const float div = t.fdiv > 0.0f ? t.fdiv : (float)c;
    const float pv = t.P[off];
    const float g = (t.acc.sum[off] + t.rin * pv) / div + t.rout * pv;
    t.acc.sum[off] = 0.0f;
    if (gate) {
      if (t.opt == OPT_ADAGRAD) {
        const float av = t.A[off] + g * g;
        t.A[off] = av;
        t.P[off] = pv - (t.lr * g) / fmaxf(sqrtf(av), 1e-7f);
      } else {
        t.P[off] = pv - t.lr * g;
      }
    }
  }
}

__global__ void k_zero_counts_slots(int* __restrict__ cnt, const int* __restrict__ touched,
                                    int nslots) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += gridDim.x * blockDim.x) {
    const int row = touched[i];
    if (row >= 0) cnt[row] = 0;
  }
}

// explicit updater call: rows idx[i] with gradients g[i]
template <int KM>
__global__ __launch_bounds__(256) void k_update_rows(TableDev t, const float* __restrict__ g,
                                                     const int* __restrict__ idx, int U) {
  const int wpb = blockDim.x >> 6;
  const int l = lane_id();
  for (int i = blockIdx.x * wpb + (threadIdx.x >> 6); i < U; i += gridDim.x * wpb) {
    const int row = __builtin_amdgcn_readfirstlane(idx[i]);
    float gv[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int e = l + 64 * k;
      gv[k] = e < t.width ? g[(size_t)i * t.width + e] : 0.0f;
    }
    update_row<KM>(t, row, gv);
  }
}

__global__ __launch_bounds__(256) void k_update_rows_wide(TableDev t, const float* __restrict__ g,
                                                          const int* __restrict__ idx, int U) {
  const long long w = t.width;
  const long long total = (long long)U * w;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (long long)gridDim.x * blockDim.x) {
    const long long i = q / w;
    const long long e = q - i * w;
    const size_t off = (size_t)idx[i] * w + e;
    const float gv = g[q];
    if (t.opt == OPT_ADAGRAD) {
      const float av = t.A[off] + gv * gv;
      t.A[off] = av;
      t.P[off] = t.P[off] - (t.lr * gv) / fmaxf(sqrtf(av), 1e-7f);
    } else {
      t.P[off] = t.P[off] - t.lr * gv;
    }
  }
}

// ---- collect: sorted unique touched rows + mean rows (API path) ----
#define SKGE_CHUNK 4096  // rows per block: 256 threads x 16

__global__ __launch_bounds__(256) void k_count_nz(const int* __restrict__ cnt, int rows,
                                                  int* __restrict__ bsum) {
  __shared__ int s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  const int base = blockIdx.x * SKGE_CHUNK + threadIdx.x * 16;
  int c = 0;
  for (int q = 0; q < 16; ++q) {
    const int r = base + q;
    if (r < rows && cnt[r] != 0) ++c;
  }
  atomicAdd(&s, c);
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = s;
}

// inclusive scan of 256 values in LDS (Hillis-Steele)
__device__ __forceinline__ int block_scan_incl(int v, int* s) {
  const int t = threadIdx.x;
  s[t] = v;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const int x = t >= off ? s[t - off] : 0;
    __syncthreads();
    s[t] += x;
    __syncthreads();
  }
  return s[t];
}

__global__ __launch_bounds__(256) void k_scan_blocks(const int* __restrict__ bsum, int nb,
                                                     int* __restrict__ boff, int* __restrict__ U) {
  __shared__ int s[256];
  int carry = 0;
  for (int base = 0; base < nb; base += 256) {
    const int i = base + threadIdx.x;
    const int v = i < nb ? bsum[i] : 0;
    const int inc = block_scan_incl(v, s);
    if (i < nb) boff[i] = carry + inc - v;
    const int tot = s[255];
    __syncthreads();
    carry += tot;
  }
  if (threadIdx.x == 0) *U = carry;
}

__global__ __launch_bounds__(256) void k_compact(const int* __restrict__ cnt, int rows,
                                                 const int* __restrict__ boff,
                                                 int* __restrict__ idx_out) {
  __shared__ int s[256];
  const int base = blockIdx.x * SKGE_CHUNK + threadIdx.x * 16;
  int c = 0;
  for (int q = 0; q < 16; ++q) {
    const int r = base + q;
    if (r < rows && cnt[r] != 0) ++c;
  }
  const int inc = block_scan_incl(c, s);
  int pos = boff[blockIdx.x] + inc - c;
  for (int q = 0; q < 16; ++q) {
    const int r = base + q;
    if (r < rows && cnt[r] != 0) idx_out[pos++] = r;
  }
}

template <int KM>
__global__ __launch_bounds__(256) void k_gather_mean(TableDev t, const int* __restrict__ idx,
                                                     const int* __restrict__ Up,
                                                     float* __restrict__ g_out) {
  const int U = *Up;
  const int wpb = blockDim.x >> 6;
  const int l = lane_id();
  for (int i = blockIdx.x * wpb + (threadIdx.x >> 6); i < U; i += gridDim.x * wpb) {
    const int row = __builtin_amdgcn_readfirstlane(idx[i]);
    const int c = __builtin_amdgcn_readfirstlane(t.acc.cnt[row]);
    float g[KM];
    mean_row<KM>(t, row, c, g);
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int e = l + 64 * k;
      if (e < t.width) g_out[(size_t)i * t.width + e] = g[k];
    }
  }
}

__global__ __launch_bounds__(256) void k_gather_mean_wide(TableDev t, const int* __restrict__ idx,
                                                          const int* __restrict__ Up,
                                                          float* __restrict__ g_out) {
  const long long w = t.width;
  const long long total = (long long)(*Up) * w;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (long long)gridDim.x * blockDim.x) {
    const long long i = q / w;
    const long long e = q - i * w;
    const int row = idx[i];
    const size_t off = (size_t)row * w + e;
    const float div = t.fdiv > 0.0f ? t.fdiv : (float)t.acc.cnt[row];
    const float pv = t.P[off];
    g_out[q] = (t.acc.sum[off] + t.rin * pv) / div + t.rout * pv;
    t.acc.sum[off] = 0.0f;
  }
}

// zero the counts of the listed rows
__global__ void k_zero_counts(int* __restrict__ cnt, const int* __restrict__ idx,
                              const int* __restrict__ Up) {
  const int U = *Up;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < U; i += gridDim.x * blockDim.x)
    cnt[idx[i]] = 0;
}

// reset: zero every touched row's sum (counts by k_zero_counts_slots)
__global__ __launch_bounds__(256) void k_reset(TableDev t, int nslots) {
  const long long w = t.width;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < (long long)nslots * w;
       q += (long long)gridDim.x * blockDim.x) {
    const long long i = q / w;
    const int row = t.acc.touched[i];
    if (row >= 0) t.acc.sum[(size_t)row * w + (q - i * w)] = 0.0f;
  }
}

static int grid_for_waves(long long waves) {
  long long b = (waves + 3) / 4;
  if (b < 1) b = 1;
  if (b > 16384) b = 16384;
  return (int)b;
}

static int grid_for_elems(long long elems) {
  long long b = (elems + 255) / 256;
  if (b < 1) b = 1;
  if (b > 8192) b = 8192;
  return (int)b;
}

}  // namespace skge

using namespace skge;

extern "C" size_t skge_collect_workspace_bytes(int rows) {
  const size_t nb = ((size_t)rows + SKGE_CHUNK - 1) / SKGE_CHUNK;
  return 2 * nb * sizeof(int) + 64;
}

extern "C" int skge_accum_collect(void* stream, const skge_table_t* t, int* idx_out, float* g_out,
                                  int* U_out, void* workspace, size_t ws_bytes) {
  int rc = check_table(t, "table", true);
  if (rc) return rc;
  SKGE_CHECK_ARG(idx_out && g_out && U_out, "outputs NULL");
  SKGE_CHECK_ARG(workspace && ws_bytes >= skge_collect_workspace_bytes(t->rows),
                 "workspace too small");
  hipStream_t st = as_stream(stream);
  const int nb = (t->rows + SKGE_CHUNK - 1) / SKGE_CHUNK;
  int* bsum = (int*)workspace;
  int* boff = bsum + nb;
  TableDev td = table_dev(t);
  hipLaunchKernelGGL(k_count_nz, dim3(nb), dim3(256), 0, st, t->acc_cnt, t->rows, bsum);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(256), 0, st, bsum, nb, boff, U_out);
  hipLaunchKernelGGL(k_compact, dim3(nb), dim3(256), 0, st, t->acc_cnt, t->rows, boff, idx_out);
  const int km = km_for(t->width);
  const int gw = grid_for_waves(t->rows);
#define SKGE_GM(K) \
  case K: hipLaunchKernelGGL((k_gather_mean<K>), dim3(gw), dim3(256), 0, st, td, idx_out, U_out, g_out); break;
  switch (km) {
    SKGE_GM(1)
    SKGE_GM(2)
    SKGE_GM(3)
    SKGE_GM(4)
    SKGE_GM(8)
    SKGE_GM(16)
    default:
      hipLaunchKernelGGL(k_gather_mean_wide, dim3(grid_for_elems((long long)t->rows * t->width)),
                         dim3(256), 0, st, td, idx_out, U_out, g_out);
      hipLaunchKernelGGL(k_zero_counts, dim3(grid_for_elems(t->rows)), dim3(256), 0, st,
                         t->acc_cnt, idx_out, U_out);
  }
#undef SKGE_GM
  SKGE_CHECK_LAUNCH("collect");
  return SKGE_OK;
}

extern "C" int skge_accum_reset(void* stream, const skge_table_t* t, int nslots) {
  int rc = check_table(t, "table", true);
  if (rc) return rc;
  if ((rc = check_slots(t, nslots, "table"))) return rc;
  if (nslots == 0) return SKGE_OK;
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(k_reset, dim3(grid_for_elems((long long)nslots * t->width)), dim3(256), 0, st,
                     table_dev(t), nslots);
  hipLaunchKernelGGL(k_zero_counts_slots, dim3(grid_for_elems(nslots)), dim3(256), 0, st,
                     t->acc_cnt, t->acc_touched, nslots);
  SKGE_CHECK_LAUNCH("reset");
  return SKGE_OK;
}

extern "C" int skge_update_rows(void* stream, const skge_table_t* t, const float* g,
                                const int* idx, int U) {
  int rc = check_table(t, "table", false);
  if (rc) return rc;
  SKGE_CHECK_ARG(t->opt == SKGE_SGD || t->opt == SKGE_ADAGRAD, "unknown updater %d", t->opt);
  SKGE_CHECK_ARG(t->opt == SKGE_SGD || t->state, "AdaGrad needs state");
  SKGE_CHECK_ARG(t->post >= 0 && t->post <= 2, "unknown post %d", t->post);
  SKGE_CHECK_ARG(U >= 0, "U < 0");
  if (U == 0) return SKGE_OK;
  SKGE_CHECK_ARG(g && idx, "g/idx NULL");
  hipStream_t st = as_stream(stream);
  TableDev td = table_dev(t);
  const int km = km_for(t->width);
#define SKGE_UR(K) \
  case K: hipLaunchKernelGGL((k_update_rows<K>), dim3(grid_for_waves(U)), dim3(256), 0, st, td, g, idx, U); break;
  switch (km) {
    SKGE_UR(1)
    SKGE_UR(2)
    SKGE_UR(3)
    SKGE_UR(4)
    SKGE_UR(8)
    SKGE_UR(16)
    default:
      SKGE_CHECK_ARG(t->post == SKGE_POST_NONE, "projection needs width <= 1024");
      hipLaunchKernelGGL(k_update_rows_wide, dim3(grid_for_elems((long long)U * t->width)),
                         dim3(256), 0, st, td, g, idx, U);
  }
#undef SKGE_UR
  SKGE_CHECK_LAUNCH("update rows");
  return SKGE_OK;
}

extern "C" int skge_accum_apply(void* stream, const skge_table_t* tables, int ntables,
                                const int* nslots) {
  SKGE_CHECK_ARG(tables && nslots && ntables >= 1 && ntables <= 4, "1..4 tables");
  hipStream_t st = as_stream(stream);
  // narrow tables share one launch; each wide table gets its own
  Tables4 narrow = {};
  int km = 0;
  long long waves = 0;
  for (int i = 0; i < ntables; ++i) {
    const skge_table_t* t = tables + i;
    int rc = check_table(t, "table", true);
    if (rc) return rc;
    if ((rc = check_slots(t, nslots[i], "table"))) return rc;
    SKGE_CHECK_ARG(t->opt == SKGE_SGD || t->state, "AdaGrad needs state");
    SKGE_CHECK_ARG(t->post >= 0 && t->post <= 2, "unknown post %d", t->post);
    if (nslots[i] == 0) continue;
    const int k = km_for(t->width);
    if (k == 0) {
      SKGE_CHECK_ARG(t->post == SKGE_POST_NONE, "projection needs width <= 1024");
      hipLaunchKernelGGL(k_apply_wide, dim3(grid_for_elems((long long)nslots[i] * t->width)),
                         dim3(256), 0, st, table_dev(t), nslots[i]);
      hipLaunchKernelGGL(k_zero_counts_slots, dim3(grid_for_elems(nslots[i])), dim3(256), 0, st,
                         t->acc_cnt, t->acc_touched, nslots[i]);
    } else {
      narrow.t[narrow.n] = table_dev(t);
      narrow.nslots[narrow.n++] = nslots[i];
      if (k > km) km = k;
      waves += nslots[i];
    }
  }
  if (narrow.n) {
    const int gw = grid_for_waves(waves);
#define SKGE_AP(K) \
  case K: hipLaunchKernelGGL((k_apply<K>), dim3(gw), dim3(256), 0, st, narrow); break;
    switch (km) {
      SKGE_AP(1)
      SKGE_AP(2)
      SKGE_AP(3)
      SKGE_AP(4)
      SKGE_AP(8)
      SKGE_AP(16)
    }
#undef SKGE_AP
  }
  SKGE_CHECK_LAUNCH("apply");
  return SKGE_OK;
}

extern "C" int skge_pair_step(void* stream, int model, int af, const skge_table_t* ent,
                              const skge_table_t* rel, int d, const int* pos, const int* neg,
                              int P, float margin, float* coef_ws, int* nviol) {
  SKGE_CHECK_ARG(nviol, "nviol word required (it gates the update)");
  int rc = skge_pair_grad(stream, model, af, ent, rel, d, pos, neg, P, margin, nullptr, nullptr,
                          model == SKGE_RESCAL ? coef_ws : nullptr, nviol);
  if (rc) return rc;
  if (model == SKGE_RESCAL) {
    SKGE_CHECK_ARG(coef_ws, "RESCAL needs a coef workspace of 2P floats");
    rc = skge_rescal_wgrad(stream, ent, rel, d, pos, coef_ws, P, neg, coef_ws + P, P);
    if (rc) return rc;
  }
  skge_table_t t[2] = {*ent, *rel};
  t[0].gate = nviol;
  t[1].gate = nviol;
  const int ns[2] = {4 * P, model == SKGE_RESCAL ? rel->rows : 2 * P};
  return skge_accum_apply(stream, t, 2, ns);
}
