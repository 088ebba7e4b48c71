// Segment mean + updater + projection kernels (skge/param.py:108-174,
// skge/util.py:53-101, StochasticTrainer._batch_step skge/base.py:1306-1316).
//
// Narrow rows (width <= 1024: E, R) are updated by one wavefront per row with
// the row in registers, so the projection's row norm is a wave reduction and
// the row is read and written exactly once.  Wide rows (RESCAL's W, width
// d*d, no projection) are updated elementwise.
#include <algorithm>

#include "skge_host.h"

namespace skge {

// error bits raised by apply kernels (read with skge_device_error):
// 2 = a packed int16x4 row's count exceeded 32767 (its sums may have wrapped)
// 4 = a deterministic fixed-point (ACC_FX64) sum wrapped (its 2^23 range in
//     gradient units; every add checks its own signed overflow, acc_row) or
//     decoded at or past half its range.  The range is sized so the largest
//     case measured (WN18 RESCAL at nb = 2) stays orders of magnitude inside
//     it (skge_device.h).
__device__ int g_skge_dev_err = 0;

int* dev_err_word() {   // the error word's device address (Accum::err)
  static int* p = nullptr;
  if (!p && hipGetSymbolAddress(reinterpret_cast<void**>(&p), HIP_SYMBOL(g_skge_dev_err)) != hipSuccess)
    p = nullptr;
  return p;
}

// FX64 sums wrap silently past +-2^63 (2^23 in gradient units, FX_SCALE):
// flag any decoded element at or past half of that range (partial: see above)
__device__ __forceinline__ void fx_check(long long x) {
  constexpr long long HALF = 1ll << 62;
  if (x >= HALF || x <= -HALF) atomicOr(&g_skge_dev_err, 4);
}

struct TableDev {
  float* P;
  float* A;
  Accum acc;
  int rows, width, opt, post;
  float lr, rin, rout, fdiv;
  const int* gate;
  int* ucnt;   // optional AdaGrad update counter per row (skge/param.py:149-150)
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
  d.ucnt = t->upd_count;
  return d;
}


// SGD._update / AdaGrad._update + post projection for one register-resident row
template <int KM>
__device__ __forceinline__ void update_row(const TableDev& t, int row, const float (&g)[KM]) {
  const int l = lane_id();
  const int w = t.width;
  float* prow = t.P + (size_t)row * w;
  float* arow = t.A ? t.A + (size_t)row * w : nullptr;
  const bool ada = t.opt == OPT_ADAGRAD;
  float p[KM], a[KM];
  if (ada && t.ucnt && l == 0) atomicAdd(t.ucnt + (row), 1);   // updateCounts[i] += 1  param.py:149-150
#pragma unroll
  for (int k = 0; k < KM; ++k) {   // unconditional loads (see load_row)
    const int e = l + 64 * k;
    const int ec = e < w ? e : w - 1;
    p[k] = prow[ec];
    a[k] = ada ? arow[ec] : 0.0f;
  }
  float ss = 0.0f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    float pv = p[k];
    if (ada) {
      a[k] = a[k] + g[k] * g[k];                       // p2[idx] += g*g        param.py:147
      const float h = fmaxf(sqrtf(a[k]), 1e-7f);       // H = max(sqrt(p2),1e-7) param.py:152
      pv = pv - (t.lr * g[k]) / h;                     // P -= lr*g/H           param.py:155
    } else {
      pv = pv - t.lr * g[k];                           // P -= lr*g             param.py:130
    }
    p[k] = e < w ? pv : 0.0f;
    ss += p[k] * p[k];
  }
  if (t.post != POST_NONE) {
    ss = wave_sum(ss);
    const float nrm = t.post == POST_NORMALIZE ? sqrtf(ss)              // param.py:165-166
                                               : (ss < 1.0f ? 1.0f : ss); // param.py:171-173
#pragma unroll
    for (int k = 0; k < KM; ++k) p[k] = p[k] / nrm;
  }
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    if (e < w) {
      prow[e] = p[k];
      if (ada) arow[e] = a[k];
    }
  }
}

// g = (sum + rin*P) / div + rout*P; then reset the accumulator row
template <int KM>
__device__ __forceinline__ void mean_row(const TableDev& t, int row, int c, float (&g)[KM]) {
  const int l = lane_id();
  const int w = t.width;
  const bool fx = t.acc.mode == ACC_FX64;
  float* srow = t.acc.sum + (size_t)row * w;
  long long* xrow = reinterpret_cast<long long*>(t.acc.sum) + (size_t)row * w;
  const float* prow = t.P + (size_t)row * w;
  const float div = t.fdiv > 0.0f ? t.fdiv : (float)c;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    const int ec = e < w ? e : w - 1;
    const float sv = fx ? fx_dec(xrow[ec]) : srow[ec], pv = prow[ec];
    if (fx) fx_check(xrow[ec]);
    g[k] = e < w ? (sv + t.rin * pv) / div + t.rout * pv : 0.0f;
  }
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    if (e < w) {
      if (fx)
        xrow[e] = 0;
      else
        srow[e] = 0.0f;
    }
  }
  if (l == 0) t.acc.cnt[row] = 0;
}

// Segment mean + updater + projection of one row, with every load of the row
// (sum, param, state) issued together right after the row id is known: one
// memory round trip instead of a chain (the sum is zeroed afterwards).
template <int KM>
__device__ __forceinline__ void apply_row(const TableDev& t, int row, bool upd) {
  const int l = lane_id();
  // claim the row: the first wave to swap its count out owns it (touched
  // slots may repeat a row); issued together with the row loads below
  int c = 0;
  if (l == 0) c = atomicExch(t.acc.cnt + row, 0);
  const int w = t.width;
  const bool fx = t.acc.mode == ACC_FX64;   // deterministic fixed-point sums
  float* __restrict__ srow = t.acc.sum + (size_t)row * w;
  long long* __restrict__ xrow = reinterpret_cast<long long*>(t.acc.sum) + (size_t)row * w;
  float* __restrict__ prow = t.P + (size_t)row * w;
  float* __restrict__ arow = t.A ? t.A + (size_t)row * w : nullptr;
  const bool ada = t.opt == OPT_ADAGRAD;
  float s[KM], p[KM], a[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    const bool in = e < w;
    const int ec = in ? e : w - 1;   // unconditional loads (see load_row)
    const float sv = fx ? fx_dec(xrow[ec]) : srow[ec], pv = prow[ec];
    const float av = ada ? arow[ec] : 0.0f;
    s[k] = in ? sv : 0.0f;
    p[k] = in ? pv : 0.0f;
    a[k] = in ? av : 0.0f;
  }
  c = __builtin_amdgcn_readfirstlane(c);
  if (c == 0) return;   // another wave owns the row, or a stale slot
  if (fx) {
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (l + 64 * k < w) fx_check(xrow[l + 64 * k]);
  }
  if (upd && ada && t.ucnt && l == 0) atomicAdd(t.ucnt + (row), 1);   // param.py:149-150
  const float div = t.fdiv > 0.0f ? t.fdiv : (float)c;
  float ss = 0.0f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const float g = (s[k] + t.rin * p[k]) / div + t.rout * p[k];   // segment mean (+ rparam)
    float pv = p[k];
    if (ada) {
      const float av = a[k] + g * g;                 // p2[idx] += g*g           param.py:147
      a[k] = av;
      pv = pv - (t.lr * g) / fmaxf(sqrtf(av), 1e-7f); // P -= lr*g/max(sqrt,1e-7) param.py:152-155
    } else {
      pv = pv - t.lr * g;                            // P -= lr*g                param.py:130
    }
    p[k] = pv;
    ss += pv * pv;
  }
  if (t.post != POST_NONE && upd) {
    ss = wave_sum(ss);
    const float nrm = t.post == POST_NORMALIZE ? sqrtf(ss) : (ss < 1.0f ? 1.0f : ss);
#pragma unroll
    for (int k = 0; k < KM; ++k) p[k] = p[k] / nrm;   // param.py:165-166 / 171-173
  }
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    if (e < w) {
      if (fx)
        xrow[e] = 0;
      else
        srow[e] = 0.0f;
      if (upd) {
        prow[e] = p[k];
        if (ada) arow[e] = a[k];
      }
    }
  }
}

// (the accumulator holds exact integer sums, four per qword)
// ACC_I16X4 form of apply_row, in two halves so one wave can keep several
// rows' claims and loads in flight (apply_slots_i16): i16_load claims row
// (lane 0 swaps its count out) and loads its packed sums, parameters and
// state in the same memory round trip; i16_finish applies the update if the
// claim was won.  Rows in the quad layout (see load_row4): one 16-byte load /
// store per lane per 1 KB of row.
template <int KQ>
__device__ __forceinline__ void i16_load(const TableDev& t, int row, int& c,
                                         unsigned long long (&sv)[KQ], float4 (&p)[KQ],
                                         float4 (&a)[KQ]) {
  const int l = lane_id();
  const int w = t.width, nq = w >> 2;
  c = 0;
  if (l == 0 && row >= 0) c = atomicExch(t.acc.cnt + row, 0);
  row = row >= 0 ? row : 0;   // a stale (-1) row still loads from a valid address
  unsigned long long* __restrict__ srow =
      reinterpret_cast<unsigned long long*>(t.acc.sum) + (size_t)row * nq;
  float4* __restrict__ prow = reinterpret_cast<float4*>(t.P + (size_t)row * w);
  float4* __restrict__ arow = t.A ? reinterpret_cast<float4*>(t.A + (size_t)row * w) : nullptr;
  const bool ada = t.opt == OPT_ADAGRAD;
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l, qc = q < nq ? q : nq - 1;
    sv[m] = srow[qc];
    p[m] = prow[qc];
    a[m] = ada ? arow[qc] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
}

template <int KQ>
__device__ __forceinline__ void i16_finish(const TableDev& t, int row, bool upd, int c,
                                           unsigned long long (&sv)[KQ], float4 (&p)[KQ],
                                           float4 (&a)[KQ]) {
  const int l = lane_id();
  const int w = t.width, nq = w >> 2;
  unsigned long long* __restrict__ srow =
      reinterpret_cast<unsigned long long*>(t.acc.sum) + (size_t)row * nq;
  float4* __restrict__ prow = reinterpret_cast<float4*>(t.P + (size_t)row * w);
  float4* __restrict__ arow = t.A ? reinterpret_cast<float4*>(t.A + (size_t)row * w) : nullptr;
  const bool ada = t.opt == OPT_ADAGRAD;
  c = __builtin_amdgcn_readfirstlane(c);
  if (c == 0) return;   // another wave owns the row, or a stale slot
  if (upd && ada && t.ucnt && l == 0) atomicAdd(t.ucnt + (row), 1);   // param.py:149-150
  // each occurrence adds a coefficient no larger than its count: c <= 32767
  // means no 16-bit field can have wrapped
  if (c > 32767 && l == 0) atomicOr(&g_skge_dev_err, 2);
  const float div = t.fdiv > 0.0f ? t.fdiv : (float)c;
  float ss = 0.0f;
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const bool in = 64 * m + l < nq;
    const float4 sm = unpack_i16x4(in ? sv[m] : 0ull);
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
  if (t.post != POST_NONE && upd) {
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
#pragma unroll
  for (int m = 0; m < KQ; ++m) {
    const int q = 64 * m + l;
    if (q < nq) {
      srow[q] = 0ull;
      if (upd) {
        prow[q] = p[m];
        if (ada) arow[q] = a[m];
      }
    }
  }
}


template <int KQ>
__device__ __forceinline__ void apply_row_i16(const TableDev& t, int row, bool upd) {
  int c;
  unsigned long long sv[KQ];
  float4 p[KQ], a[KQ];
  i16_load<KQ>(t, row, c, sv, p, a);
  i16_finish<KQ>(t, row, upd, c, sv, p, a);
}

// APPLY_SLOTS slot-recorded rows per wave, all their claims and loads in
// flight together; row -1 = empty slot.  Measured on config 5 (|E| = 50M,
// d = 512) in one run: one slot per wave is fastest -- the chip already has
// enough waves in flight, and a multi-row wave holds its slot for the
// slowest of its rows -- so the default is 1.
#ifndef SKGE_APPLY_SLOTS
#define SKGE_APPLY_SLOTS 1   // A/B on config 5 (same run): 1 slot 302 us, 2 slots 323, 4 slots 347
#endif
constexpr int APPLY_SLOTS = SKGE_APPLY_SLOTS;

template <int KQ>
__device__ __forceinline__ void apply_slots_i16(const TableDev& t, int s0, int n) {
  int r[APPLY_SLOTS];
  bool any = false;
#pragma unroll
  for (int k = 0; k < APPLY_SLOTS; ++k) {
    r[k] = s0 + k < n ? __builtin_amdgcn_readfirstlane(t.acc.touched[s0 + k]) : -1;
    any = any || r[k] >= 0;
  }
  if (!any) return;
  const bool upd = t.gate == nullptr || *t.gate != 0;
  int c[APPLY_SLOTS];
  unsigned long long v[APPLY_SLOTS][KQ];
  float4 p[APPLY_SLOTS][KQ], a[APPLY_SLOTS][KQ];
#pragma unroll
  for (int k = 0; k < APPLY_SLOTS; ++k) i16_load<KQ>(t, r[k], c[k], v[k], p[k], a[k]);
#pragma unroll
  for (int k = 0; k < APPLY_SLOTS; ++k)
    if (r[k] >= 0) i16_finish<KQ>(t, r[k], upd, c[k], v[k], p[k], a[k]);
}

// Dense table with replicated accumulators: one WORKGROUP per row.  Its 256
// threads spread over (copy, dword) pairs, fold the copies into LDS with
// integer adds (packed sums are linear) or float adds, and clear them; wave 0
// then updates the row.  Few registers, so the entity waves sharing the launch
// keep their occupancy.
template <int MODE, int KR>
__device__ __forceinline__ void apply_row_rep_block(const TableDev& t, int row, bool upd,
                                                    int* lds) {
  const int tid = threadIdx.x, R = t.acc.replicas, rows = t.rows, w = t.width;
  const int dw = acc_row_dwords(MODE, w);             // accumulator dwords per row
  // fold the copies: each thread owns one accumulator word (or the count) and
  // loads it from every copy with the loads in flight together, summing in
  // copy order (fixed order: deterministic), then clears the copies
  if (tid < 64) {   // counts: lane k holds copy k (R <= 32), one wave sum
    int v = 0;
    int* cp = t.acc.cnt + (size_t)tid * rows + row;
    if (tid < R) v = *cp;
    if (v) *cp = 0;
    // each copy's 16-bit fields are exact while that copy's count is <= 32767
    // (producers spread over copies by position, so a copy sees at most
    // ceil(batch / R) of a hot row's occurrences)
    if (MODE == ACC_I16X4 && v > 32767) atomicOr(&g_skge_dev_err, 2);
    v = wave_sum_int(v);
    if (tid == 0) lds[w] = v;
  }
  if (MODE == ACC_I16X4) {   // every copy decoded on its own, summed as int32 per element
    const int nq = w >> 2;
    for (int q = tid; q < nq; q += blockDim.x) {
      unsigned long long* sp = reinterpret_cast<unsigned long long*>(t.acc.sum) + (size_t)row * nq + q;
      const size_t stride = (size_t)rows * nq;
      unsigned long long v[32];
#pragma unroll
      for (int k = 0; k < 32; ++k) v[k] = k < R ? sp[k * stride] : 0ull;
      int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        const float4 f = unpack_i16x4(v[k]);
        s0 += (int)f.x;
        s1 += (int)f.y;
        s2 += (int)f.z;
        s3 += (int)f.w;
        if (k < R && v[k]) sp[k * stride] = 0ull;
      }
      lds[4 * q] = s0;
      lds[4 * q + 1] = s1;
      lds[4 * q + 2] = s2;
      lds[4 * q + 3] = s3;
    }
  } else {
    for (int q = tid; q < dw; q += blockDim.x) {
      float* sp = t.acc.sum + (size_t)row * dw + q;
      const size_t stride = (size_t)rows * dw;
      float v[32];
#pragma unroll
      for (int k = 0; k < 32; ++k) v[k] = k < R ? sp[k * stride] : 0.0f;
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        acc += v[k];
        if (k < R && v[k] != 0.0f) sp[k * stride] = 0.0f;
      }
      reinterpret_cast<float*>(lds)[q] = acc;
    }
  }
  __syncthreads();
  const int c = lds[w];
  if (tid < 64 && c != 0) {
    const int l = tid;
    const bool ada = t.opt == OPT_ADAGRAD;
    const float div = t.fdiv > 0.0f ? t.fdiv : (float)c;
    float ss = 0.0f;
    // element e = l + 64k, KR = ceil(width / 64) per lane
    float p[KR], a[KR];
    float* prow = t.P + (size_t)row * w;
    float* arow = t.A ? t.A + (size_t)row * w : nullptr;
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int e = l + 64 * k;
      p[k] = 0.0f;
      a[k] = 0.0f;
      {
        const int ec = e < w ? e : w - 1;
        float sv;
        if (MODE == ACC_I16X4) {
          sv = (float)lds[ec];
        } else {
          sv = __int_as_float(lds[ec]);
        }
        const float pv = prow[ec];
        const float av = ada ? arow[ec] : 0.0f;
        const float g = (sv + t.rin * pv) / div + t.rout * pv;
        float np = pv, na = av;
        if (ada) {
          na = av + g * g;
          // packed (exact integer) sums: the fast step of every packed apply
          np = MODE == ACC_I16X4 ? pv - adagrad_step_fast(t.lr, g, na)
                                 : pv - (t.lr * g) / fmaxf(sqrtf(na), 1e-7f);
        } else {
          np = pv - t.lr * g;
        }
        p[k] = e < w ? np : 0.0f;
        a[k] = na;
        ss += p[k] * p[k];
      }
    }
    if (t.post != POST_NONE && upd) {
      ss = wave_sum(ss);
      if (MODE == ACC_I16X4) {
        const float inv = proj_scale_fast(t.post, ss);
#pragma unroll
        for (int k = 0; k < KR; ++k) p[k] = p[k] * inv;
      } else {
        const float nrm = t.post == POST_NORMALIZE ? sqrtf(ss) : (ss < 1.0f ? 1.0f : ss);
#pragma unroll
        for (int k = 0; k < KR; ++k) p[k] = p[k] / nrm;
      }
    }
    if (upd && ada && t.ucnt && l == 0) atomicAdd(t.ucnt + (row), 1);   // param.py:149-150
    if (upd) {
#pragma unroll
      for (int k = 0; k < KR; ++k) {
        const int e = l + 64 * k;
        if (e < w) {
          prow[e] = p[k];
          if (ada) arow[e] = a[k];
        }
      }
    }
  }
  __syncthreads();   // lds is reused by the next row
}

template <int K, int MODE>
__device__ __forceinline__ void apply_slot(const TableDev& t, int slot) {
  const int row = t.acc.touched ? __builtin_amdgcn_readfirstlane(t.acc.touched[slot]) : slot;
  if (row < 0) return;
  const bool upd = t.gate == nullptr || *t.gate != 0;
  if (MODE == ACC_I16X4)
    apply_row_i16<K>(t, row, upd);
  else
    apply_row<K>(t, row, upd);
}

// fused apply: one wavefront per slot of table 0 (slots [0, n0)) or table 1
// (slots [n0, n0 + n1)); a dense table (no slot records) has one slot per
// row.  If table 1 is dense with replicated accumulators, its rows are handled
// by the workgroups past nblk0 instead (one workgroup per row).  Two explicit
// table arguments keep every table field in scalar registers.
template <int K, int MODE, int KR>
__global__ __launch_bounds__(256) void k_apply(TableDev t0, int n0, TableDev t1, int n1,
                                               int nblk0) {
  __shared__ int lds[1025];
  int blk = (int)blockIdx.x;
  if (t1.acc.replicas > 1) {
    // the replicated rows' workgroups come FIRST in dispatch order: each runs
    // a fold -> update chain, so as the grid's tail they set its length
    const int nrep = (int)gridDim.x - nblk0;
    if (blk < nrep) {
      for (int r = blk; r < n1; r += nrep)
        apply_row_rep_block<MODE, KR>(t1, r, t1.gate == nullptr || *t1.gate != 0, lds);
      return;
    }
    blk -= nrep;
    n1 = 0;   // table 1 is not a wave-per-slot table
  }
  const int wpb = blockDim.x >> 6;
  const int nw = (t1.acc.replicas > 1 ? nblk0 : gridDim.x) * wpb;
  // a slot-recorded packed table 0 is applied APPLY_SLOTS slots per wave
  const bool two = MODE == ACC_I16X4 && t0.acc.touched != nullptr;
  const int w0 = two ? (n0 + APPLY_SLOTS - 1) / APPLY_SLOTS : n0;
  for (int w = blk * wpb + (threadIdx.x >> 6); w < w0 + n1; w += nw) {
    if (w >= w0)
      apply_slot<K, MODE>(t1, w - w0);
    else if (two)
      apply_slots_i16<K>(t0, APPLY_SLOTS * w, n0);
    else
      apply_slot<K, MODE>(t0, w);
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
      if (e == 0 && t.opt == OPT_ADAGRAD && t.ucnt) atomicAdd(t.ucnt + (row), 1);   // param.py:149-150
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
      const float x = g[(size_t)i * t.width + (e < t.width ? e : t.width - 1)];
      gv[k] = e < t.width ? x : 0.0f;
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
    if (e == 0 && t.opt == OPT_ADAGRAD && t.ucnt) atomicAdd(t.ucnt + (idx[i]), 1);   // param.py:149-150
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
// fold the copies of a replicated fp32 accumulator into copy 0 (collect path)
__global__ __launch_bounds__(256) void k_fold_replicas(float* __restrict__ sum,
                                                       int* __restrict__ cnt, int reps, int rows,
                                                       int width) {
  const long long n = (long long)rows * width;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (long long)gridDim.x * blockDim.x) {
    float v = sum[e];
    for (int k = 1; k < reps; ++k) {
      float* q = sum + (size_t)k * n + e;
      v += *q;
      *q = 0.0f;
    }
    sum[e] = v;
    if (e < rows) {
      int c = cnt[e];
      for (int k = 1; k < reps; ++k) {
        int* q = cnt + (size_t)k * rows + e;
        c += *q;
        *q = 0;
      }
      cnt[e] = c;
    }
  }
}

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

// The RESCAL W step (WStep, after k_rescal_front_fused) beside the entity
// apply, one launch: the first nwb workgroups take four consecutive elements
// of a 64 x 64 dW tile per thread -- the split partials summed in split order,
// then the W updater's step (skge/param.py:115-155; the arithmetic of
// k_rescal_wgrad_fin, bitwise) -- the rest apply the entity slots as k_apply.
constexpr int WS_T = 64;   // dW tile edge (skge_rescal.hip WG_T)
__device__ __forceinline__ void wstep_quad(const WStep& w, long long q) {
  const int nt = (w.d + WS_T - 1) / WS_T;
  const long long per_rel = (long long)nt * nt * (WS_T * WS_T / 4);
  const int p = (int)(q / per_rel);
  const int rem = (int)(q - (long long)p * per_rel);
  const int tile = rem / (WS_T * WS_T / 4), e = 4 * (rem - tile * (WS_T * WS_T / 4));
  const int off = w.rel_off[p], cnt = w.rel_off[p + 1] - off;
  const int gv = *w.gate;
  if (cnt == 0 || gv == 0) return;   // relation not in the batch / the model returned None
  const int rt = tile / nt, ct = tile - rt * nt;
  const int r = rt * WS_T + e / WS_T, c = ct * WS_T + e % WS_T;
  if (r >= w.d || c >= w.d) return;
  if (tile == 0 && e == 0 && w.opt == OPT_ADAGRAD && w.ucnt) atomicAdd(w.ucnt + (p), 1);   // param.py:149-150
  // split-K groups of 128 of the relation's dW items (skge_rescal.hip
  // WS_GROUP): splits past its groups wrote nothing
  const int nit = w.dwcnt ? w.dwcnt[p] : cnt;
  const int ngr = (nit + 127) / 128, nsp = min(w.splits, ngr);
  const float* part = w.part + ((size_t)(p * nt * nt + tile) * w.splits) * (WS_T * WS_T) + e;
  float4 s = *reinterpret_cast<const float4*>(part);
  const size_t o = (size_t)p * w.d * w.d + (size_t)r * w.d + c;
  const bool ada = w.opt == OPT_ADAGRAD;
  float pv[4], av[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const bool in = c + m < w.d;
    pv[m] = in ? w.W[o + m] : 0.0f;
    av[m] = in && ada ? w.A[o + m] : 0.0f;
  }
  for (int k = 1; k < nsp; ++k) {   // split order: deterministic sums
    const float4 v = *reinterpret_cast<const float4*>(part + (size_t)k * (WS_T * WS_T));
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  const float sv[4] = {s.x, s.y, s.z, s.w};
  const float div = w.fdiv > 0.0f ? w.fdiv : (float)cnt;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    if (c + m >= w.d) continue;
    const float g = (sv[m] + w.rin * pv[m]) / div + w.rout * pv[m];
    if (ada) {
      const float a2 = av[m] + g * g;
      w.W[o + m] = pv[m] - (w.lr * g) / fmaxf(sqrtf(a2), 1e-7f);
      w.A[o + m] = a2;
    } else {
      w.W[o + m] = pv[m] - w.lr * g;
    }
  }
}

template <int K>
__global__ __launch_bounds__(256) void k_apply_wstep(TableDev t0, int n0, WStep w, int nwb) {
  if (w.cur) {   // the W step was done in the front: make it current if the batch updates
    if ((int)blockIdx.x < nwb) {
      if (blockIdx.x == 0 && threadIdx.x < 64 && *w.gate != 0) {   // wave 0
        if (threadIdx.x == 0) *w.cur ^= 1;
        if (w.opt == OPT_ADAGRAD && w.ucnt)   // updateCounts, skge/param.py:149-150: lane p
          for (int p = threadIdx.x; p < w.M; p += 64)
            if (w.rel_off[p + 1] > w.rel_off[p]) atomicAdd(w.ucnt + (p), 1);
      }
      return;
    }
  } else if ((int)blockIdx.x < nwb) {
    const long long nq = (long long)w.M * ((w.d + WS_T - 1) / WS_T) * ((w.d + WS_T - 1) / WS_T) *
                         (WS_T * WS_T / 4);
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < nq;
         q += (long long)nwb * blockDim.x)
      wstep_quad(w, q);
    return;
  }
  const int wpb = blockDim.x >> 6;
  const int nw = ((int)gridDim.x - nwb) * wpb;
  for (int s = ((int)blockIdx.x - nwb) * wpb + (threadIdx.x >> 6); s < n0; s += nw)
    apply_slot<K, ACC_F32>(t0, s);
}

int apply_with_wstep(hipStream_t st, const skge_table_t* ent, int nslots, const WStep& w) {
  int rc = check_table(ent, "ent", true);
  if (rc) return rc;
  if ((rc = check_slots(ent, nslots, "ent"))) return rc;
  SKGE_CHECK_ARG((ent->acc_mode == SKGE_ACC_F32 || ent->acc_mode == SKGE_ACC_FX64) &&
                     ent->acc_replicas <= 1,
                 "W step beside the apply: single fp32 (or fixed-point) entity accumulator");
  SKGE_CHECK_ARG(ent->opt == SKGE_SGD || ent->state, "AdaGrad needs state");
  SKGE_CHECK_ARG(w.opt == SKGE_SGD || w.A, "AdaGrad needs state");
  const int nt = (w.d + WS_T - 1) / WS_T;
  const long long nq = (long long)w.M * nt * nt * (WS_T * WS_T / 4);
  const int nwb = w.cur ? 1 : grid_for_elems(nq);
  const int grid = nwb + grid_for_waves(nslots);
  const TableDev td = table_dev(ent);
  switch (km_for(ent->width)) {
    case 1: hipLaunchKernelGGL((k_apply_wstep<1>), dim3(grid), dim3(256), 0, st, td, nslots, w, nwb); break;
    case 2: hipLaunchKernelGGL((k_apply_wstep<2>), dim3(grid), dim3(256), 0, st, td, nslots, w, nwb); break;
    case 3: hipLaunchKernelGGL((k_apply_wstep<3>), dim3(grid), dim3(256), 0, st, td, nslots, w, nwb); break;
    case 4: hipLaunchKernelGGL((k_apply_wstep<4>), dim3(grid), dim3(256), 0, st, td, nslots, w, nwb); break;
    case 8: hipLaunchKernelGGL((k_apply_wstep<8>), dim3(grid), dim3(256), 0, st, td, nslots, w, nwb); break;
    case 16: hipLaunchKernelGGL((k_apply_wstep<16>), dim3(grid), dim3(256), 0, st, td, nslots, w, nwb); break;
    default: set_error("entity width %d unsupported", ent->width); return SKGE_ENOTSUP;
  }
  SKGE_CHECK_LAUNCH("apply + W step");
  return SKGE_OK;
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
  if ((rc = check_f32(t, "table"))) return rc;
  SKGE_CHECK_ARG(workspace && ws_bytes >= skge_collect_workspace_bytes(t->rows),
                 "workspace too small");
  hipStream_t st = as_stream(stream);
  const int nb = (t->rows + SKGE_CHUNK - 1) / SKGE_CHUNK;
  int* bsum = (int*)workspace;
  int* boff = bsum + nb;
  TableDev td = table_dev(t);
  if (t->acc_replicas > 1) {   // one copy first (the fold order is fixed: copy 0, 1, ...)
    hipLaunchKernelGGL(k_fold_replicas, dim3(grid_for_elems((long long)t->rows * t->width)),
                       dim3(256), 0, st, t->acc_sum, t->acc_cnt, t->acc_replicas, t->rows,
                       t->width);
    td.acc.replicas = 1;
  }
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
  hipStream_t st = as_stream(stream);
  const size_t row_bytes = (size_t)acc_row_dwords(t->acc_mode, t->width) * 4;
  if (t->acc_touched == nullptr) {   // dense table: clear everything (every copy)
    const size_t reps = t->acc_replicas > 1 ? (size_t)t->acc_replicas : 1;
    SKGE_CHECK_HIP(hipMemsetAsync(t->acc_sum, 0, reps * row_bytes * t->rows, st));
    SKGE_CHECK_HIP(hipMemsetAsync(t->acc_cnt, 0, reps * sizeof(int) * t->rows, st));
    return SKGE_OK;
  }
  if (nslots == 0) return SKGE_OK;
  TableDev td = table_dev(t);
  td.width = (int)(row_bytes / 4);   // zero dwords, whatever their encoding
  hipLaunchKernelGGL(k_reset, dim3(grid_for_elems((long long)nslots * td.width)), dim3(256), 0, st,
                     td, nslots);
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
  // narrow tables are applied two per launch (same accumulator mode); each
  // wide table gets its own launch
  auto kdim = [&](int i) {
    return tables[i].acc_mode == SKGE_ACC_I16X4 ? (tables[i].width / 4 + 63) / 64
                                                : km_for(tables[i].width);
  };
  auto slots_of = [&](int i) {
    return tables[i].acc_touched ? nslots[i] : tables[i].rows;   // dense: one slot per row
  };
  auto reps = [&](int i) { return tables[i].acc_replicas > 1 ? tables[i].acc_replicas : 1; };
  auto launch_pair = [&](int i, int j) -> int {
    if (j >= 0 && reps(i) > 1) std::swap(i, j);   // a replicated table goes second
    if (j < 0 && reps(i) > 1) {                   // a replicated table alone
      j = i;
      i = -1;
    }
    int k = i >= 0 ? kdim(i) : 1;
    if (j >= 0 && reps(j) == 1) k = std::max(k, kdim(j));
    const int mode = tables[i >= 0 ? i : j].acc_mode;
    const int na = i >= 0 ? slots_of(i) : 0;
    const int nb = j >= 0 ? slots_of(j) : 0;
    // waves of table i: APPLY_SLOTS slots per wave for a slot-recorded packed table
    const int wa = (i >= 0 && tables[i].acc_mode == SKGE_ACC_I16X4 && tables[i].acc_touched)
                       ? (na + APPLY_SLOTS - 1) / APPLY_SLOTS : na;
    int nblk0, grid;
    if (j >= 0 && reps(j) > 1) {
      nblk0 = std::max(1, std::min((wa + 3) / 4, 16384));
      grid = nblk0 + std::min(nb, 4096);
    } else {
      nblk0 = grid = grid_for_waves((long long)wa + nb);
    }
    TableDev b = j >= 0 ? table_dev(tables + j) : table_dev(tables + i);
    TableDev a = i >= 0 ? table_dev(tables + i) : b;
    if (i < 0) a.acc.replicas = 1;   // placeholder table 0 with no slots
    if (j < 0) b.acc.replicas = 1;
    const int kr = (j >= 0 && reps(j) > 1) ? km_for(tables[j].width) : 1;
#define SKGE_AP3(K, M, KR) \
  hipLaunchKernelGGL((k_apply<K, M, KR>), dim3(grid), dim3(256), 0, st, a, na, b, nb, nblk0)
#define SKGE_AP(K, M)                             \
  do {                                            \
    if (kr <= 1) SKGE_AP3(K, M, 1);               \
    else if (kr <= 2) SKGE_AP3(K, M, 2);          \
    else if (kr <= 4) SKGE_AP3(K, M, 4);          \
    else if (kr <= 8) SKGE_AP3(K, M, 8);          \
    else SKGE_AP3(K, M, 16);                      \
  } while (0)
    if (mode == SKGE_ACC_I16X4) {
      if (k <= 1) SKGE_AP(1, ACC_I16X4);
      else if (k <= 2) SKGE_AP(2, ACC_I16X4);
      else SKGE_AP(4, ACC_I16X4);
    } else {
      switch (k) {
        case 1: SKGE_AP(1, ACC_F32); break;
        case 2: SKGE_AP(2, ACC_F32); break;
        case 3: SKGE_AP(3, ACC_F32); break;
        case 4: SKGE_AP(4, ACC_F32); break;
        case 8: SKGE_AP(8, ACC_F32); break;
        default: SKGE_AP(16, ACC_F32); break;
      }
    }
#undef SKGE_AP3
#undef SKGE_AP
    return SKGE_OK;
  };
  int pend = -1;   // narrow table waiting for a partner
  for (int i = 0; i < ntables; ++i) {
    const skge_table_t* t = tables + i;
    int rc = check_table(t, "table", true);
    if (rc) return rc;
    if ((rc = check_slots(t, nslots[i], "table"))) return rc;
    SKGE_CHECK_ARG(t->opt == SKGE_SGD || t->state, "AdaGrad needs state");
    SKGE_CHECK_ARG(t->post >= 0 && t->post <= 2, "unknown post %d", t->post);
    if (slots_of(i) == 0) continue;
    if (km_for(t->width) == 0) {
      SKGE_CHECK_ARG(t->post == SKGE_POST_NONE, "projection needs width <= 1024");
      SKGE_CHECK_ARG(t->acc_touched != nullptr, "wide tables need slot records");
      hipLaunchKernelGGL(k_apply_wide, dim3(grid_for_elems((long long)nslots[i] * t->width)),
                         dim3(256), 0, st, table_dev(t), nslots[i]);
      hipLaunchKernelGGL(k_zero_counts_slots, dim3(grid_for_elems(nslots[i])), dim3(256), 0, st,
                         t->acc_cnt, t->acc_touched, nslots[i]);
    } else if (pend < 0) {
      pend = i;
    } else if (tables[pend].acc_mode == t->acc_mode) {
      launch_pair(pend, i);
      pend = -1;
    } else {
      launch_pair(pend, -1);
      pend = i;
    }
  }
  if (pend >= 0) launch_pair(pend, -1);
  SKGE_CHECK_LAUNCH("apply");
  return SKGE_OK;
}

// RESCAL on the matrix cores (skge_rescal.hip)
size_t skge_rescal_mfma_ws_bytes(int n, int M, int d);
int skge_rescal_triple_grad_mfma(hipStream_t st, const skge_table_t* ent,
                                 const skge_table_t* rel, int d, const int* trip,
                                 const float* ys, int T, void* workspace, size_t ws_bytes,
                                 float* score, float* loss, bool apply_w);
bool skge_rescal_mfma_ok(int d, int M);
int skge_rescal_pair_grad_mfma(hipStream_t st, int af, const skge_table_t* ent,
                               const skge_table_t* rel, int d, const int* pos, const int* neg,
                               int P, float margin, void* workspace, size_t ws_bytes,
                               float* pscore, float* nscore, int* nviol, bool apply_w);

// the MFMA path wherever it applies (d <= 1024, M within the scan's LDS)
static bool rescal_use_mfma(int d, int M) { return skge_rescal_mfma_ok(d, M); }
bool rescal_pair_mfma_selected(int d, int M) { return rescal_use_mfma(d, M); }

extern "C" int skge_device_error(void* stream, int reset) {
  int v = 0;
  hipStream_t st = as_stream(stream);
  SKGE_CHECK_HIP(hipStreamSynchronize(st));
  SKGE_CHECK_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_skge_dev_err), sizeof(int)));
  if (reset && v) {
    const int z = 0;
    SKGE_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_skge_dev_err), &z, sizeof(int)));
  }
  return v;
}

extern "C" size_t skge_pair_step_workspace_bytes(int model, int P, int M, int d) {
  if (model != SKGE_RESCAL || P <= 0) return 0;
  const size_t coef = (size_t)2 * P * sizeof(float);   // coef of every pair (VALU path)
  if (skge_rescal_mfma_ok(d, M)) return std::max(coef, skge_rescal_mfma_ws_bytes(2 * P, M, d));
  return coef;
}

extern "C" int skge_pair_step(void* stream, int model, int af, const skge_table_t* ent,
                              const skge_table_t* rel, int d, const int* pos, const int* neg,
                              int P, float margin, void* workspace, size_t ws_bytes, int* nviol) {
  SKGE_CHECK_ARG(nviol, "nviol word required (it gates the update)");
  int rc;
  if (model == SKGE_RESCAL && P > 0) {
    const size_t need = skge_pair_step_workspace_bytes(model, P, rel->rows, d);
    SKGE_CHECK_ARG(workspace && ws_bytes >= need, "RESCAL needs a %zu-byte workspace", need);
    if (rescal_use_mfma(d, rel->rows)) {
      if ((rc = check_table(ent, "ent", true)) || (rc = check_table(rel, "rel", false)) ||
          (rc = check_f32(ent, "ent")) || (rc = check_f32(rel, "rel")) ||
          (rc = check_single(ent, "ent")) || (rc = check_single(rel, "rel")))
        return rc;
      SKGE_CHECK_ARG(ent->width == d && rel->width == d * d, "RESCAL table widths");
      SKGE_CHECK_ARG(af >= 0 && af <= 3, "unknown activation %d", af);
      if ((rc = check_slots(ent, 4ll * P, "ent")) || (rc = check_slots(rel, rel->rows, "W")))
        return rc;
      SKGE_CHECK_ARG(rel->opt == SKGE_SGD || rel->state, "AdaGrad needs state");
      // W is updated inside the dW kernel (its owner workgroup per tile):
      // only the entity table is left for skge_accum_apply
      rc = skge_rescal_pair_grad_mfma(as_stream(stream), af, ent, rel, d, pos, neg, P, margin,
                                      workspace, ws_bytes, nullptr, nullptr, nviol, true);
      if (rc) return rc;
      skge_table_t te = *ent;
      te.gate = nviol;
      const int ns = 4 * P;
      return skge_accum_apply(stream, &te, 1, &ns);
    } else {
      float* coef = (float*)workspace;
      rc = skge_pair_grad(stream, model, af, ent, rel, d, pos, neg, P, margin, nullptr, nullptr,
                          coef, nviol);
      if (!rc) rc = skge_rescal_wgrad(stream, ent, rel, d, pos, coef, P, neg, coef + P, P);
    }
  } else {
    rc = skge_pair_grad(stream, model, af, ent, rel, d, pos, neg, P, margin, nullptr, nullptr,
                        nullptr, nviol);
  }
  if (rc) return rc;
  skge_table_t t[2] = {*ent, *rel};
  t[0].gate = nviol;
  t[1].gate = nviol;
  const int ns[2] = {4 * P, model == SKGE_RESCAL ? rel->rows : 2 * P};
  return skge_accum_apply(stream, t, 2, ns);
}

extern "C" size_t skge_triple_step_workspace_bytes(int model, int T, int M, int d) {
  if (model != SKGE_RESCAL || T <= 0) return 0;
  const size_t coef = (size_t)T * sizeof(float);   // fs of every triple (VALU path)
  if (skge_rescal_mfma_ok(d, M)) return std::max(coef, skge_rescal_mfma_ws_bytes(T, M, d));
  return coef;
}

extern "C" int skge_triple_step(void* stream, int model, const skge_table_t* ent,
                                const skge_table_t* rel, int d, const int* trip, const float* ys,
                                int T, void* workspace, size_t ws_bytes, float* loss) {
  int rc;
  if (model == SKGE_RESCAL && T > 0) {
    const size_t need = skge_triple_step_workspace_bytes(model, T, rel->rows, d);
    SKGE_CHECK_ARG(workspace && ws_bytes >= need, "RESCAL needs a %zu-byte workspace", need);
    SKGE_CHECK_ARG(trip && ys, "trip/ys NULL");
    if (rescal_use_mfma(d, rel->rows)) {
      if ((rc = check_table(ent, "ent", true)) || (rc = check_table(rel, "rel", false)) ||
          (rc = check_f32(ent, "ent")) || (rc = check_f32(rel, "rel")) ||
          (rc = check_single(ent, "ent")) || (rc = check_single(rel, "rel")))
        return rc;
      SKGE_CHECK_ARG(ent->width == d && rel->width == d * d, "RESCAL table widths");
      if ((rc = check_slots(ent, 2ll * T, "ent")) || (rc = check_slots(rel, rel->rows, "W")))
        return rc;
      SKGE_CHECK_ARG(rel->opt == SKGE_SGD || rel->state, "AdaGrad needs state");
      rc = skge_rescal_triple_grad_mfma(as_stream(stream), ent, rel, d, trip, ys, T, workspace,
                                        ws_bytes, nullptr, loss, true);   // W updated in place
      if (rc) return rc;
      const int ns = 2 * T;
      return skge_accum_apply(stream, ent, 1, &ns);
    } else {
      float* coef = (float*)workspace;
      rc = skge_triple_grad(stream, model, ent, rel, d, trip, ys, T, nullptr, coef, loss);
      if (!rc) rc = skge_rescal_wgrad(stream, ent, rel, d, trip, coef, T, nullptr, nullptr, 0);
    }
  } else {
    rc = skge_triple_grad(stream, model, ent, rel, d, trip, ys, T, nullptr, nullptr, loss);
  }
  if (rc) return rc;
  skge_table_t t[2] = {*ent, *rel};
  const int ns[2] = {2 * T, model == SKGE_RESCAL ? rel->rows : T};
  return skge_accum_apply(stream, t, 2, ns);
}
