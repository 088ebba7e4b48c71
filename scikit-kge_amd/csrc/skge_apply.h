// The fp32 (and fixed-point) row apply and the RESCAL W step's element quad,
// shared by the apply kernels (skge_update.hip) and the one-launch RESCAL
// batch (skge_rescal.hip k_rescal_batch).  The error word is an argument:
// skge_update.hip passes its g_skge_dev_err, other translation units its
// device address (skge::device_error_word()).
#pragma once
#include "skge_host.h"

namespace skge {

struct TableDev {
  float* P;
  float* A;
  Accum acc;
  int rows, width, opt, post;
  float lr, rin, rout, fdiv;
  const int* gate;
  int* ucnt;   // optional AdaGrad update counter per row (skge/param.py:149-150)
};

inline TableDev table_dev(const skge_table_t* t) {
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

// FX64 sums wrap silently past +-2^63 (2^23 in gradient units, FX_SCALE):
// flag any decoded element at or past half of that range (bit 4; partial, see
// skge_update.hip)
__device__ __forceinline__ void fx_check_at(long long x, int* err) {
  constexpr long long HALF = 1ll << 62;
  if (x >= HALF || x <= -HALF) atomicOr(err, 4);
}

// Segment mean + updater + projection of one row, with every load of the row
// (sum, param, state) issued together right after the row id is known: one
// memory round trip instead of a chain (the sum is zeroed afterwards).
template <int KM>
__device__ __forceinline__ void apply_row_f(const TableDev& t, int row, bool upd, int* err) {
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
      if (l + 64 * k < w) fx_check_at(xrow[l + 64 * k], err);
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

// slot `slot` of an fp32 / fixed-point table (row -1: empty slot)
template <int K>
__device__ __forceinline__ void apply_slot_f(const TableDev& t, int slot, int* err) {
  const int row = t.acc.touched ? __builtin_amdgcn_readfirstlane(t.acc.touched[slot]) : slot;
  if (row < 0) return;
  apply_row_f<K>(t, row, t.gate == nullptr || *t.gate != 0, err);
}

// The RESCAL W step (WStep) for four consecutive elements of a 64 x 64 dW
// tile: the split partials summed in split order, then the W updater's step
// (skge/param.py:115-155; the arithmetic of k_rescal_wgrad_fin, bitwise).
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

// the W step made current by the apply side (in-front W step, WStep::cur):
// flip the buffer word when the batch updates, and count the relations'
// updates (updateCounts, skge/param.py:149-150).  One thread.
__device__ __forceinline__ void wstep_flip(const WStep& w) {
  if (*w.gate == 0) return;
  *w.cur ^= 1;
  if (w.opt == OPT_ADAGRAD && w.ucnt)
    for (int p = 0; p < w.M; ++p)
      if (w.rel_off[p + 1] > w.rel_off[p]) atomicAdd(w.ucnt + (p), 1);
}

}  // namespace skge
