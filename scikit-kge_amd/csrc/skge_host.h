// Host-side helpers for the C ABI: error reporting and argument checks.
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../include/skge_hip.h"
#include "skge_device.h"

namespace skge {

void set_error(const char* fmt, ...);

#define SKGE_CHECK_ARG(cond, ...)            \
  do {                                       \
    if (!(cond)) {                           \
      ::skge::set_error(__VA_ARGS__);        \
      return SKGE_EINVAL;                    \
    }                                        \
  } while (0)

#define SKGE_CHECK_LAUNCH(what)                                                   \
  do {                                                                            \
    hipError_t _e = hipGetLastError();                                            \
    if (_e != hipSuccess) {                                                       \
      ::skge::set_error("%s: %s", what, hipGetErrorString(_e));                   \
      return SKGE_EHIP;                                                           \
    }                                                                             \
  } while (0)

#define SKGE_CHECK_HIP(call)                                                      \
  do {                                                                            \
    hipError_t _e = (call);                                                       \
    if (_e != hipSuccess) {                                                       \
      ::skge::set_error("%s: %s", #call, hipGetErrorString(_e));                  \
      return SKGE_EHIP;                                                           \
    }                                                                             \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// registers per lane needed to hold a row of width d in the lane-strided
// layout (see skge_device.h); 0 = unsupported
inline int km_for(int d) {
  if (d <= 64) return 1;
  if (d <= 128) return 2;
  if (d <= 192) return 3;
  if (d <= 256) return 4;
  if (d <= 512) return 8;
  if (d <= 1024) return 16;
  return 0;
}

int* dev_err_word();   // skge_update.hip: the device error word (Accum::err)
inline Accum accum_of(const skge_table_t* t) {
  Accum a;
  a.sum = t->acc_sum;
  a.cnt = t->acc_cnt;
  a.touched = t->acc_touched;
  a.width = t->width;
  a.mode = t->acc_mode;
  a.replicas = t->acc_replicas > 1 ? t->acc_replicas : 1;
  a.rows = t->rows;
  a.err = t->acc_mode == SKGE_ACC_FX64 ? dev_err_word() : nullptr;
  return a;
}

inline int check_table(const skge_table_t* t, const char* name, bool need_acc) {
  SKGE_CHECK_ARG(t != nullptr, "%s: table is NULL", name);
  SKGE_CHECK_ARG(t->param != nullptr, "%s: param is NULL", name);
  SKGE_CHECK_ARG(t->rows > 0 && t->width > 0, "%s: bad shape %d x %d", name, t->rows, t->width);
  SKGE_CHECK_ARG(t->acc_mode == SKGE_ACC_F32 || t->acc_mode == SKGE_ACC_I16X4 ||
                     t->acc_mode == SKGE_ACC_FX64,
                 "%s: unknown accumulator mode %d", name, t->acc_mode);
  SKGE_CHECK_ARG(t->acc_mode != SKGE_ACC_FX64 || (t->width <= 1024 && t->acc_replicas <= 1),
                 "%s: the deterministic (fixed-point) accumulator needs width <= 1024 and one "
                 "copy", name);
  SKGE_CHECK_ARG(t->acc_mode == SKGE_ACC_F32 || (t->width % 4 == 0 && t->width <= 1024),
                 "%s: packed accumulator needs width %% 4 == 0 and <= 1024", name);
  // packed sums are TransE-L1's exact integer sign sums: no regularisation
  // terms and the occurrence count as the divisor (the packed applies' fast
  // AdaGrad step / projection forms are argued for exactly that case,
  // skge_device.h adagrad_step_fast)
  SKGE_CHECK_ARG(t->acc_mode != SKGE_ACC_I16X4 ||
                     (t->rin == 0.0f && t->rout == 0.0f && t->fixed_div <= 0.0f),
                 "%s: packed accumulator needs rin == rout == 0 and no fixed divisor", name);
  if (need_acc) {
    SKGE_CHECK_ARG(t->acc_sum && t->acc_cnt, "%s: accumulator buffers missing", name);
  }
  SKGE_CHECK_ARG(t->acc_replicas <= 1 || t->acc_touched == nullptr,
                 "%s: replicated accumulators must be dense (acc_touched NULL)", name);
  SKGE_CHECK_ARG(t->acc_replicas <= 1 || t->acc_replicas == 2 || t->acc_replicas == 4 ||
                     t->acc_replicas == 8 || t->acc_replicas == 16 || t->acc_replicas == 32,
                 "%s: acc_replicas must be 1, 2, 4, 8, 16 or 32", name);
  return SKGE_OK;
}

// producers that do not spread over replicas
inline int check_single(const skge_table_t* t, const char* name) {
  SKGE_CHECK_ARG(t->acc_replicas <= 1, "%s: this producer needs a single accumulator copy", name);
  return SKGE_OK;
}

// producers that only write fp32 accumulators
inline int check_f32(const skge_table_t* t, const char* name) {
  // float-valued sums: fp32 atomics, or the deterministic fixed-point form
  // (producers add through acc_row, which handles both)
  SKGE_CHECK_ARG(t->acc_mode == SKGE_ACC_F32 || t->acc_mode == SKGE_ACC_FX64,
                 "%s: this producer needs an fp32 (or fixed-point) accumulator", name);
  return SKGE_OK;
}

// slot records: a table without acc_touched is dense (nothing recorded)
inline int check_slots(const skge_table_t* t, long long nslots, const char* name) {
  if (t->acc_touched == nullptr) return SKGE_OK;
  SKGE_CHECK_ARG(nslots >= 0 && nslots <= t->touched_cap,
                 "%s: %lld touched slots needed, capacity %d", name, nslots, t->touched_cap);
  return SKGE_OK;
}

inline TripleSet triple_set_view(const void* set, int64_t capacity) {
  TripleSet ts;
  ts.slots = (const int4*)set;
  ts.filter = (const uint32_t*)((const int4*)set + capacity);
  ts.mask = (uint64_t)(capacity - 1);
  ts.fmask = (uint64_t)(8 * capacity - 1);
  return ts;
}

// skge_pipeline.hip: draw every negative of the epoch whose key is *epoch_key
// (rec[j] = (s, o, p, s' or -1), rec_n1[j] = o' or -1 for positive j of the
// epoch's order)
int launch_epoch_sample(hipStream_t st, const int* trip, long long T, uint64_t seed,
                        const uint64_t* epoch_key, TripleSet set, int n_ent, int ntries,
                        int4* rec, int* rec_n1);

// skge_grad.hip: HolE pairwise, one positive (both of its pairs) per wave
bool hole_pos_ok(int af, const skge_table_t* ent, const skge_table_t* rel, int d);
// the per-positive HolE kernels run their correlations through the wave FFT
// (skge_hole_fft.h) for this d (unless SKGE_HOLE_DIRECT=1)
bool hole_use_fft(int d);
int launch_hole_pos(hipStream_t st, int af, const skge_table_t* ent, const skge_table_t* rel,
                    int d, const int4* rec, const int* rec_n1, long long start, int count,
                    float margin, int* nviol, int* fold, int* total);

// The RESCAL W updater's step after the fused front (skge_rescal.hip
// k_rescal_front_fused): W[p] from relation p's split-K dW partial tiles,
// gated on the batch's violations; run by the entity apply's launch
// (skge_update.hip k_apply_wstep).  part == nullptr: no W step pending.
struct WStep {
  const float* part;      // [M][nt * nt][splits][64 * 64]
  const int* rel_off;     // [M + 1] the batch's relation bucket offsets
  const int* dwcnt;       // [M] dW items per relation (combined dW), or nullptr: the buckets
  float* W;
  float* A;               // AdaGrad state or nullptr
  int* ucnt;              // optional updateCounts
  const int* gate;        // the batch's violation count
  int M, d, splits, opt;
  float lr, rin, rout, fdiv;
  // the W step done inside the fused front, speculatively into the other
  // buffer (one dW split per tile): the apply only makes it current when the
  // batch has violations (*cur ^= 1); cur == nullptr: the step above
  int* cur;               // 0: W_b in W / A (the caller's), 1: in W1 / A1
  float* W1;
  float* A1;
  // set by the row-grouped RESCAL apply (skge_rescal.hip k_rescal_fold): the
  // entity rows and the W step's flip are done; only the epoch end's W sync
  // (cur) is left to the caller
  int applied;
};
int apply_with_wstep(hipStream_t st, const skge_table_t* ent, int nslots, const WStep& w);
// end of an epoch with the in-front W step: the current buffer back into the
// caller's W / state, cur = 0 (skge_rescal.hip)
int rescal_w_sync(hipStream_t st, const WStep& w);

}  // namespace skge

// skge_rescal.hip / skge_update.hip: the device pair loop's RESCAL batch
bool rescal_pair_mfma_selected(int d, int M);
// the device pair loop's RESCAL buckets for a whole epoch (skge_rescal.hip)
bool rescal_epoch_ok(int M);
size_t rescal_epoch_ws_bytes(int bs, int nb, int M, int d);
int rescal_epoch_bucket(hipStream_t st, const int* pos, const int* neg, long long T, int bs, int nb,
                        int M, int d, void* ws, const int4* rec = nullptr,
                        const int* rec_n1 = nullptr);
// the epoch's row grouping fits (k_rs_rows_ep: 4 bs slots per batch in LDS)
bool rs_rows_ok(int bs);
int skge_rescal_pos_grad_mfma_ep(hipStream_t st, int af, const skge_table_t* ent,
                                 const skge_table_t* rel, int d, const int4* rec,
                                 const int* rec_n1, long long T, int bs, int nb, int b,
                                 float margin, void* ws, int* nviol,
                                 skge::WStep* wstep = nullptr);
int skge_rescal_pos_grad_mfma(hipStream_t st, int af, const skge_table_t* ent,
                              const skge_table_t* rel, int d, const int* pos, const int* neg,
                              const int4* rec, const int* rec_n1, long long start, int count,
                              float margin, void* workspace, size_t ws_bytes, int* nviol);
