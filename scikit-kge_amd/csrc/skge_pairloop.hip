// Device pair loop for every model: one epoch of PairwiseStochasticTrainer
// with RandomModeSampler(1, [0, 1]) (skge/base.py:1242-1291, 1394-1427;
// skge/sample.py:28-46), captured once into a hipGraph and replayed.
//
//   k_epoch_sample (skge_pipeline.hip)  the epoch's permutation and every
//       negative, one thread per positive: records (s, o, p, s'), o'
//   k_pairs_of_epoch  every batch's explicit pairs at once, in the reference's
//       order (the records do not depend on the parameters) -- positive j
//       gives pair 2j (s-corrupted) and 2j+1 (o-corrupted); a negative the
//       sampler did not find in ntries draws becomes a SKIPPED pair (positive
//       relation -1, see skge_pair_grad) -- and clears the batches' gate words
//   per batch b (the reference's np.split geometry):
//     skge_pair_step  score + margin test + contributions (+ RESCAL dW) +
//       segment mean + updater + projection, gated on the batch's violations
//       (its own gate word)
//   k_pairs_epoch_end  the gate words' total into the caller's count, key + 1
//
// The per-batch kernels are the ones of the explicit-pair API, so a device
// epoch trains exactly like feeding the same pairs through skge_pair_step.
// Exception: HolE (d % 4 == 0, d <= 256) scores both pairs of a positive in
// one wave straight from the records (k_hole_pos, skge_grad.hip): the same
// pairs, contributions and counts, 7 correlations per positive instead of 12.
#include <cstdlib>
#include <vector>

#include "skge_host.h"
#include "skge_hole_fft.h"
#include "skge_sampler.h"

namespace skge {

__global__ __launch_bounds__(256) void k_pairs_of_epoch(const int4* __restrict__ rec,
                                                        const int* __restrict__ rec_n1,
                                                        long long T, int* __restrict__ pos,
                                                        int* __restrict__ neg,
                                                        int* __restrict__ gates, int nb,
                                                        int dedup) {
  for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x; j < T;
       j += (long long)gridDim.x * blockDim.x) {
    if (j < nb) gates[j] = 0;
    if (pos == nullptr) continue;   // HolE positive path: the records are its input
    const int4 r = rec[j];
    const int n1 = rec_n1[j];
    if (dedup) {   // RESCAL: each positive once ([T][3]), its two negatives ([T][2][3])
      const bool k0 = r.w >= 0, k1 = n1 >= 0;
      int* pp = pos + 3 * (size_t)j;
      int* nn = neg + 6 * (size_t)j;
      pp[0] = r.x;
      pp[1] = r.y;
      pp[2] = (k0 || k1) ? r.z : -1;
      nn[0] = k0 ? r.w : r.x;
      nn[1] = r.y;
      nn[2] = k0 ? r.z : -1;
      nn[3] = r.x;
      nn[4] = k1 ? n1 : r.y;
      nn[5] = k1 ? r.z : -1;
      continue;
    }
    int* pp = pos + 6 * (size_t)j;
    int* nn = neg + 6 * (size_t)j;
    // pair 2j: mode 0 corrupts s; pair 2j+1: mode 1 corrupts o (sample.py:41-46)
    const bool k0 = r.w >= 0, k1 = n1 >= 0;
    pp[0] = r.x;
    pp[1] = r.y;
    pp[2] = k0 ? r.z : -1;
    nn[0] = k0 ? r.w : -1;
    nn[1] = k0 ? r.y : -1;
    nn[2] = k0 ? r.z : -1;
    pp[3] = r.x;
    pp[4] = r.y;
    pp[5] = k1 ? r.z : -1;
    nn[3] = k1 ? r.x : -1;
    nn[4] = k1 ? n1 : -1;
    nn[5] = k1 ? r.z : -1;
  }
}

__global__ __launch_bounds__(256) void k_pairs_epoch_end(const int* __restrict__ gates, int nb,
                                                         int* nviol_total, uint64_t* ek) {
  __shared__ int part[4];
  int v = 0;
  for (int k = threadIdx.x; k < nb; k += blockDim.x) v += gates[k];
  v = wave_sum_int(v);
  if (lane_id() == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (nviol_total) *nviol_total += part[0] + part[1] + part[2] + part[3];
    *ek += 1;
  }
}

}  // namespace skge

using namespace skge;

struct skge_pair_runner {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  int nlaunch = 0;
  int4* rec = nullptr;
  int* rec_n1 = nullptr;
  int* pairs = nullptr;   // the epoch's pairs: pos [2T][3], then neg [2T][3]
  int* nviol = nullptr;   // [nbatches]: each batch's gate word (its violations)
  void* ws = nullptr;
  size_t ws_bytes = 0;
};

static void pair_runner_free(skge_pair_runner_t* r) {
  if (!r) return;
  if (r->exec) (void)hipGraphExecDestroy(r->exec);
  if (r->graph) (void)hipGraphDestroy(r->graph);
  if (r->rec) (void)hipFree(r->rec);
  if (r->rec_n1) (void)hipFree(r->rec_n1);
  if (r->pairs) (void)hipFree(r->pairs);
  if (r->nviol) (void)hipFree(r->nviol);
  if (r->ws) (void)hipFree(r->ws);
  (void)hipGetLastError();   // a failed allocation must not poison later checks
  delete r;
}

extern "C" skge_pair_runner_t* skge_pair_runner_create(
    void* stream, int model, int af, const skge_table_t* ent, const skge_table_t* rel, int d,
    const int* trip, int64_t T, const void* set, int64_t set_capacity, int nbatches,
    uint64_t seed, uint64_t* epoch_key, float margin, int ntries, int* nviol_total) {
  auto fail = [](const char* fmt, const char* what) -> skge_pair_runner_t* {
    set_error(fmt, what);
    return nullptr;
  };
  if (!ent || !rel || !trip || !set || !epoch_key) return fail("%s", "NULL argument");
  if (model < SKGE_TRANSE_L1 || model > SKGE_RESCAL) return fail("%s", "unknown model");
  if (T <= 0 || T > INT32_MAX) return fail("%s", "T must be in [1, 2^31)");
  if (nbatches < 1 || nbatches > T) return fail("%s", "nbatches must be in [1, T]");
  if (set_capacity < 2 * T || (set_capacity & (set_capacity - 1)))
    return fail("%s", "set capacity must be a power of 2 >= 2T");
  if (ntries < 1) return fail("%s", "ntries >= 1");
  if (stream == nullptr) return fail("%s", "runner needs a non-default stream (graph capture)");
  hipStream_t st = as_stream(stream);
  // batch geometry of StochasticTrainer._optim (skge/base.py:1246-1268)
  const int64_t bs = T / nbatches;
  std::vector<std::pair<int64_t, int64_t>> batches;
  int64_t maxb = 0;
  for (int64_t s0 = 0; s0 < T; s0 += bs) {
    const int64_t c = (s0 + bs <= T) ? bs : T - s0;
    batches.push_back({s0, c});
    maxb = std::max(maxb, c);
  }
  const int Pmax = (int)(2 * maxb);
  if ((long long)4 * Pmax > ent->touched_cap && ent->acc_touched)
    return fail("%s", "entity accumulator needs 8 * batch_size touched slots");
  // HolE with the register-tiled correlations: both pairs of a positive in
  // one wave straight from the records, 4 entity slots and 1 relation slot per
  // positive (SKGE_HOLE_PAIRS=1 keeps the explicit pairs)
  const char* hp = getenv("SKGE_HOLE_PAIRS");
  const bool hpos = model == SKGE_HOLE && !(hp && atoi(hp)) && hole_pos_ok(af, ent, rel, d);
  // RESCAL on the matrix cores: each positive once in the GEMMs and dW, both
  // of its pairs per scatter wave (k_rescal_pos_scatter; SKGE_RESCAL_PAIRS=1
  // keeps the explicit pairs)
  const char* rp = getenv("SKGE_RESCAL_PAIRS");
  const bool rpos = model == SKGE_RESCAL && !(rp && atoi(rp)) &&
                    rescal_pair_mfma_selected(d, rel->rows);
  const int nb = (int)batches.size();
  // RESCAL: every batch's relation buckets built once per epoch, up front (the
  // items do not depend on the parameters); SKGE_RESCAL_EPOCH_BUCKETS=0 keeps
  // the per-batch bucketing
  const char* eb = getenv("SKGE_RESCAL_EPOCH_BUCKETS");
  const bool rep = rpos && rescal_epoch_ok(rel->rows) && !(eb && atoi(eb) == 0);
  skge_pair_runner_t* r = new skge_pair_runner_t();
  r->ws_bytes = rep ? rescal_epoch_ws_bytes((int)bs, nb, rel->rows, d)
                    : skge_pair_step_workspace_bytes(model, Pmax, rel->rows, d);
  if (hipMalloc(&r->rec, (size_t)T * sizeof(int4)) != hipSuccess ||
      hipMalloc(&r->rec_n1, (size_t)T * sizeof(int)) != hipSuccess ||
      (!hpos && hipMalloc(&r->pairs, (size_t)T * 12 * sizeof(int)) != hipSuccess) ||
      hipMalloc(&r->nviol, (size_t)nb * sizeof(int)) != hipSuccess ||
      (r->ws_bytes && hipMalloc(&r->ws, r->ws_bytes) != hipSuccess) ||
      hipMemset(r->nviol, 0, (size_t)nb * sizeof(int)) != hipSuccess) {
    pair_runner_free(r);
    return fail("%s", "pair runner: device allocation failed");
  }
  int* pos = r->pairs;
  int* neg = r->pairs ? r->pairs + (size_t)T * 6 : nullptr;
  const TripleSet ts = triple_set_view(set, set_capacity);
  if (model == SKGE_HOLE && hole_use_fft(d) && !hole_fft_table(d)) {   // before the capture
    pair_runner_free(r);
    return fail("%s", "pair runner: HolE FFT twiddle table allocation failed");
  }
  if (hipStreamSynchronize(st) != hipSuccess ||
      hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    pair_runner_free(r);
    return fail("%s", "hipStreamBeginCapture failed");
  }
  int rc = launch_epoch_sample(st, trip, (long long)T, seed, epoch_key, ts, ent->rows, ntries,
                               r->rec, r->rec_n1);
  if (!rc) {
    const int64_t blocks = std::max((int64_t)1, std::min((T + 255) / 256, (int64_t)4096));
    hipLaunchKernelGGL(k_pairs_of_epoch, dim3((unsigned)blocks), dim3(256), 0, st, r->rec,
                       r->rec_n1, (long long)T, pos, neg, r->nviol, nb, rpos ? 1 : 0);
    if (hipGetLastError() != hipSuccess) {
      set_error("pairs launch failed");
      rc = SKGE_EHIP;
    }
    if (!rc && rep) rc = rescal_epoch_bucket(st, pos, neg, (long long)T, (int)bs, nb, rel->rows, d,
                                             r->ws, r->rec, r->rec_n1);
  }
  WStep wsync{};   // RESCAL with the in-front W step: synced back at the epoch's end
  for (int k = 0; k < nb && !rc; ++k) {
    const long long start = batches[k].first;
    const int count = (int)batches[k].second;
    int* gate = r->nviol + k;
    if (hpos) {
      rc = launch_hole_pos(st, af, ent, rel, d, r->rec, r->rec_n1, start, count, margin, gate,
                           nullptr, nullptr);
      if (!rc) {
        skge_table_t t[2] = {*ent, *rel};
        t[0].gate = gate;
        t[1].gate = gate;
        const int ns[2] = {4 * count, count};
        rc = skge_accum_apply(stream, t, 2, ns);
      }
    } else if (rpos) {
      WStep wst{};   // set by the fused front (Linear): the W step rides the entity apply
      rc = rep ? skge_rescal_pos_grad_mfma_ep(st, af, ent, rel, d, r->rec, r->rec_n1, (long long)T,
                                              (int)bs, nb, k, margin, r->ws, gate, &wst)
               : skge_rescal_pos_grad_mfma(st, af, ent, rel, d, pos + 3 * start, neg + 6 * start,
                                           r->rec, r->rec_n1, start, count, margin, r->ws,
                                           r->ws_bytes, gate);
      if (!rc && wst.applied) {   // the row-grouped apply updated the entity rows and W
        if (wst.cur) wsync = wst;
      } else if (!rc) {   // the entity table's apply (and W's, unless the dW kernel updated it)
        skge_table_t te = *ent;
        te.gate = gate;
        const int ns = 4 * count;
        rc = wst.part ? apply_with_wstep(st, &te, ns, wst) : skge_accum_apply(stream, &te, 1, &ns);
        if (wst.cur) wsync = wst;
      }
    } else {
      rc = skge_pair_step(stream, model, af, ent, rel, d, pos + 6 * start, neg + 6 * start,
                          2 * count, margin, r->ws, r->ws_bytes, gate);
    }
  }
  if (!rc && wsync.cur) rc = rescal_w_sync(st, wsync);
  if (!rc) {
    hipLaunchKernelGGL(k_pairs_epoch_end, dim3(1), dim3(256), 0, st, r->nviol, nb, nviol_total,
                       epoch_key);
    if (hipGetLastError() != hipSuccess) {
      set_error("epoch end launch failed");
      rc = SKGE_EHIP;
    }
  }
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(st, &g);
  if (rc || e != hipSuccess) {
    if (!rc) set_error("hipStreamEndCapture: %s", hipGetErrorString(e));
    if (g) (void)hipGraphDestroy(g);
    pair_runner_free(r);
    return nullptr;
  }
  r->graph = g;
  size_t nnodes = 0;
  if (hipGraphGetNodes(g, nullptr, &nnodes) == hipSuccess) r->nlaunch = (int)nnodes;
  e = hipGraphInstantiate(&r->exec, g, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    set_error("hipGraphInstantiate: %s", hipGetErrorString(e));
    pair_runner_free(r);
    return nullptr;
  }
  return r;
}

extern "C" int skge_epoch_sample(void* stream, const int* trip, int64_t T, const void* set,
                                 int64_t set_capacity, int n_ent, uint64_t seed,
                                 const uint64_t* epoch_key, int ntries, int* rec, int* rec_n1) {
  SKGE_CHECK_ARG(trip && set && epoch_key && rec && rec_n1, "NULL argument");
  SKGE_CHECK_ARG(T > 0 && T <= INT32_MAX, "T must be in [1, 2^31)");
  SKGE_CHECK_ARG(set_capacity >= 2 * T && !(set_capacity & (set_capacity - 1)),
                 "set capacity must be a power of 2 >= 2T");
  SKGE_CHECK_ARG(n_ent > 0 && ntries >= 1, "bad n_ent / ntries");
  return launch_epoch_sample(as_stream(stream), trip, (long long)T, seed, epoch_key,
                             triple_set_view(set, set_capacity), n_ent, ntries, (int4*)rec,
                             rec_n1);
}

extern "C" int skge_pair_runner_run(skge_pair_runner_t* r, void* stream, int nepochs) {
  SKGE_CHECK_ARG(r && r->exec, "bad runner");
  for (int i = 0; i < nepochs; ++i) SKGE_CHECK_HIP(hipGraphLaunch(r->exec, as_stream(stream)));
  return SKGE_OK;
}

extern "C" int skge_pair_runner_nlaunches(const skge_pair_runner_t* r) {
  return r ? r->nlaunch : -1;
}

extern "C" void skge_pair_runner_destroy(skge_pair_runner_t* r) { pair_runner_free(r); }
