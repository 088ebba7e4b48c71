// Device pair loop for every model: one epoch of PairwiseStochasticTrainer
// with RandomModeSampler(1, [0, 1]) (skge/base.py:1242-1291, 1394-1427;
// skge/sample.py:28-46), captured once into a hipGraph and replayed.
//
//   k_epoch_sample (skge_pipeline.hip)  the epoch's permutation and every
//       negative, one thread per positive: records (s, o, p, s'), o'
//   per batch b (the reference's np.split geometry):
//     k_pairs_of_records  the batch's explicit pairs in the reference's order
//       -- positive j gives pair 2j (s-corrupted) and 2j+1 (o-corrupted); a
//       negative the sampler did not find in ntries draws becomes a SKIPPED
//       pair (positive relation -1, see skge_pair_grad) -- and folds the
//       previous batch's violation count into the epoch total
//     skge_pair_step  score + margin test + contributions (+ RESCAL dW) +
//       segment mean + updater + projection, gated on the batch's violations
//   k_pairs_epoch_end  last fold, epoch key + 1
//
// The per-batch kernels are the ones of the explicit-pair API, so a device
// epoch trains exactly like feeding the same pairs through skge_pair_step.
// Exception: HolE (d % 4 == 0, d <= 256) scores both pairs of a positive in
// one wave straight from the records (k_hole_pos, skge_grad.hip): the same
// pairs, contributions and counts, 7 correlations per positive instead of 12.
#include <cstdlib>
#include <vector>

#include "skge_host.h"
#include "skge_sampler.h"

namespace skge {

__global__ __launch_bounds__(256) void k_pairs_of_records(const int4* __restrict__ rec,
                                                          const int* __restrict__ rec_n1,
                                                          long long start, int count,
                                                          int* __restrict__ pos,
                                                          int* __restrict__ neg, int* nviol,
                                                          int* nviol_total) {
  const int j0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (j0 == 0) {   // the previous batch's gate word -> epoch total, then re-arm
    if (nviol_total) *nviol_total += *nviol;
    *nviol = 0;
  }
  for (int j = j0; j < count; j += gridDim.x * blockDim.x) {
    const int4 r = rec[start + j];
    const int n1 = rec_n1[start + j];
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

// nviol2: the second gate word of the HolE positive path (batch parity), or null
__global__ void k_pairs_epoch_end(int* nviol, int* nviol2, int* nviol_total, uint64_t* ek) {
  if (nviol_total) *nviol_total += *nviol + (nviol2 ? *nviol2 : 0);
  *nviol = 0;
  if (nviol2) *nviol2 = 0;
  *ek += 1;
}

}  // namespace skge

using namespace skge;

struct skge_pair_runner {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  int nlaunch = 0;
  int4* rec = nullptr;
  int* rec_n1 = nullptr;
  int* pairs = nullptr;   // pos [2*bs][3], then neg [2*bs][3]
  int* nviol = nullptr;   // the batch's gate word
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
  skge_pair_runner_t* r = new skge_pair_runner_t();
  r->ws_bytes = skge_pair_step_workspace_bytes(model, Pmax, rel->rows, d);
  if (hipMalloc(&r->rec, (size_t)T * sizeof(int4)) != hipSuccess ||
      hipMalloc(&r->rec_n1, (size_t)T * sizeof(int)) != hipSuccess ||
      hipMalloc(&r->pairs, (size_t)Pmax * 6 * sizeof(int)) != hipSuccess ||
      hipMalloc(&r->nviol, 256) != hipSuccess ||
      (r->ws_bytes && hipMalloc(&r->ws, r->ws_bytes) != hipSuccess) ||
      hipMemset(r->nviol, 0, 256) != hipSuccess) {
    pair_runner_free(r);
    return fail("%s", "pair runner: device allocation failed");
  }
  int* pos = r->pairs;
  int* neg = r->pairs + (size_t)Pmax * 3;
  const TripleSet ts = triple_set_view(set, set_capacity);
  if (hipStreamSynchronize(st) != hipSuccess ||
      hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    pair_runner_free(r);
    return fail("%s", "hipStreamBeginCapture failed");
  }
  // HolE with the register-tiled correlations: both pairs of a positive in
  // one wave straight from the records, 4 entity slots and 1 relation slot per
  // positive (SKGE_HOLE_PAIRS=1 keeps the explicit pairs).  Its gate words
  // alternate by batch parity: each batch's kernel folds the previous batch's
  // word into the epoch total.
  const char* hp = getenv("SKGE_HOLE_PAIRS");
  const bool hpos = model == SKGE_HOLE && !(hp && atoi(hp)) && hole_pos_ok(af, ent, rel, d);
  int* gate[2] = {r->nviol, r->nviol + 32};   // separate 128-B lines
  int rc = launch_epoch_sample(st, trip, (long long)T, seed, epoch_key, ts, ent->rows, ntries,
                               r->rec, r->rec_n1);
  r->nlaunch = 1;
  for (size_t k = 0; k < batches.size() && !rc; ++k) {
    const int count = (int)batches[k].second;
    if (hpos) {
      rc = launch_hole_pos(st, af, ent, rel, d, r->rec, r->rec_n1, (long long)batches[k].first,
                           count, margin, gate[k & 1], gate[(k + 1) & 1], nviol_total);
      if (!rc) {
        skge_table_t t[2] = {*ent, *rel};
        t[0].gate = gate[k & 1];
        t[1].gate = gate[k & 1];
        const int ns[2] = {4 * count, count};
        rc = skge_accum_apply(stream, t, 2, ns);
      }
      r->nlaunch += 1;
      continue;
    }
    const int blocks = std::max(1, std::min((count + 255) / 256, 1024));
    hipLaunchKernelGGL(k_pairs_of_records, dim3(blocks), dim3(256), 0, st, r->rec, r->rec_n1,
                       (long long)batches[k].first, count, pos, neg, r->nviol, nviol_total);
    if (hipGetLastError() != hipSuccess) {
      set_error("pairs launch failed");
      rc = SKGE_EHIP;
      break;
    }
    rc = skge_pair_step(stream, model, af, ent, rel, d, pos, neg, 2 * count, margin, r->ws,
                        r->ws_bytes, r->nviol);
    r->nlaunch += 1;
  }
  if (!rc) {
    hipLaunchKernelGGL(k_pairs_epoch_end, dim3(1), dim3(1), 0, st, r->nviol,
                       hpos ? r->nviol + 32 : nullptr, nviol_total, epoch_key);
    r->nlaunch += 1;
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
