/*
 * skge_hip.h -- C ABI of libskgehip.so, the MI355X (gfx950) HIP implementation
 * of scikit-kge's mini-batch training hot path (score + gradient + update).
 *
 * The reference is pure Python/NumPy; its "FFI" for this path is the duck-typed
 * model / updater / trainer protocol of skge.  Each
 * entry point below replaces one piece of that protocol; the Python facade
 * (scikit-kge_amd/skge_amd) binds them with ctypes and keeps the reference's
 * class names, kwargs and return shapes.
 *
 * Conventions
 *  - Ownership: the caller allocates every buffer (device memory, e.g. torch
 *    tensors).  The library never frees caller memory.
 *  - Async: every call is stream-ordered on the caller's hipStream_t (passed as
 *    void*; NULL = the legacy default stream).  No call synchronises, allocates
 *    or copies to the host, so sequences of calls can be captured in a hipGraph.
 *  - Errors: int return, 0 = OK, <0 = error (SKGE_E*); the message of the
 *    last failure on the calling thread is returned by skge_last_error().
 *  - Triples are (s, o, p) int32 triplets, row-major [n][3]
 *    (skge/base.py:511, skge/util.py:104-110).
 *  - Parameters are fp32 row-major tables [rows][width]; width = d for E / R,
 *    d*d for RESCAL's W.
 *  - Accumulator invariant: between batches acc_sum == 0 and acc_cnt == 0
 *    for every table (zero them once at allocation).
 */
#ifndef SKGE_HIP_H
#define SKGE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SKGE_ABI_VERSION 2

enum {
  SKGE_OK = 0,
  SKGE_EINVAL = -1,   /* bad argument (shape, enum, null pointer) */
  SKGE_EHIP = -2,     /* a HIP runtime call failed */
  SKGE_ENOTSUP = -3   /* unsupported configuration (e.g. d > 1024) */
};

/* models (skge/transe.py, skge/hole.py, skge/rescal.py) */
enum { SKGE_TRANSE_L1 = 0, SKGE_TRANSE_L2 = 1, SKGE_HOLE = 2, SKGE_RESCAL = 3 };
/* activation functions (skge/actfun.py:13-57) */
enum { SKGE_AF_LINEAR = 0, SKGE_AF_SIGMOID = 1, SKGE_AF_TANH = 2, SKGE_AF_RELU = 3 };
/* updaters (skge/param.py:124-155) */
enum { SKGE_SGD = 0, SKGE_ADAGRAD = 1 };
/* post-update projections (skge/param.py:161-174) */
enum { SKGE_POST_NONE = 0, SKGE_POST_NORMALIZE = 1, SKGE_POST_NORMLESS1 = 2 };
/* accumulator encodings */
enum {
  SKGE_ACC_F32 = 0,    /* acc_sum: fp32 [rows][width] */
  SKGE_ACC_I16X4 = 1,  /* acc_sum: exact integer sums of TransE-L1 sign contributions,
                          four elements per int64 (elements 4q..4q+3 in qword q, added
                          with one 64-bit integer atomic; exact while each 16-bit
                          field's total stays within +-32767, which a row whose
                          per-batch count is <= 32767 guarantees: the apply kernels
                          flag larger counts, skge_device_error bit 2) -- produced
                          only by skge_transe_sample_grad / the pipelined runner with
                          l1 != 0 and width % 4 == 0 */
  SKGE_ACC_FX64 = 3,   /* the deterministic reduce mode (float-valued models, off by
                          default): acc_sum is int64 [rows][width] fixed point with 40
                          fractional bits; every contribution is rounded once to that
                          grid and added with an exact integer atomic, so the sums --
                          and the parameters after the apply -- are the same bits run
                          to run whatever order the adds arrive in (the reference's
                          CSR mat-vec is deterministic too, skge/util.py:53-101).
                          Entity / narrow relation tables (width <= 1024, one copy) of
                          the per-batch paths and the device pair loop */
  SKGE_ACC_I8X4 = 4,   /* pipelined TransE-L1 runner's ENTITY table only: the exact sums
                          in four 8-bit fields per uint32 (acc_sum [rows][width/4]
                          dwords, one 32-bit integer atomic per quad), exact while a
                          row's per-batch count is <= 127 (the runner flags larger
                          counts); half the atomic bytes of int16x4 */
  SKGE_ACC_I32X2 = 2   /* pipelined runner's RELATION table only: the same exact sums
                          with 32-bit fields, two elements per int64 (a hot
                          relation's per-batch count passes 32767 long before any
                          entity row's does); the runner keeps these sums itself */
};

/*
 * One parameter table with its updater state and its segment-sum accumulator.
 * The gradient of a touched row r is
 *     g = (acc_sum[r] + rin * param[r]) / div + rout * param[r],
 *     div = fixed_div > 0 ? fixed_div : acc_cnt[r]
 * which covers every variant of the reference:
 *   mean                 Sm.dot(G) / n                     (transe.py:136)
 *   mean + rparam*P      hole.py:33,40,83  rescal.py:70,239
 *   (sum + rparam*P)/n   rescal.py:299-302 (rparam inside)
 *   (sum + rparam*W)/2   rescal.py:287-290 (divisor quirk)
 *
 * Touched rows are recorded in FIXED SLOTS (no shared counter): every
 * contribution site of a launch owns one slot of acc_touched and writes there
 * the row id it counted (or -1 if it added nothing); several slots may name
 * the same row, and consumers claim each row once (atomicExch on acc_cnt).
 * Slot maps:
 *   skge_pair_grad          ent: 4i+{0:sp,1:op,2:sn,3:on}   rel: 2i+{0:pp,1:pn}
 *   skge_triple_grad        ent: 2i+{0:s,1:o}               rel (HolE): i
 *   skge_rescal_wgrad       W:   slot p (all M slots)
 *   skge_transe_sample_grad ent: 4j+{0:s,1:o,2:s',3:o'}     rel: j
 * Consumers (apply / reset) take the slot count of the producing launch.
 * A narrow table with acc_touched == NULL is applied DENSELY: every row whose
 * count is non-zero (meant for small tables such as TransE's R; producers
 * then record nothing for it).  Replicated accumulators (acc_replicas > 1)
 * are produced by skge_transe_sample_grad only.
 */
typedef struct skge_table {
  float *param;        /* [rows][width] */
  float *state;        /* AdaGrad accumulator p2 [rows][width]; NULL for SGD */
  float *acc_sum;      /* [rows][width] */
  int *acc_cnt;        /* [rows] */
  int *acc_touched;    /* [touched_cap] slot -> row or -1; NULL: dense apply */
  int rows;
  int width;
  int touched_cap;     /* capacity of acc_touched (slots) */
  int acc_mode;        /* SKGE_ACC_F32 | SKGE_ACC_I16X4 | SKGE_ACC_FX64 (| runner-only modes) */
  int acc_replicas;    /* dense tables only: acc_sum / acc_cnt hold this many
                          copies ([replicas][rows][...]); producers spread their
                          adds over the copies (fewer same-address atomics on
                          hot rows such as TransE's 18 relations) and the apply
                          sums them.  0 or 1 = a single copy; else 2, 4, 8, 16
                          or 32. */
  int opt;             /* SKGE_SGD | SKGE_ADAGRAD */
  int post;            /* SKGE_POST_* */
  float lr;
  float rin, rout, fixed_div;
  const int *gate;     /* optional: if non-NULL and *gate == 0, the update is
                          skipped (the model returned None: no violations) */
  int *upd_count;      /* optional [rows]: AdaGrad applies add 1 per updated row
                          (Parameter.updateCounts, skge/param.py:149-150) */
  int *violations;     /* optional [rows], entity table of a TransE pair launch:
                          +1 per violating pair for each distinct entity of
                          {sn, on, sp, op} (E.violations, skge/transe.py:78-83) */
} skge_table_t;

int skge_abi_version(void);
const char *skge_last_error(void);
/* Synchronizes the stream and returns the error bits raised by device kernels
 * since the last reset (2 = a packed row's count exceeded 32767; 4 = an
 * SKGE_ACC_FX64 sum wrapped past its 2^23 range in gradient units -- every
 * fixed-point add checks its own signed overflow -- or a decoded sum was at
 * or past 2^22, half that range); reset != 0 clears them. */
int skge_device_error(void *stream, int reset);

/*
 * Pairwise scoring + contribution scatter for P explicit (positive, negative)
 * pairs.  Replaces the numeric part of Model._pairwise_gradients:
 *   TransE  skge/transe.py:48-165   (ent = E, rel = R)
 *   HolE    skge/hole.py:44-100     (ent = E, rel = R; af applied to scores)
 *   RESCAL  skge/rescal.py:78-139   (ent = E, rel = W; the dW part is
 *                                    skge_rescal_wgrad, fed by `coef`)
 * Writes the raw scores (pscore/nscore may be NULL), atomically adds the
 * violation count to *nviol, and accumulates every violating pair's
 * contribution rows into ent->acc_* / rel->acc_* (segment sum + counts).
 * coef (RESCAL only, [2P]): gp for every pair, then gn for every pair.
 * margin == -INFINITY: score only (nothing accumulated, no slots written).
 * A pair whose positive has relation -1 is SKIPPED (no score, no violation,
 * no contribution, coef 0; its negative is not read): the device pair loop
 * (skge_pair_runner_*) marks so a positive whose sampler found no negative
 * in ntries draws (skge/sample.py:41-46 drops that pair).  The same holds for
 * skge_pair_step.
 */
int skge_pair_grad(void *stream, int model, int af, const skge_table_t *ent,
                   const skge_table_t *rel, int d, const int *pos, const int *neg, int P,
                   float margin, float *pscore, float *nscore, float *coef, int *nviol);

/*
 * Logistic-loss scoring + contribution scatter for T labelled triples.
 * Replaces HolE._gradients (skge/hole.py:22-42) and RESCAL._gradients
 * (skge/rescal.py:37-76).  score may be NULL; *loss += sum logaddexp(0,-y*f);
 * coef [T] receives fs = -y*sigmoid(-y*f) (used by skge_rescal_wgrad).
 */
int skge_triple_grad(void *stream, int model, const skge_table_t *ent, const skge_table_t *rel,
                     int d, const int *trip, const float *ys, int T, float *score, float *coef,
                     float *loss);

/*
 * RESCAL relation-matrix gradient: for every relation p appearing in lists
 * a and b, acc_sum[p] = sum_i coef_i * outer(E[s_i], E[o_i]) and acc_cnt[p] =
 * number of occurrences (skge/rescal.py:61-70 and 113-125).
 */
int skge_rescal_wgrad(void *stream, const skge_table_t *ent, const skge_table_t *rel, int d,
                      const int *trip_a, const float *coef_a, int n_a, const int *trip_b,
                      const float *coef_b, int n_b);

/*
 * Materialise the segment mean held in a table's accumulator as the
 * reference's (grad_rows, sorted unique idx) pair (skge/util.py:53-101):
 * idx_out [rows], g_out [rows][width], *U_out = number of touched rows.
 * Resets the accumulator.  workspace: skge_collect_workspace_bytes(rows).
 */
size_t skge_collect_workspace_bytes(int rows);
int skge_accum_collect(void *stream, const skge_table_t *t, int *idx_out, float *g_out,
                       int *U_out, void *workspace, size_t ws_bytes);

/* Reset a table's accumulator (the rows in the first nslots slots) without
 * producing gradients. */
int skge_accum_reset(void *stream, const skge_table_t *t, int nslots);

/*
 * Updater call: param[idx] -= ... for U explicit (row, gradient) pairs, then
 * the projection.  Replaces ParameterUpdate.__call__ (skge/param.py:115-118)
 * with SGD._update (param.py:129-130) or AdaGrad._update (param.py:140-155),
 * then normalize / normless1 (param.py:161-174).  idx must be unique.
 */
int skge_update_rows(void *stream, const skge_table_t *t, const float *g, const int *idx, int U);

/*
 * Fused: segment mean + updater + projection straight from the accumulators
 * of up to 4 tables (trainer._batch_step, skge/base.py:1306-1316), resetting
 * the accumulator rows it reads.  nslots[i]: slot count of table i (the
 * producing launch's slot map, see skge_table_t).
 */
int skge_accum_apply(void *stream, const skge_table_t *tables, int ntables, const int *nslots);

/*
 * Explicit-pair training step: skge_pair_grad + (RESCAL dW) + apply
 * (one _pairwise_gradients + _batch_step, skge/base.py:1417-1427).  RESCAL
 * needs a workspace of skge_pair_step_workspace_bytes(model, P, rel->rows, d)
 * bytes (0 for the other models): for d <= 1024 and <= 8192 relations the
 * triples are grouped by relation and W[p] E[o], E[s] W[p] and dW run as fp32
 * MFMA GEMMs (skge_rescal.hip), otherwise as per-pair GEMVs.
 */
size_t skge_pair_step_workspace_bytes(int model, int P, int M, int d);
int skge_pair_step(void *stream, int model, int af, const skge_table_t *ent,
                   const skge_table_t *rel, int d, const int *pos, const int *neg, int P,
                   float margin, void *workspace, size_t ws_bytes, int *nviol);

/*
 * Labelled-triple (logistic) training step: skge_triple_grad + (RESCAL dW) +
 * apply (one StochasticTrainer._process_batch, skge/base.py:1293-1316).
 * RESCAL needs skge_triple_step_workspace_bytes(model, T, rel->rows, d)
 * bytes of workspace (0 for HolE): relation-grouped fp32 MFMA GEMMs for
 * d <= 1024 and <= 8192 relations, per-triple GEMVs otherwise.
 */
size_t skge_triple_step_workspace_bytes(int model, int T, int M, int d);
int skge_triple_step(void *stream, int model, const skge_table_t *ent, const skge_table_t *rel,
                     int d, const int *trip, const float *ys, int T, void *workspace,
                     size_t ws_bytes, float *loss);

/* ---------------- device-resident batch loop (throughput path) ---------------- */

/*
 * Build the set of training triples used by the negative sampler's rejection
 * test (skge/sample.py:41-44): an open-addressing table of `capacity` 16-byte
 * slots (power of two >= 2*T) followed by a one-hash filter of 8*capacity
 * bits that answers most "not a training triple" queries with one load.
 * `set` must hold skge_triple_set_bytes(capacity) bytes; zeroed by this call.
 */
size_t skge_triple_set_bytes(int64_t capacity);
int skge_triple_set_build(void *stream, const int *trip, int64_t T, void *set,
                          int64_t capacity);

/*
 * One PairwiseStochasticTrainer mini-batch of TransE, fully on device
 * (skge/base.py:1268-1284 + 1394-1427 with RandomModeSampler(1, [0, 1])):
 * positive j of the batch is triple perm_epoch(start + j) (a keyed bijection
 * of [0, T), keyed by *epoch_key so that a captured graph reshuffles per
 * epoch); for each positive, mode 0 corrupts s and mode 1 corrupts o with up
 * to ntries rejection draws against the triple set; both pairs are scored,
 * margin-tested and their contributions accumulated.  nviol_total (optional)
 * accumulates over batches; neg_out (optional, [count][2]) records the sampled
 * corrupted entity per mode (-1 = skipped).
 */
int skge_transe_sample_grad(void *stream, int l1, const skge_table_t *ent,
                            const skge_table_t *rel, int d, const int *trip, int64_t T,
                            const void *set, int64_t set_capacity, int64_t start, int count,
                            uint64_t seed, const uint64_t *epoch_key, float margin, int ntries,
                            int *nviol, int *nviol_total, int *neg_out);

/* Data-parallel TransE-L1 (one model over G ranks): the pipelined runner's
 * data-parallel form, skge_pipe_runner_dp_* below. */

/* perm_out[j] = perm_epoch(j) for j < n (tests / host-side replay). */
int skge_epoch_permutation(void *stream, int64_t T, uint64_t seed, const uint64_t *epoch_key,
                           int64_t *perm_out, int64_t n);

/* *epoch_key += 1 (one-thread kernel, so a captured epoch graph advances it). */
int skge_epoch_advance(void *stream, uint64_t *epoch_key);

/*
 * Native epoch runner: captures one epoch of the device batch loop
 * (nbatches sample_grad + apply launches + epoch_advance; the reference's
 * np.split geometry, skge/base.py:1246-1268) into a hipGraph once, then
 * replays it.  Returns an opaque handle (NULL on error).
 */
typedef struct skge_runner skge_runner_t;
skge_runner_t *skge_runner_create(void *stream, int l1, const skge_table_t *ent,
                                  const skge_table_t *rel, int d, const int *trip, int64_t T,
                                  const void *set, int64_t set_capacity, int nbatches,
                                  uint64_t seed, uint64_t *epoch_key, float margin, int ntries,
                                  int *nviol, int *nviol_total);
int skge_runner_run(skge_runner_t *r, void *stream, int nepochs);
int skge_runner_nlaunches(const skge_runner_t *r);
void skge_runner_destroy(skge_runner_t *r);

/*
 * Device pair loop for any model (TransE L1/L2, HolE, RESCAL): one epoch of
 * PairwiseStochasticTrainer with RandomModeSampler(1, [0, 1])
 * (skge/base.py:1242-1291, 1394-1427; skge/sample.py:28-46) captured into a
 * hipGraph: the epoch's permutation and negatives (the same keyed draws as
 * the TransE runners), then per batch the explicit pairs (positive j ->
 * pairs 2j: s-corrupted, 2j+1: o-corrupted; a negative not found in ntries
 * draws -> a skipped pair) and one skge_pair_step.  ent needs 8 * batch_size
 * touched slots, rel (if it records slots) 4 * batch_size.  *nviol_total
 * accumulates the violations.  nlaunches reports the graph's node count.
 */
typedef struct skge_pair_runner skge_pair_runner_t;
/* The epoch's draws as the pair loop (and the pipelined TransE runner) make
 * them: rec [T][4] = (s, o, p, s' or -1), rec_n1 [T] = o' or -1, for
 * position j of the epoch's order (tests / host-side replay). */
int skge_epoch_sample(void *stream, const int *trip, int64_t T, const void *set,
                      int64_t set_capacity, int n_ent, uint64_t seed, const uint64_t *epoch_key,
                      int ntries, int *rec, int *rec_n1);
skge_pair_runner_t *skge_pair_runner_create(void *stream, int model, int af,
                                            const skge_table_t *ent, const skge_table_t *rel,
                                            int d, const int *trip, int64_t T, const void *set,
                                            int64_t set_capacity, int nbatches, uint64_t seed,
                                            uint64_t *epoch_key, float margin, int ntries,
                                            int *nviol_total);
int skge_pair_runner_run(skge_pair_runner_t *r, void *stream, int nepochs);
int skge_pair_runner_nlaunches(const skge_pair_runner_t *r);
void skge_pair_runner_destroy(skge_pair_runner_t *r);

/*
 * Pipelined epoch runner for TransE-L1 with packed accumulators (the
 * throughput path).  Same result, bit for bit, as skge_runner_create's loop
 * with the same tables and arguments: all negatives of an epoch are drawn in
 * one launch, then each mini-batch is ONE launch that scores batch b while
 * applying batch b-1's updates.  Below 16k slot records per batch with d <= 64
 * (the default there; SKGE_PIPE_FUSED=1 forces it up to d <= 256): k_pipe_fused,
 * whose work items are first one scoring item per positive, then one item per
 * four slot records of the previous batch (applied) and four of the batch
 * before (zeroed); a row the previous batch touched is updated by each of its
 * readers itself, from its pre-update value, which stays readable because the
 * applier writes the row's other buffer (the runner's second copy of E and
 * its AdaGrad state; run() and profile() end by copying every row back into
 * the caller's tables).  Otherwise k_pipe_batch: apply waves beside scoring
 * waves that wait for a pending row's publisher (one apply wave per slot
 * record below 16k slot records; above, owner marks over the slot records).
 * Needs ent
 * in SKGE_ACC_I16X4 mode (SKGE_ACC_I8X4: int8x4 sums, counts <= 127), rel in
 * SKGE_ACC_I16X4 or SKGE_ACC_I32X2 mode (the encoding of the relation sums
 * the runner keeps), d % 4 == 0, an entity table with slot records (capacity
 * >= 4 * batch), a dense single-copy relation table and no gates.  Any batch
 * size: a row's 16-bit packed sums are exact while its per-batch count is
 * <= 32767 (each occurrence adds a coefficient no larger than the count it
 * adds), and the apply reports a larger count through skge_pipe_runner_error
 * (bit 2); 32-bit relation sums are exact below 2^29 positives.  Allocates
 * its extra accumulator copies, row buffers and per-row words itself (freed
 * by destroy).  *epoch_key must only advance (the runner advances it once per
 * epoch).  Replaces the per-batch loop of skge/base.py:1268-1284.
 */
typedef struct skge_pipe_runner skge_pipe_runner_t;
skge_pipe_runner_t *skge_pipe_runner_create(void *stream, const skge_table_t *ent,
                                            const skge_table_t *rel, int d, const int *trip,
                                            int64_t T, const void *set, int64_t set_capacity,
                                            int nbatches, uint64_t seed, uint64_t *epoch_key,
                                            float margin, int ntries, int *nviol_total);
/* skge_pipe_runner_create with a flags word: 0, or SKGE_PIPE_DP (the
 * data-parallel form below: TransE-L1, no hot rows, driven launch by launch;
 * run() / profile() refuse it). */
#define SKGE_PIPE_DP 1
skge_pipe_runner_t *skge_pipe_runner_create_ex(void *stream, const skge_table_t *ent,
                                               const skge_table_t *rel, int d, const int *trip,
                                               int64_t T, const void *set, int64_t set_capacity,
                                               int nbatches, uint64_t seed, uint64_t *epoch_key,
                                               float margin, int ntries, int *nviol_total,
                                               int flags);
/*
 * Pipelined HolE pairwise runner (skge/hole.py:44-100, E post normless1):
 * the same epoch structure as skge_pipe_runner_create -- launch g scores
 * batch b (both pairs of a positive per wave: k_hole_pos's seven correlations
 * and arithmetic) while other workgroups apply batch b-1's rows -- with fp32
 * sums: ent F32 with slot records (capacity >= 4 * batch), rel F32 dense
 * single copy, d % 4 == 0, 4 <= d <= 256, af an SKGE_AF_* code, no gates.
 * Draws the same pairs as skge_pair_runner_create's HolE path; parameters
 * equal its to fp32 rounding.  Driven by skge_pipe_runner_run / _profile /
 * _error / _nlaunches / _destroy.  Replaces skge/base.py:1268-1284 for HolE.
 */
skge_pipe_runner_t *skge_hole_pipe_runner_create(void *stream, int af, const skge_table_t *ent,
                                                 const skge_table_t *rel, int d, const int *trip,
                                                 int64_t T, const void *set, int64_t set_capacity,
                                                 int nbatches, uint64_t seed, uint64_t *epoch_key,
                                                 float margin, int ntries, int *nviol_total);
int skge_pipe_runner_run(skge_pipe_runner_t *r, void *stream, int nepochs);
/* synchronizes the stream; returns 0, or a bit set (results then invalid):
 * 1 = a bounded cross-workgroup wait gave up, 2 = a row's per-batch count
 * exceeded 32767 (packed sums may have wrapped); or a negative error code */
int skge_pipe_runner_error(skge_pipe_runner_t *r, void *stream);
int skge_pipe_runner_nlaunches(const skge_pipe_runner_t *r);
/* Hot entity rows of a TransE pipelined runner (hand-off kernel, int16x4
 * sums): rows whose subject/object occurrences put them in >= 4 slots of an
 * average batch and >= 8x the average row's (the hubs of a skewed KG), at
 * most 256.  Their per-batch sums and counts are spread over 4 replicas
 * (positive w into replica w % 4), and every scoring wave that reads a hub
 * computes its updated value itself from the replicas (exact integer sums:
 * bitwise the same result), so nothing waits on a hub and its atomics do not
 * serialise on one row.  Returns their number (0: none). */
int skge_pipe_runner_hot_rows(const skge_pipe_runner_t *r);
/* The batch kernel the runner launches: 0 k_pipe_batch, 1 k_pipe_fused,
 * 2 k_hole_pipe (-1: NULL runner) -- what a profile of its launches is named. */
int skge_pipe_runner_kernel(const skge_pipe_runner_t *r);
/* One epoch launched eagerly (trains like run(1)) with HIP events around every
 * launch: us_out[i] = launch i's duration (i = 0: negative draws, 1..nb1:
 * batches, nb1+1: flush, nb1+2: key advance); stats_out[3i..3i+2] = entity
 * rows applied, relation rows applied, violating pairs scored by launch i.
 * Both arrays need nlaunches entries (x3 for stats).  For the roofline.
 * Diagnostics: if trace_out is given, batch launch trace_launch (1..nb1+1)
 * records per-wave s_memrealtime stamps (10 ns): trace_out[0] = scoring
 * waves B, [1] = apply waves A, then 6 words per scoring wave (start, rows
 * loaded, pending rows settled, scored, atomics done, pending mask | 256 if
 * violating) and 2 per apply wave (start, end); trace_len must hold them. */
int skge_pipe_runner_profile(skge_pipe_runner_t *r, void *stream, float *us_out, int *stats_out,
                             int n, int trace_launch, uint64_t *trace_out, int64_t trace_len);
void skge_pipe_runner_destroy(skge_pipe_runner_t *r);
/* Batches per epoch (nb1; launch nb1 is the flush), or -1. */
int skge_pipe_runner_nbatches(const skge_pipe_runner_t *r);

/* ---- data-parallel form of the pipelined runner (SKGE_PIPE_DP) ----
 * ONE model replicated over G ranks (skge_amd/dp.py; skge/base.py:1268-1284,
 * 1394-1427 over the union batch).  Every rank creates the runner with the
 * same tables, KG, nbatches and seed (so every rank draws the same epoch
 * records) and runs, per epoch:
 *   dp_begin;
 *   for b in 0..nb1-1:
 *     dp_batch(b, lo, hi, rec_out, fold = G == 1)  -- ONE launch: applies batch
 *         b-1's rows (all ranks' contributions) and scores the rank's slice
 *         [lo, hi) of batch b, adding its contributions locally and writing
 *         one record per scored positive (skge_pipe_dp_record_bytes(d) each);
 *     all-gather of the slices' records (the caller's collective, rank-major:
 *         union position w's record at w);
 *     dp_scatter(b, gathered, lo, hi)  -- adds the other ranks' positives
 *         (skipped work when there are none);
 *   dp_batch(nb1, 0, 0, NULL, 0) (the flush); dp_end.
 * Sums are exact integers, so every replica equals one GPU's run over the
 * union batches bit for bit.  Each rank's violations (its slices) go to its
 * nviol_total at the flush. */
size_t skge_pipe_dp_record_bytes(int d);
int skge_pipe_runner_dp_begin(skge_pipe_runner_t *r, void *stream);
int skge_pipe_runner_dp_batch(skge_pipe_runner_t *r, void *stream, int b, int lo, int hi,
                              void *rec_out, int fold);
int skge_pipe_runner_dp_scatter(skge_pipe_runner_t *r, void *stream, int b, const void *recs,
                                int lo, int hi);
int skge_pipe_runner_dp_end(skge_pipe_runner_t *r, void *stream);

/* ---------------- row-sharded TransE-L1 step ----------------
 *
 * The entity table split by row over G ranks (rank g owns rows r % G == g at
 * local index r / G), the relation table replicated.  One mini-batch of
 * PairwiseStochasticTrainer (skge/base.py:1394-1427, TransE._pairwise_gradients
 * skge/transe.py:48-165, AdaGrad + normalize skge/param.py:140-167) over the
 * union of every rank's positives is, on each rank:
 *   skge_shard_route   -> exchange request ids (all-to-all) ->
 *   skge_shard_gather  -> exchange rows back (all-to-all) ->
 *   skge_shard_score   -> exchange contributions (all-to-all) ->
 *   skge_shard_accum   -> all-reduce the relation sums and counts ->
 *   skge_accum_apply({entity shard: nslots = requests received}, {rel: dense}).
 * The exchanges belong to the caller (RCCL via torch.distributed).  All sums
 * are exact integers, so the result equals one GPU's step on the union batch
 * bit for bit.  Positives come from skge_epoch_sample records (rec, rec_n1).
 */

/* Bucket the requests (s, o, s', o') of positives [start, start+count) by
 * owner: send_ids [4*count] (owner-major, request order within a bucket),
 * req_pos [4*count] = slot of request 4j+k in send_ids (-1: skipped negative),
 * counts [G] int64 = bucket sizes.  G <= 64. */
size_t skge_shard_route_workspace_bytes(int count, int G);
int skge_shard_route(void *stream, const int *rec, const int *rec_n1, int64_t start, int count,
                     int G, int *send_ids, int *req_pos, long long *counts, void *workspace,
                     size_t ws_bytes);
/* The fixed-capacity layout of the graph-capturable step (no host-side split
 * sizes): send_ids [G][C] = bucket g holds the requests owned by rank g in
 * request order, unused slots -1 (the all-to-alls then move G equal slices);
 * req_pos [4*count] = bucket slot of request 4j+k (-1: skipped negative).  A
 * bucket needing more than C slots sets *err |= 1 (its requests are dropped:
 * the caller must check *err).  The consumers below skip ids < 0. */
int skge_shard_route_cap(void *stream, const int *rec, const int *rec_n1, int64_t start,
                         int count, int G, int C, int *send_ids, int *req_pos, void *workspace,
                         size_t ws_bytes, int *err);
/* Owner side: rows_out[i] = E_shard[ids[i] / G] for i < n ([n][d] fp32;
 * ids[i] < 0: nothing written). */
int skge_shard_gather(void *stream, const float *E_shard, int d, int G, const int *ids, int64_t n,
                      float *rows_out);
/* Contribution record of one request: int32 count, pad to 16 B, int8[d]. */
long long skge_shard_contrib_stride(int d);
/* Requester side: score both pairs of every positive from the fetched rows
 * (fetched[req_pos[4j+k]]) and rel (dense packed accumulator, replicated
 * table), apply the strict margin test, write one contribution record per
 * request into contrib [n_send][stride] and add the relation contributions
 * into rel's accumulator; violations into the 64 sharded counters vshards
 * (64 x 32 ints, folded by skge_shard_fold_violations). */
int skge_shard_score(void *stream, const skge_table_t *rel, int d, const int *rec,
                     const int *rec_n1, int64_t start, int count, const float *fetched,
                     const int *req_pos, float margin, void *contrib, int *vshards);
/* Owner side: add the n received records into ent_shard's packed sums (local
 * row ids[i] / G), touched slot i per record (-1 for ids[i] < 0); touched_cap >= n. */
int skge_shard_accum(void *stream, const skge_table_t *ent_shard, int G, const int *ids,
                     const void *contrib, int64_t n);
/* *nviol_total += the violation shards, which are cleared. */
int skge_shard_fold_violations(void *stream, int *vshards, int *nviol_total);

/* ---------------- measurement ----------------
 *
 * Measured gather + RMW-scatter roofline: one launch of the same row traffic
 * as a training launch without its dependencies.  n_rmw waves each read and
 * write back one random row of P, A (fp32 [rows][d]) and S (packed sums,
 * u64 [rows][d/4]) = 20d bytes; then n_gather waves each gather
 * rows_per_wave random rows of P (4d bytes each) and add atom_rows_per_wave
 * rows of 64-bit atomics into S (2d bytes each).  out [n_gather] receives a
 * per-wave checksum.  The values of P, A, S are left unchanged.  Not part of
 * the training path (bench.py times it beside the training kernels). */
int skge_roofline_gather(void *stream, float *P, float *A, void *S, int rows, int d, int n_gather,
                         int rows_per_wave, int atom_rows_per_wave, int n_rmw, uint32_t salt,
                         float *out);
/* Hand-off latency probe: the pipelined runner's publish / wait form (16-B
 * write-through payload, drain, write-through flag; the waiter polls the flag
 * and re-reads the payload with write-through loads) ping-ponged `rounds`
 * times between two workgroups.  buf: >= 1024 device bytes (zeroed here);
 * out [3] (device u64): out[0] = 10-ns ticks for all rounds (two hops each),
 * out[1] = payload mismatches (0 expected), out[2] = 1 if a bounded wait gave
 * up.  Lets a bench line say how slow this box's hand-offs are. */
int skge_handoff_probe(void *stream, void *buf, int rounds, uint64_t *out);

/* ---------------- evaluation ---------------- */

/*
 * Filtered link-prediction ranks: FilteredRankingEval.positions
 * (skge/base.py:913-1031) with TransEEval (skge/run_transe.py:15-29; the L1
 * distance for either norm, as there) or HolEEval (skge/run_hole.py:12-19);
 * RESCAL scores E_s W_p E_o the same way.  For each test triple i = (s, o, p)
 * of queries[nq][3]: ranks_out[4i..4i+3] = tail rank of o given (s, p) raw and
 * filtered, head rank of s given (o, p) raw and filtered, where rank = 1 +
 * #entities scoring strictly higher (ties in the true entity's favour) and
 * the filtered count skips entities forming a known triple (set: a triple set
 * built by skge_triple_set_build over the known triples; NULL = no filter).
 * E [N][d], R [M][d] (W [M][d][d] for RESCAL), d <= 1024; workspace of
 * skge_rank_workspace_bytes(nq, d) bytes.
 */
size_t skge_rank_workspace_bytes(int nq, int d);
/*
 * skge_rank with the filter given as each query's KNOWN ANSWERS instead of a
 * triple set: tail_ent[tail_off[i] .. tail_off[i+1]) = every o' != o with
 * (s, o', p) known, head_ent[head_off[i] .. head_off[i+1]) = every s' != s
 * with (s', o, p) known (int32, offsets nq + 1).  rank_filtered = rank_raw -
 * #{those answers scoring strictly above the true entity}: the same positions
 * as skge_rank, with no triple-set lookups in the all-entity pass (which also
 * spreads each query block over entity slices).  Workspace:
 * skge_rank_known_workspace_bytes(nq, d).
 */
size_t skge_rank_known_workspace_bytes(int nq, int d);
int skge_rank_known(void *stream, int model, const float *E, const float *R, int N, int d,
                    const int *queries, int nq, const int *tail_off, const int *tail_ent,
                    const int *head_off, const int *head_ent, void *workspace, size_t ws_bytes,
                    int *ranks_out);
int skge_rank(void *stream, int model, const float *E, const float *R, int N, int d,
              const int *queries, int nq, const void *set, int64_t set_capacity,
              void *workspace, size_t ws_bytes, int *ranks_out);

#ifdef __cplusplus
}
#endif
#endif /* SKGE_HIP_H */
