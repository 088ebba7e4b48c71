// RESCAL pairwise training step on the matrix cores (fp32 MFMA).
//
// The reference scores and differentiates RESCAL one pair at a time with
// GEMVs against the pair's d x d relation matrix (skge/rescal.py:78-139):
// per pair W[p] E[o] and E[s] W[p] for the positive and the negative, and per
// relation the sum of outer products E[s] (x) E[o] for dW.  Reading W[p]
// (160 KB at d=200) once per GEMV makes that path L2-bound.  Here the batch's
// triples (positives and negatives) are grouped by relation, and per relation
// the three contractions become small GEMMs on v_mfma_f32_16x16x4_f32 (exact
// fp32: a k-ordered fmaf chain, MI355X_MICROARCH.md "Matrix cores"):
//   WE^T = E_o W[p]^T      [items x d]   (WE_i = W[p] E[o_i],  rescal.py:261)
//   EW   = E_s W[p]        [items x d]   (EW_i = E[s_i] W[p],  rescal.py:262)
//   dW[p] = E_s^T diag(coef) E_o  [d x d] (rescal.py:113-125, all pairs)
// with score_i = E[s_i] . WE_i.  Kernels:
//   k_rs_count/scan/scatter  stable counting sort of the 2P triples by
//                     relation (per-64-item-chunk ballot ranks), 16-item tiles
//   k_rescal_gemm     one workgroup per (64-triple tile, 64-column block,
//                     product): LDS-tiled, double-buffered fp32 MFMA GEMM;
//                     writes WE^T / EW rows and partial scores
//   k_rescal_scatter  one wave per pair: activation, strict margin test, the
//                     entity contributions (gp WE_p, gn WE_n over s; gp EW_p,
//                     gn EW_n over o) into the entity accumulator, coef
//   k_rescal_wgrad_mfma  one workgroup per (relation, 64x64 tile of dW[p]):
//                     the tile is applied to W[p] in place by its owner (the
//                     W updater) or written with plain stores
// Scores, WE, EW and dW have fixed summation orders (stable buckets, fixed
// MFMA k order, fixed cross-wave reduction order), so the relation gradient
// is bitwise reproducible; the entity sums use float atomics, as elsewhere.
#include <string>

#include "skge_host.h"

namespace skge {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int RT_ITEMS = 64;    // triples per GEMM tile
constexpr int GC = 64;          // output columns per GEMM tile
#ifndef SKGE_RS_KS
#define SKGE_RS_KS 32
#endif
#ifndef SKGE_RS_GKS_DEFAULT
#define SKGE_RS_GKS_DEFAULT 1   // A/B: SKGE_RS_GKS
#endif
constexpr int KS = SKGE_RS_KS;  // k per staged step
// the fused front's k-step below RS_KS_SMALL_BS positives per batch (k order
// unchanged: the same bits); WN18 d = 200, same box: nb = 100 KS 16 / 32 / 64
// -> 36.3 / 35.8 / 26.8 M triples/s, nb = 2 KS 16 / 32 -> 70.1 / 72.5 M
// (profiles/r06/ab_rescal_ks.txt)
constexpr int KS_SMALL = 16, RS_KS_SMALL_BS = 8192;
constexpr int RS_MAX_D = 1024;  // d of the MFMA path
constexpr int RS_MAX_M = 8192;  // relations (k_rs_scan keeps 2M+1 ints in LDS)

static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct RescalWs {
  int* chunk;       // [nchunks][M] per-chunk counts, then offsets
  int* rel_off;     // [M+1]
  int* items;       // [n] triple ids grouped by relation, stable
  int* tile_rel;    // [tmax]
  int* tile_start;  // [tmax]
  int* tile_cnt;    // [tmax]
  int* ntiles;      // [1]
  int* sorted_s;    // [n] E row of s / o of items[i] (bucket order)
  int* sorted_o;
  int* bpos;        // [n] bucket position of triple k (items[bpos[k]] == k)
  float* spart;     // [n][ceil(d/64)] partial scores of the WE column blocks
  float* coef;      // [n] dW coefficient of items[i] (bucket order)
  float* WE;        // [n][d]
  float* EW;        // [n][d]
  float* wpart;     // [M][nt * nt][splits][64 * 64] split-K dW partial tiles (or null)
  float* ecoef;     // [n] Linear dW coefficients in bucket order, written with the
                    // epoch's buckets (device pair loop only, else null)
  // deduplicated GEMM rows (epoch buckets; npos = the batch's positives, 0 =
  // off): a positive j and its s-corrupted negative share W E_o, j and its
  // o-corrupted negative share E_s W, so product 0 (WE) runs over the
  // positives and the o-corrupted negatives, product 1 (EW) over the
  // positives and the s-corrupted negatives -- 2 rows per positive each
  // instead of 3 -- and a positive's WE row also gives its s-corrupted
  // negative's partial scores (s2: that negative's s' row, bucket order)
  int* s2;
  int npos;
  // deduplicated buckets, combined dW (fused front): a positive's items enter
  // dW as ONE outer product E_s (x) (ecoef E_o + E_o') -- its o-corrupted
  // negative folded in (o2: that negative's o' row, or -1) -- so dW runs over
  // product 1's rows, n01[p] items of relation p from rel_off[p]
  int* o2;
  int* n01;
  // the in-front W step's second W / state buffer and the current-buffer
  // word (WStep::cur; epoch buckets, or null)
  float* W1;
  float* A1;
  int* wcur;
  // the batch's entity rows grouped (epoch buckets: k_rs_rows_ep; else null):
  // a distinct row's slots in slot order, two per work item -- urec[w] = (row,
  // slot a, slot b or -1, chunk << 16 | chunks of the row), a row's chunks
  // consecutive, row -1 past the last item; a slot packed as j << 4 | k1 << 3
  // | k0 << 2 | role (positive j, role 0-3 = s, o, s', o'; k0 / k1: its
  // negatives exist); rowctr[w0]: arrivals of a multi-chunk row's items (w0
  // its first); nuniq: distinct rows; vword: k_rescal_fold's violation count
  // (low half) and arrivals (high half); all zeroed with the grouping.
  // part / pcnt (shared by the batches): a multi-chunk item's partial sum and
  // count
  int4* urec;
  int* rowctr;
  int* nuniq;
  unsigned long long* vword;
  float* part;
  int* pcnt;
  // GEMM K split (SKGE_RS_GKS, 1 = off): the WE / EW rows and partial scores
  // come in gks slices over k, slice k at WE + k * part_stride (spart + k *
  // spart_stride); consumers add the slices in index order (deterministic)
  int gks;
  long long part_stride, spart_stride;
};

// WE / EW row i of the batch: the K slices summed in slice order
template <int KM>
__device__ __forceinline__ void load_row_gk(const float* __restrict__ base, const RescalWs& ws,
                                            int i, int d, float (&v)[KM]) {
  load_row<KM>(base, i, d, v);
  if (ws.gks > 1) {
    float u[KM];
    load_row<KM>(base + ws.part_stride, i, d, u);
#pragma unroll
    for (int k = 0; k < KM; ++k) v[k] += u[k];
  }
}
// the raw score of item i: the column blocks' partial scores (and their K
// slices) in a fixed order
__device__ __forceinline__ float spart_sum(const RescalWs& ws, int i, int ncb) {
  float r = 0.0f;
  for (int q = 0; q < ncb; ++q) {
    r += ws.spart[(size_t)i * ncb + q];
    if (ws.gks > 1) r += ws.spart[ws.spart_stride + (size_t)i * ncb + q];
  }
  return r;
}

// Test forms of the RESCAL path (SKGE_RESCAL_FORM, comma-separated tokens;
// unset = the default, measured-best form).  Each token selects the simpler
// form a GPU test compares the default against on the same draws
// (tests/test_gpu_pairloop.py): "unfused" (no fused front), "nosplit" (one dW
// kernel, no split-K partial tiles), "nodedup" (three GEMM rows per positive),
// "dw3" (three dW items per positive), "wapply" (the W step in the entity
// apply's launch), "fsplit=N" (dW splits of the fused front), "order=N" (the
// front's role order: 0 dW first, 1 GEMM first, >= 2 interleaved),
// "scatter" (the entity sums by the scatter kernel's atomics and the apply
// launch, instead of the row-grouped apply k_rescal_fold).  The
// round-5 A/B-only switches (GEMM K split, the W step in its own launch) are
// compile-time only now (SKGE_RS_GKS_DEFAULT).
struct RsForm {
  bool unfused = false, nosplit = false, nodedup = false, dw3 = false, wapply = false,
       scatter = false;
  int fsplit = 1, order = 1;
};
static RsForm rs_form() {
  RsForm f;
  const char* e = getenv("SKGE_RESCAL_FORM");
  if (!e) return f;
  std::string v(e);
  size_t i = 0;
  while (i <= v.size()) {
    size_t j = v.find(',', i);
    if (j == std::string::npos) j = v.size();
    const std::string t = v.substr(i, j - i);
    if (t == "unfused") f.unfused = true;
    else if (t == "nosplit") f.nosplit = true;
    else if (t == "nodedup") f.nodedup = true;
    else if (t == "dw3") f.dw3 = true;
    else if (t == "wapply") f.wapply = true;
    else if (t == "scatter") f.scatter = true;
    else if (t.rfind("fsplit=", 0) == 0) f.fsplit = std::max(1, atoi(t.c_str() + 7));
    else if (t.rfind("order=", 0) == 0) f.order = std::max(0, atoi(t.c_str() + 6));
    i = j + 1;
  }
  return f;
}

// K slices of the GEMMs (SKGE_RS_GKS_DEFAULT: 1 or 2; d needs at least 2
// k-steps; the split measured 34 -> 26 M triples/s, so 1)
static int rs_gks(int d) {
  const int g = SKGE_RS_GKS_DEFAULT;
  return g >= 2 && (d + SKGE_RS_KS - 1) / SKGE_RS_KS >= 2 ? 2 : 1;
}

// the fused front's in-front W step (WStep::cur): W_b is in buffer *cur
// (0: W0 / A0 = the caller's); the dW workgroups write W_{b+1} into the other
struct WFront {
  const int* cur;   // nullptr: off
  float* W0;
  float* A0;
  float* W1;
  float* A1;
  int opt;
  float lr, rin, rout, fdiv;
};

static int rs_tmax(int n, int M) { return n / RT_ITEMS + M + 1; }
// deduplicated GEMM rows (RescalWs::npos): 2M segments of 2P rows in all
static int rs_tmax_dedup(int P, int M) { return 4 * P / RT_ITEMS + 2 * M + 1; }
// the device pair loop's epoch buckets deduplicate the GEMM rows
// (SKGE_RESCAL_FORM=nodedup: three rows per positive)
static bool rs_dedup_on() { return !rs_form().nodedup; }

// dW split over K (a relation's items): at the reference's batch size a
// relation holds ~235 items, which one workgroup per 64 x 64 dW tile walks in
// two dependent rounds of gathers; `splits` workgroups per tile take every
// splits-th group of 128 items each and write partial tiles, summed in split
// order (deterministic) by the finishing kernel.  1 = the single fused kernel.
#ifndef SKGE_RS_WG_SPLIT
#define SKGE_RS_WG_SPLIT 8   // most splits per tile (1 disables)
#endif
constexpr int WS_TILE = 64;                 // == WG_T below
#ifndef SKGE_RS_WG_PF
// chunks of 64 items loaded together in the dW tiles; A/B on WN18 d=200: round
// 1 1 group of 4 chunks 20.5M, 2 chunks 24.2M; round 6 (fused front, config 4,
// profiles/r06/ab_rescal_dw_prefetch.txt) 1 / 2 / 4 -> 30.7 / 36.2 / 23.5 M
#define SKGE_RS_WG_PF 2
#endif
constexpr int WS_GROUP = SKGE_RS_WG_PF * 64;   // items per group == WG_PF * WG_CH below
static int rs_wsplit(int n, int M, int d) {
  const long long nt = (d + WS_TILE - 1) / WS_TILE;
  // (at the reference's batch, ~2 groups per relation, the extra launch costs
  // more than the split saves: 22.5 M vs 24.1 M triples/s on WN18 d = 200;
  // nb = 2, ~92 groups: 52.5 M vs 42.0 M)
  const long long groups = ((long long)n / M + WS_GROUP - 1) / WS_GROUP;
  int sp = groups < 4 ? 1 : (int)std::min<long long>(SKGE_RS_WG_SPLIT, groups);
  if (rs_form().nosplit) sp = 1;   // test form: the fused kernel only
  while (sp > 1 && (long long)M * nt * nt * sp * WS_TILE * WS_TILE * 4 > (64ll << 20)) --sp;
  return std::max(sp, 1);
}
static size_t rs_wpart_bytes(int n, int M, int d) {
  const int sp = rs_wsplit(n, M, d);
  const size_t nt = (d + WS_TILE - 1) / WS_TILE;
  return sp > 1 ? (size_t)M * nt * nt * sp * WS_TILE * WS_TILE * 4 : 0;
}
// the fused front (k_rescal_front_fused): splits of its dW grid -- the split-K
// count where that applies, else the form's fsplit (default 1; each split adds
// a workgroup per tile beside the GEMM's); 0 = no fused front (form "unfused",
// or the partial tiles would pass 64 MB)
static int rs_front_splits(int n, int M, int d) {
  const RsForm f = rs_form();
  if (f.unfused) return 0;
  const long long nt = (d + WS_TILE - 1) / WS_TILE;
  int sp = rs_wsplit(n, M, d);
  if (sp == 1) {
    sp = f.fsplit;
    const long long groups = ((long long)n / M + WS_GROUP - 1) / WS_GROUP;
    sp = (int)std::max(1ll, std::min<long long>(sp, groups));
  }
  if ((long long)M * nt * nt * sp * WS_TILE * WS_TILE * 4 > (64ll << 20)) return 0;
  return sp;
}
static size_t rs_front_wpart_bytes(int n, int M, int d) {
  const size_t nt = (d + WS_TILE - 1) / WS_TILE;
  return (size_t)M * nt * nt * rs_front_splits(n, M, d) * WS_TILE * WS_TILE * 4;
}

// carve the workspace (base may be null: size only)
// n: triples in the batch (2P for pairs: positives then negatives; T for
// labelled triples)
static size_t rescal_ws_layout(int n, int M, int d, void* base, RescalWs* ws) {
  const int nchunks = (n + 63) / 64, tmax = rs_tmax(n, M);
  size_t off = 0;
  char* b = (char*)base;
  auto take = [&](size_t bytes) {
    char* p = b ? b + off : nullptr;
    off += al256(bytes);
    return p;
  };
  RescalWs w;
  w.chunk = (int*)take((size_t)nchunks * M * 4);
  w.rel_off = (int*)take((size_t)(M + 1) * 4);
  w.items = (int*)take((size_t)n * 4);
  w.tile_rel = (int*)take((size_t)tmax * 4);
  w.tile_start = (int*)take((size_t)tmax * 4);
  w.tile_cnt = (int*)take((size_t)tmax * 4);
  w.ntiles = (int*)take(4);
  w.sorted_s = (int*)take((size_t)n * 4);
  w.sorted_o = (int*)take((size_t)n * 4);
  w.bpos = (int*)take((size_t)n * 4);
  const int gks = rs_gks(d);
  w.gks = gks;
  w.part_stride = (long long)n * d;
  w.spart_stride = (long long)n * ((d + GC - 1) / GC);
  w.spart = (float*)take((size_t)gks * n * ((d + GC - 1) / GC) * 4);
  w.coef = (float*)take((size_t)n * 4);
  w.WE = (float*)take((size_t)gks * n * d * 4);
  w.EW = (float*)take((size_t)gks * n * d * 4);
  const size_t wpb = rs_wpart_bytes(n, M, d);
  w.wpart = wpb ? (float*)take(wpb) : nullptr;
  w.ecoef = nullptr;
  w.s2 = nullptr;
  w.npos = 0;
  w.o2 = nullptr;
  w.n01 = nullptr;
  w.W1 = w.A1 = nullptr;
  w.wcur = nullptr;
  w.urec = nullptr;
  w.rowctr = w.nuniq = nullptr;
  w.vword = nullptr;
  w.part = nullptr;
  w.pcnt = nullptr;
  if (ws) *ws = w;
  return off;
}

// triple k of the batch: list a (na triples: the positives), then list b
__device__ __forceinline__ const int* item_trip(const int* a, const int* b, int na, int k) {
  return k < na ? a + 3 * (size_t)k : b + 3 * (size_t)(k - na);
}

// ---------------------------------------------------------------------------
// stable counting sort by relation, in three small launches:
//   k_rs_count    one wave per 64-triple chunk: per-relation counts (ballot
//                 "match" loop; the table is zeroed by a memset before)
//   k_rs_scan     one workgroup: per relation, wave-parallel exclusive scan
//                 over the chunks; relation offsets; the 16-triple tile list
//   k_rs_scatter  one wave per chunk: ranks again, writes the grouped lists
// ---------------------------------------------------------------------------
__device__ __forceinline__ int wave_incl_scan(int v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o, 64);
    if (l >= o) v += t;
  }
  return v;
}

// item of enumeration position u (-1: none).  Plain: u itself.  Deduplicated
// epoch buckets (ws.npos == P > 0): three blocks of cpad = P rounded up to 64
// -- the s-corrupted negatives (item P + 2j), the positives (j), the
// o-corrupted negatives (P + 2j + 1) -- so every relation's stable bucket is
// [s-corrupted | positives | o-corrupted]: product 1's rows (the first two
// parts) and product 0's (the last two) are contiguous, and the blocks start
// on chunk boundaries (their per-relation offsets are chunk prefixes)
__device__ __forceinline__ int rs_item(int u, int P, int n, bool dedup) {
  if (!dedup) return u < n ? u : -1;
  const int cpad = (P + 63) & ~63;
  const int blk = u >= 2 * cpad ? 2 : (u >= cpad ? 1 : 0), j = u - blk * cpad;
  if (j >= P) return -1;
  return blk == 1 ? j : P + 2 * j + (blk == 2 ? 1 : 0);
}
__device__ __forceinline__ int rs_nchunks(int P, int n, bool dedup) {
  return dedup ? 3 * (((P + 63) & ~63) >> 6) : (n + 63) / 64;
}

__device__ __forceinline__ void rs_count_chunk(const int* __restrict__ pos,
                                               const int* __restrict__ neg, int P, int n, int M,
                                               const RescalWs& ws, int c) {
  const int l = lane_id();
  const int k = rs_item(c * 64 + l, P, n, ws.npos > 0);
  const int b = k >= 0 ? item_trip(pos, neg, P, k)[2] : -1;
  if (M <= 64) {   // lane p owns relation p: the whole row is written, no memset
    int mine = 0;
    for (int p = 0; p < M; ++p) {
      const int cp = __popcll(__ballot(b == p));
      if (l == p) mine = cp;
    }
    if (l < M) ws.chunk[(size_t)c * M + l] = mine;
    return;
  }
  uint64_t act = __ballot(b >= 0);   // the table was zeroed by a memset
  while (act) {
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int bl = __builtin_amdgcn_readlane(b, leader);
    const uint64_t m = __ballot(b == bl) & act;
    if (l == leader) ws.chunk[(size_t)c * M + bl] = __popcll(m);
    act &= ~m;
  }
}

__global__ __launch_bounds__(256) void k_rs_count(const int* __restrict__ pos,
                                                  const int* __restrict__ neg, int P, int n,
                                                  int M, RescalWs ws) {
  const int nchunks = (n + 63) / 64;
  const int c = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  rs_count_chunk(pos, neg, P, n, M, ws, c);
}

__device__ __forceinline__ void rs_scan_body(int n, int M, const RescalWs& ws, int* lds) {
  int* cnt = lds;   // cnt[M], tile_base[M+1] (deduplicated: then 2M segment starts, 2M
  int* tbase = lds + M;   // lengths, 2M + 1 segment tile bases)
  const bool dedup = ws.npos > 0;
  const int nchunks = rs_nchunks(ws.npos, n, dedup);
  const int tid = threadIdx.x, l = lane_id(), wave = tid >> 6, nw = blockDim.x >> 6;
  for (int p = wave; p < M; p += nw) {   // exclusive scan of relation p over the chunks
    int carry = 0;
    for (int c0 = 0; c0 < nchunks; c0 += 64) {
      const int c = c0 + l;
      const int v = c < nchunks ? ws.chunk[(size_t)c * M + p] : 0;
      const int inc = wave_incl_scan(v);
      if (c < nchunks) ws.chunk[(size_t)c * M + p] = carry + inc - v;
      carry += __shfl(inc, 63, 64);
    }
    if (l == 0) cnt[p] = carry;
  }
  __syncthreads();
  if (wave == 0) {   // relation offsets and tile bases (exclusive scans over p)
    int off = 0, toff = 0;
    for (int p0 = 0; p0 < M; p0 += 64) {
      const int p = p0 + l;
      const int v = p < M ? cnt[p] : 0, tv = (v + RT_ITEMS - 1) / RT_ITEMS;
      const int inc = wave_incl_scan(v), tinc = wave_incl_scan(tv);
      if (p < M) {
        ws.rel_off[p] = off + inc - v;
        tbase[p] = toff + tinc - tv;
      }
      off += __shfl(inc, 63, 64);
      toff += __shfl(tinc, 63, 64);
    }
    if (l == 0) {
      ws.rel_off[M] = off;
      tbase[M] = toff;
      *ws.ntiles = toff;
    }
  }
  __syncthreads();
  if (dedup) {   // 2M GEMM segments: product 0 of relation g, then product 1 of g - M
    int* sst = lds + 2 * M + 1;
    int* sln = sst + 2 * M;
    int* sb = sln + 2 * M;
    const int cpc = ((ws.npos + 63) & ~63) >> 6;   // chunks per enumeration block
    for (int p = tid; p < M; p += blockDim.x) {
      const int r0 = ws.rel_off[p];
      const int n0 = ws.chunk[(size_t)cpc * M + p];       // s-corrupted negatives of p
      const int n01 = ws.chunk[(size_t)2 * cpc * M + p];  // ... and its positives
      sst[p] = r0 + n0;           // product 0: positives, o-corrupted negatives
      sln[p] = cnt[p] - n0;
      sst[M + p] = r0;            // product 1: s-corrupted negatives, positives
      sln[M + p] = n01;
      ws.n01[p] = n01;            // (the combined dW's items)
    }
    __syncthreads();
    if (wave == 0) {
      int toff = 0;
      for (int g0 = 0; g0 < 2 * M; g0 += 64) {
        const int g = g0 + l;
        const int tv = g < 2 * M ? (sln[g] + RT_ITEMS - 1) / RT_ITEMS : 0;
        const int tinc = wave_incl_scan(tv);
        if (g < 2 * M) sb[g] = toff + tinc - tv;
        toff += __shfl(tinc, 63, 64);
      }
      if (l == 0) {
        sb[2 * M] = toff;
        ws.ntiles[0] = toff;
        ws.ntiles[1] = sb[M];   // product-0 tiles come first
      }
    }
    __syncthreads();
    const int nt2 = sb[2 * M];
    for (int t = tid; t < nt2; t += blockDim.x) {
      int lo = 0, hi = 2 * M - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (sb[mid] <= t) lo = mid; else hi = mid - 1;
      }
      const int g = lo, s = (t - sb[g]) * RT_ITEMS;
      ws.tile_rel[t] = g < M ? g : g - M;
      ws.tile_start[t] = sst[g] + s;
      ws.tile_cnt[t] = min(RT_ITEMS, sln[g] - s);
    }
    return;
  }
  const int nt = tbase[M];
  for (int t = tid; t < nt; t += blockDim.x) {   // tile t: relation p with tbase[p] <= t
    int lo = 0, hi = M - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tbase[mid] <= t) lo = mid; else hi = mid - 1;
    }
    const int p = lo, s = (t - tbase[p]) * RT_ITEMS;
    int off = 0;   // rel_off[p] again: prefix of cnt (cheap: read back)
    off = ws.rel_off[p];
    ws.tile_rel[t] = p;
    ws.tile_start[t] = off + s;
    ws.tile_cnt[t] = min(RT_ITEMS, cnt[p] - s);
  }
}

__global__ __launch_bounds__(1024) void k_rs_scan(int n, int M, RescalWs ws) {
  extern __shared__ int lds[];
  rs_scan_body(n, M, ws, lds);
}

__device__ __forceinline__ void rs_scatter_chunk(const int* __restrict__ pos,
                                                 const int* __restrict__ neg, int P, int n, int M,
                                                 const RescalWs& ws, int c) {
  const int l = lane_id();
  const int k = rs_item(c * 64 + l, P, n, ws.npos > 0);
  const int* tr = item_trip(pos, neg, P, k >= 0 ? k : 0);
  const int ts = tr[0], to = tr[1], b = k >= 0 ? tr[2] : -1;
  // deduplicated: a positive's s-corrupted negative's s' row (or -1)
  const int ts2 = (ws.npos > 0 && k >= 0 && k < P && neg[6 * (size_t)k + 2] >= 0)
                      ? neg[6 * (size_t)k] : -1;
  // ... and its o-corrupted negative's o' row (or -1)
  const int to2 = (ws.npos > 0 && k >= 0 && k < P && neg[6 * (size_t)k + 5] >= 0)
                      ? neg[6 * (size_t)k + 4] : -1;
  // epoch buckets (dedup lists: positive j's negatives at neg[6j .. 6j + 5]):
  // the Linear dW coefficient, gp (k0 + k1) = -(k0 + k1) for a positive and
  // gn = +1 for a negative, as k_rescal_pos_scatter computes it
  float ec = 1.0f;
  if (ws.ecoef && k >= 0 && k < P)
    ec = -(float)((neg[6 * (size_t)k + 2] >= 0 ? 1 : 0) + (neg[6 * (size_t)k + 5] >= 0 ? 1 : 0));
  uint64_t act = __ballot(b >= 0);
  while (act) {
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int bl = __builtin_amdgcn_readlane(b, leader);
    const uint64_t m = __ballot(b == bl) & act;
    if (b == bl) {
      const int at = ws.rel_off[bl] + ws.chunk[(size_t)c * M + bl] +
                     __popcll(m & ((1ull << l) - 1ull));
      ws.items[at] = k;
      ws.sorted_s[at] = ts;
      ws.sorted_o[at] = to;
      ws.bpos[k] = at;
      if (ws.ecoef) ws.ecoef[at] = ec;
      if (ws.npos > 0) {
        ws.s2[at] = ts2;
        ws.o2[at] = to2;
      }
    }
    act &= ~m;
  }
}

__global__ __launch_bounds__(256) void k_rs_scatter(const int* __restrict__ pos,
                                                    const int* __restrict__ neg, int P, int n,
                                                    int M, RescalWs ws) {
  const int nchunks = (n + 63) / 64;
  const int c = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  rs_scatter_chunk(pos, neg, P, n, M, ws, c);
}

// ---- the whole epoch's buckets at once (device pair loop, M <= 64) ----
// The epoch's items do not depend on the parameters (k_pairs_of_epoch), so
// every batch's stable relation buckets are built by three launches per
// EPOCH instead of three per batch.  Batch b (np.split geometry: bs positives,
// the last batch the remainder) is items [0, 3 count_b) of its dedup lists;
// its bucket arrays live in its own slice of the workspace (RescalEpoch).
struct RescalEpoch {
  RescalWs ws0;          // batch 0's view (the shared WE / EW / spart / coef included)
  long long stride;      // bytes between consecutive batches' bucket slices
  long long T;
  int bs, nb, M, cpb;    // cpb: 64-item chunks of a full batch
  int dedup;             // deduplicated GEMM rows (RescalWs::npos)
};

__device__ __forceinline__ int rs_batch_count(const RescalEpoch& e, int b) {
  const long long s0 = (long long)b * e.bs;
  return (int)(s0 + e.bs <= e.T ? e.bs : e.T - s0);
}

__device__ __forceinline__ RescalWs rs_batch_view(const RescalEpoch& e, int b) {
  RescalWs w = e.ws0;
  const long long o = e.stride * b;
  auto sh = [o](auto* p) { return reinterpret_cast<decltype(p)>(reinterpret_cast<char*>(p) + o); };
  w.chunk = sh(w.chunk);
  w.rel_off = sh(w.rel_off);
  w.items = sh(w.items);
  w.tile_rel = sh(w.tile_rel);
  w.tile_start = sh(w.tile_start);
  w.tile_cnt = sh(w.tile_cnt);
  w.ntiles = sh(w.ntiles);
  w.sorted_s = sh(w.sorted_s);
  w.sorted_o = sh(w.sorted_o);
  w.bpos = sh(w.bpos);
  w.ecoef = sh(w.ecoef);
  w.s2 = sh(w.s2);
  w.o2 = sh(w.o2);
  w.n01 = sh(w.n01);
  w.urec = sh(w.urec);
  w.rowctr = sh(w.rowctr);
  w.nuniq = sh(w.nuniq);
  w.vword = sh(w.vword);
  w.npos = e.dedup ? rs_batch_count(e, b) : 0;
  return w;
}

__global__ __launch_bounds__(256) void k_rs_count_ep(const int* __restrict__ pos,
                                                     const int* __restrict__ neg, RescalEpoch e) {
  const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int b = gw / e.cpb, c = gw - b * e.cpb;
  if (b >= e.nb) return;
  const int cnt = rs_batch_count(e, b), n = 3 * cnt;
  if (c >= rs_nchunks(cnt, n, e.dedup != 0)) return;
  const long long s0 = (long long)b * e.bs;
  rs_count_chunk(pos + 3 * s0, neg + 6 * s0, cnt, n, e.M, rs_batch_view(e, b), c);
}

__global__ __launch_bounds__(1024) void k_rs_scan_ep(RescalEpoch e) {
  extern __shared__ int lds[];
  const int b = blockIdx.x;
  // the epoch starts with W in the caller's buffer (the in-front W step's word)
  if (e.ws0.wcur && b == 0 && threadIdx.x == 0) *e.ws0.wcur = 0;
  rs_scan_body(3 * rs_batch_count(e, b), e.M, rs_batch_view(e, b), lds);
}

__global__ __launch_bounds__(256) void k_rs_scatter_ep(const int* __restrict__ pos,
                                                       const int* __restrict__ neg,
                                                       RescalEpoch e) {
  const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int b = gw / e.cpb, c = gw - b * e.cpb;
  if (b >= e.nb) return;
  const int cnt = rs_batch_count(e, b), n = 3 * cnt;
  if (c >= rs_nchunks(cnt, n, e.dedup != 0)) return;
  const long long s0 = (long long)b * e.bs;
  rs_scatter_chunk(pos + 3 * s0, neg + 6 * s0, cnt, n, e.M, rs_batch_view(e, b), c);
}

// The row grouping of every batch's entity slots, once per epoch (the
// records are drawn at the epoch's start): one workgroup per batch inserts
// the batch's 4 count slots' rows into an LDS hash table (linear probing),
// ranks each slot within its row (LDS atomics), compacts the table into the
// distinct rows' slot ranges, sorts each range by slot (the order, hence
// every sum, is fixed) and writes the work items k_rescal_fold reads instead
// of the scatter's atomics: two slots per item, a row of n slots as
// ceil(n / 2) consecutive items (one or two slots per row at WN18's batch;
// hub rows of skewed KGs get many, merged by their last item).
constexpr int RS_ROWS_MAX = 8192;   // hash entries = slots per batch at most (bs <= 2048)
__global__ __launch_bounds__(1024) void k_rs_rows_ep(const int4* __restrict__ rec,
                                                     const int* __restrict__ rec_n1,
                                                     RescalEpoch e) {
  __shared__ int hkey[RS_ROWS_MAX];   // row of the entry, or -1
  __shared__ int hcnt[RS_ROWS_MAX];   // its slots; after the compaction: its first position
  __shared__ int sl[RS_ROWS_MAX];     // the slots, grouped by row
  __shared__ int wt_u[16], wt_n[16], wt_r[16];
  constexpr int PER = RS_ROWS_MAX / 1024;   // entries and slots per thread
  const int b = blockIdx.x, tid = threadIdx.x, l = lane_id(), wave = tid >> 6;
  const int cnt = rs_batch_count(e, b), ns = 4 * cnt;
  const long long s0 = (long long)b * e.bs;
  const RescalWs w = rs_batch_view(e, b);
  for (int i = tid; i < RS_ROWS_MAX; i += 1024) {
    hkey[i] = -1;
    hcnt[i] = 0;
  }
  __syncthreads();
  int he[PER], rk[PER], sv[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {   // slot i = tid + 1024 q
    const int i = tid + 1024 * q;
    he[q] = -1;
    if (i >= ns) continue;
    const int j = i >> 2, role = i & 3;
    const int4 r4 = rec[s0 + j];
    const int n1 = rec_n1[s0 + j];
    const int row = role == 0 ? r4.x : (role == 1 ? r4.y : (role == 2 ? r4.w : n1));
    if (row < 0) continue;
    sv[q] = (j << 4) | ((n1 >= 0 ? 1 : 0) << 3) | ((r4.w >= 0 ? 1 : 0) << 2) | role;
    int h = (int)(fmix32((uint32_t)row) & (RS_ROWS_MAX - 1));
    while (true) {   // distinct rows <= slots <= entries: a free entry always exists
      const int old = atomicCAS(&hkey[h], -1, row);
      if (old == -1 || old == row) break;
      h = (h + 1) & (RS_ROWS_MAX - 1);
    }
    he[q] = h;
    rk[q] = atomicAdd(&hcnt[h], 1);
  }
  __syncthreads();
  // compaction: thread t owns entries [PER t, PER t + PER); a row of n slots
  // becomes ceil(n / 2) work items
  int nw = 0, nsl = 0, nu = 0, c[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    c[q] = hcnt[PER * tid + q];
    nw += (c[q] + 1) >> 1;
    nsl += c[q];
    nu += hkey[PER * tid + q] >= 0 ? 1 : 0;
  }
  const int iw = wave_incl_scan(nw), in = wave_incl_scan(nsl), iu = wave_incl_scan(nu);
  if (l == 63) {
    wt_u[wave] = iw;
    wt_n[wave] = in;
    wt_r[wave] = iu;
  }
  __syncthreads();
  int w0 = iw - nw, off = in - nsl;
  for (int v = 0; v < wave; ++v) {
    w0 += wt_u[v];
    off += wt_n[v];
  }
  int ew[PER], eo[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    ew[q] = -1;
    eo[q] = off;
    if (hkey[PER * tid + q] >= 0) {
      ew[q] = w0;
      w0 += (c[q] + 1) >> 1;
      hcnt[PER * tid + q] = off;
    }
    off += c[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PER; ++q)
    if (he[q] >= 0) sl[hcnt[he[q]] + rk[q]] = sv[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PER; ++q) {   // each row's slots in slot order, then its work items
    if (ew[q] < 0) continue;
    const int o = eo[q], n = c[q], nch = (n + 1) >> 1, row = hkey[PER * tid + q];
    for (int a = o + 1; a < o + n; ++a) {   // insertion sort (n is small but for hub rows)
      const int x = sl[a];
      int z = a - 1;
      while (z >= o && sl[z] > x) {
        sl[z + 1] = sl[z];
        --z;
      }
      sl[z + 1] = x;
    }
    for (int k = 0; k < nch; ++k)
      w.urec[ew[q] + k] = make_int4(row, sl[o + 2 * k], 2 * k + 1 < n ? sl[o + 2 * k + 1] : -1,
                                   (k << 16) | nch);
    if (nch > 1) w.rowctr[ew[q]] = 0;
  }
  int tot = 0, rows = 0;
  for (int v = 0; v < 16; ++v) {
    tot += wt_u[v];
    rows += wt_r[v];
  }
  for (int i = tot + tid; i < ns; i += 1024)   // past the items: row -1 (k_rescal_fold exits)
    w.urec[i] = make_int4(-1, -1, -1, 0);
  if (tid == 0) {
    *w.nuniq = rows;
    *w.vword = 0ull;
  }
}

// Small batches (n <= SB_MAXN triples, M <= SB_MAXM relations): the same
// stable bucketing in ONE workgroup -- totals, scans and tile list, then the
// items in rounds of 1024 (wave-ordered ranks through LDS), so the batch
// pays one launch instead of a memset and three.
constexpr int SB_MAXM = 256;
constexpr int SB_ITEMS = 1;              // items per thread, held in registers
constexpr int SB_MAXN = 1024 * SB_ITEMS;

__global__ __launch_bounds__(1024) void k_rs_bucket_small(const int* __restrict__ pos,
                                                          const int* __restrict__ neg, int P,
                                                          int n, int M, RescalWs ws) {
  __shared__ int cw[16][SB_MAXM];   // per-wave counts of the current round
  __shared__ int cnt[SB_MAXM];      // relation totals
  __shared__ int base[SB_MAXM];     // next free position of each relation
  __shared__ int tbase[SB_MAXM + 1];
  const int tid = threadIdx.x, l = lane_id(), wave = tid >> 6;
  // every item of the batch is loaded once, up front (one memory round trip)
  int rs[SB_ITEMS], ss[SB_ITEMS], os[SB_ITEMS];
#pragma unroll
  for (int u = 0; u < SB_ITEMS; ++u) {
    const int k = u * 1024 + tid;
    const int* tr = item_trip(pos, neg, P, k < n ? k : 0);
    ss[u] = tr[0];
    os[u] = tr[1];
    rs[u] = k < n ? tr[2] : -1;
  }
  for (int i = tid; i < M; i += blockDim.x) cnt[i] = 0;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < SB_ITEMS; ++u) {   // totals
    const int r = rs[u];
    uint64_t act = __ballot(r >= 0);
    while (act) {
      const int leader = __ffsll((unsigned long long)act) - 1;
      const int rl = __builtin_amdgcn_readlane(r, leader);
      const uint64_t m = __ballot(r == rl) & act;
      if (l == leader) atomicAdd(&cnt[rl], __popcll(m));
      act &= ~m;
    }
  }
  __syncthreads();
  if (wave == 0) {   // relation offsets and tile bases (exclusive scans over p)
    int off = 0, toff = 0;
    for (int p0 = 0; p0 < M; p0 += 64) {
      const int p = p0 + l;
      const int v = p < M ? cnt[p] : 0, tv = (v + RT_ITEMS - 1) / RT_ITEMS;
      const int inc = wave_incl_scan(v), tinc = wave_incl_scan(tv);
      if (p < M) {
        ws.rel_off[p] = off + inc - v;
        base[p] = off + inc - v;
        tbase[p] = toff + tinc - tv;
      }
      off += __shfl(inc, 63, 64);
      toff += __shfl(tinc, 63, 64);
    }
    if (l == 0) {
      ws.rel_off[M] = off;
      tbase[M] = toff;
      *ws.ntiles = toff;
    }
  }
  __syncthreads();
  for (int t = tid; t < tbase[M]; t += blockDim.x) {   // tile t: relation p, tbase[p] <= t
    int lo = 0, hi = M - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tbase[mid] <= t) lo = mid; else hi = mid - 1;
    }
    const int st = (t - tbase[lo]) * RT_ITEMS;
    ws.tile_rel[t] = lo;
    ws.tile_start[t] = base[lo] + st;
    ws.tile_cnt[t] = min(RT_ITEMS, cnt[lo] - st);
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < SB_ITEMS; ++u) {   // stable scatter, one round of 1024 items
    if (u * 1024 >= n) break;
    for (int i = tid; i < 16 * M; i += blockDim.x) cw[i / M][i % M] = 0;
    __syncthreads();
    const int k = u * 1024 + tid;
    const int ts = ss[u], to = os[u], r = rs[u];
    int rank = 0;
    uint64_t act = __ballot(r >= 0);
    while (act) {
      const int leader = __ffsll((unsigned long long)act) - 1;
      const int rl = __builtin_amdgcn_readlane(r, leader);
      const uint64_t m = __ballot(r == rl) & act;
      if (r == rl) rank = __popcll(m & ((1ull << l) - 1ull));
      if (l == leader) cw[wave][rl] = __popcll(m);
      act &= ~m;
    }
    __syncthreads();
    if (r >= 0) {
      int at = base[r] + rank;
      for (int w2 = 0; w2 < wave; ++w2) at += cw[w2][r];
      ws.items[at] = k;
      ws.sorted_s[at] = ts;
      ws.sorted_o[at] = to;
      ws.bpos[k] = at;
    }
    __syncthreads();
    for (int p = tid; p < M; p += blockDim.x) {
      int add = 0;
      for (int w2 = 0; w2 < 16; ++w2) add += cw[w2][p];
      base[p] += add;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Relation-grouped GEMMs, one workgroup per (64-triple tile, 64-column block,
// product):  WE^T[i][r] = sum_k Eo[i][k] W[r][k]   (product 0)
//            EW[i][j]   = sum_k Es[i][k] W[k][j]   (product 1)
// K advances 64 at a time through double-buffered LDS tiles (A: 64 triples x
// 64, B: 64 x 64 columns), the next step's global loads in flight while the
// current step's 64 MFMAs per wave run.  Wave w owns triples 16w..16w+15 and four 16x16
// accumulators (independent chains hide the MFMA latency).  Product-0 blocks
// also write each triple's partial score E[s_i] . WE_i over their 64 columns.
// ---------------------------------------------------------------------------
// B: product 0 as [GC][KS + 4] (W rows as loaded, column-major B), product 1
// as [KS][GC + 4]; both read conflict-free by the MFMA loop
constexpr int rs_sbn(int ks) {
  return GC * (ks + 4) > ks * (GC + 4) ? GC * (ks + 4) : ks * (GC + 4);
}
constexpr int SBN = rs_sbn(KS);
// one GEMM workgroup's LDS: sA [2][RT_ITEMS][KS + 4], sB [2][SBN], 4 x RT_ITEMS ints
constexpr int gemm_lds_floats(int ks) { return 2 * RT_ITEMS * (ks + 4) + 2 * rs_sbn(ks) + 4 * RT_ITEMS; }

// workgroup `bid` of the GEMM grid (k_rescal_gemm, k_rescal_front_fused)
template <bool VEC, int KS = skge::KS>
__device__ __forceinline__ void rescal_gemm_body(const float* __restrict__ E,
                                                 const float* __restrict__ W, int d,
                                                 const RescalWs& ws, int bid,
                                                 float (*sA)[RT_ITEMS][KS + 4],
                                                 float (*sB)[rs_sbn(KS)],
                                                 int* s_row, int* s_gid, int* s_es, int* s_es2) {
  const int ncb = (d + GC - 1) / GC;
  // plain: (tile, product, column block, K slice); deduplicated (ws.npos > 0):
  // (tile, column block, K slice), the product-0 tiles first
  const bool dedup = ws.npos > 0;
  const int gks = ws.gks;
  const int per = (dedup ? ncb : 2 * ncb) * gks;
  const int t = bid / per;
  // the tile's fields and the tile count in one round trip (t < rs_tmax: the
  // fields are in bounds, read before the check, used after it)
  const int nti = ws.ntiles[0], nt0 = dedup ? ws.ntiles[1] : 0;
  const int p = ws.tile_rel[t], s0 = ws.tile_start[t], cnt = ws.tile_cnt[t];
  if (t >= nti) return;
  const int rem_k = bid - t * per;
  const int ksl = rem_k % gks;   // this workgroup's K slice
  const int rem = rem_k / gks;
  const int prod = dedup ? (t < nt0 ? 0 : 1) : rem / ncb;
  const int cb = dedup ? rem : rem - (rem / ncb) * ncb;
  const int tid = threadIdx.x, l = lane_id(), wave = tid >> 6;
  const int c0 = cb * GC;
  if (tid < RT_ITEMS) {
    const bool ok = tid < cnt;
    const int at = s0 + (ok ? tid : 0);
    s_row[tid] = prod == 0 ? ws.sorted_o[at] : ws.sorted_s[at];   // A rows: E[o] or E[s]
    s_es[tid] = ws.sorted_s[at];
    s_gid[tid] = ok ? ws.items[at] : -1;
    s_es2[tid] = (dedup && prod == 0 && ok) ? ws.s2[at] : -1;
  }
  __syncthreads();
  const float* Wp = W + (size_t)p * d * d;
  const int nk_all = (d + KS - 1) / KS, nks = (nk_all + gks - 1) / gks;
  const int k_lo = ksl * nks, nk = min(nk_all, k_lo + nks);   // k-steps [k_lo, nk)
  // staging map, 16 consecutive floats of A and of B per thread and k-step:
  //   A[ai][ak..ak+15] = E[row ai][k + ak ..]
  //   product 0: B[k + bk ..][bq] = W[c0 + bq][k + bk ..]   (transposed into LDS)
  //   product 1: B[bq][bk ..]     = W[k + bq][c0 + bk ..]
  constexpr int SPT = KS / 4;   // floats per thread and operand per k-step
  const int ai = tid >> 2, ak = (tid & 3) * SPT;
  const float* arow = E + (size_t)s_row[ai] * d;
  const bool a_ok = ai < cnt;
  // product 0: thread -> W row c0 + bq, k offsets bk..; product 1: W row
  // k + bq, columns c0 + bk.. (256 / KS threads share a row of 64 columns)
  const int bq = prod == 0 ? tid >> 2 : tid / (256 / KS);
  const int bk = prod == 0 ? (tid & 3) * SPT : (tid % (256 / KS)) * SPT;
  float ra[SPT], rb[SPT];
  // raw loads from clamped in-range addresses; masks are applied when the
  // values are staged (a select right after a load would wait for it)
  auto load_step = [&](int ks) {
    const int k = ks * KS;
    const float* brow;
    int boff;
    if (prod == 0) {
      brow = Wp + (size_t)(c0 + bq < d ? c0 + bq : 0) * d;
      boff = k + bk;
    } else {
      brow = Wp + (size_t)(k + bq < d ? k + bq : 0) * d;
      boff = c0 + bk;
    }
    if (VEC) {   // d % 4 == 0: each 4-float group is inside or outside together
#pragma unroll
      for (int m = 0; m < SPT / 4; ++m) {
        const int ka = k + ak + 4 * m, kb = boff + 4 * m;
        const float4 x = *reinterpret_cast<const float4*>(arow + (ka < d ? ka : 0));
        const float4 y = *reinterpret_cast<const float4*>(brow + (kb < d ? kb : 0));
        ra[4 * m] = x.x, ra[4 * m + 1] = x.y, ra[4 * m + 2] = x.z, ra[4 * m + 3] = x.w;
        rb[4 * m] = y.x, rb[4 * m + 1] = y.y, rb[4 * m + 2] = y.z, rb[4 * m + 3] = y.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < SPT; ++e) {
        const int ka = k + ak + e, kb = boff + e;
        ra[e] = arow[ka < d ? ka : 0];
        rb[e] = brow[kb < d ? kb : 0];
      }
    }
  };
  auto store_step = [&](int buf, int ks) {
    const int k = ks * KS;
#pragma unroll
    for (int m = 0; m < SPT / 4; ++m) {
      float4 v;
      v.x = (a_ok && k + ak + 4 * m + 0 < d) ? ra[4 * m + 0] : 0.0f;
      v.y = (a_ok && k + ak + 4 * m + 1 < d) ? ra[4 * m + 1] : 0.0f;
      v.z = (a_ok && k + ak + 4 * m + 2 < d) ? ra[4 * m + 2] : 0.0f;
      v.w = (a_ok && k + ak + 4 * m + 3 < d) ? ra[4 * m + 3] : 0.0f;
      *reinterpret_cast<float4*>(&sA[buf][ai][ak + 4 * m]) = v;
    }
    if (prod == 0) {   // B[k][r] = W[r][k], kept as W's rows: sB[r][k]
      const bool rok = c0 + bq < d;
#pragma unroll
      for (int m = 0; m < SPT / 4; ++m) {
        float4 v;
        v.x = (rok && k + bk + 4 * m + 0 < d) ? rb[4 * m + 0] : 0.0f;
        v.y = (rok && k + bk + 4 * m + 1 < d) ? rb[4 * m + 1] : 0.0f;
        v.z = (rok && k + bk + 4 * m + 2 < d) ? rb[4 * m + 2] : 0.0f;
        v.w = (rok && k + bk + 4 * m + 3 < d) ? rb[4 * m + 3] : 0.0f;
        *reinterpret_cast<float4*>(&sB[buf][bq * (KS + 4) + bk + 4 * m]) = v;
      }
    } else {
      const bool kok = k + bq < d;
#pragma unroll
      for (int m = 0; m < SPT / 4; ++m) {
        float4 v;
        v.x = (kok && c0 + bk + 4 * m + 0 < d) ? rb[4 * m + 0] : 0.0f;
        v.y = (kok && c0 + bk + 4 * m + 1 < d) ? rb[4 * m + 1] : 0.0f;
        v.z = (kok && c0 + bk + 4 * m + 2 < d) ? rb[4 * m + 2] : 0.0f;
        v.w = (kok && c0 + bk + 4 * m + 3 < d) ? rb[4 * m + 3] : 0.0f;
        *reinterpret_cast<float4*>(&sB[buf][bq * (GC + 4) + bk + 4 * m]) = v;
      }
    }
  };
  f32x4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  const int row = wave * 16 + (l & 15), kq = l >> 4;
  load_step(k_lo);
  for (int ks = k_lo; ks < nk; ++ks) {
    const int buf = (ks - k_lo) & 1;
    store_step(buf, ks);
    __syncthreads();   // (also: every wave is done with buf's previous use, step ks - 2)
    if (ks + 1 < nk) load_step(ks + 1);   // in flight during this step's MFMAs
    // B[k4 + kq][16 q + c]: product 0 at sB[(16 q + c)(KS + 4) + k4 + kq]
    // (banks 36 c + kq: distinct), product 1 at sB[(k4 + kq)(GC + 4) + 16 q + c]
    if (prod == 0) {
      const float* b0 = &sB[buf][(l & 15) * (KS + 4) + kq];
#pragma unroll
      for (int k4 = 0; k4 < KS; k4 += 4) {
        const float a = sA[buf][row][k4 + kq];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b0[q * 16 * (KS + 4) + k4], acc[q], 0,
                                                        0, 0);
      }
    } else {
      const float* b1 = &sB[buf][kq * (GC + 4) + (l & 15)];
#pragma unroll
      for (int k4 = 0; k4 < KS; k4 += 4) {
        const float a = sA[buf][row][k4 + kq];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b1[k4 * (GC + 4) + q * 16], acc[q], 0,
                                                        0, 0);
      }
    }
  }
  // epilogue: D[row 4g + reg][col] of accumulator q -> triple 16w + 4g + reg, column c0 + 16q + c
  float* out = (prod == 0 ? ws.WE : ws.EW) + (size_t)ksl * ws.part_stride;
  float* const spart = ws.spart + (size_t)ksl * ws.spart_stride;
  const int g = l >> 4, c = l & 15;
  float ev[4][4], ev2[4][4];
  // a row with a second subject (deduplicated: a positive's WE row also
  // scores its s-corrupted negative); wave-uniform test, any row of the wave
  bool two = false;
  if (prod == 0) {   // E[s_i] over the block's columns, all loads issued together
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) two = two || s_es2[wave * 16 + 4 * g + reg] >= 0;
    two = __ballot(two) != 0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int col = c0 + q * 16 + c;
        ev[q][reg] = E[(size_t)s_es[wave * 16 + 4 * g + reg] * d + (col < d ? col : 0)];
        if (two) {
          const int r2 = s_es2[wave * 16 + 4 * g + reg];
          ev2[q][reg] = E[(size_t)(r2 >= 0 ? r2 : 0) * d + (col < d ? col : 0)];
        }
      }
  }
  float ps[4] = {0.0f, 0.0f, 0.0f, 0.0f}, ps2[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int col = c0 + q * 16 + c;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int it = wave * 16 + 4 * g + reg;
      if (it < cnt && col < d) out[(size_t)s_gid[it] * d + col] = acc[q][reg];
      if (prod == 0) ps[reg] += (col < d) ? acc[q][reg] * ev[q][reg] : 0.0f;
      if (prod == 0 && two) ps2[reg] += (col < d) ? acc[q][reg] * ev2[q][reg] : 0.0f;
    }
  }
  if (prod == 0) {
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      float v = ps[reg];
      v += __shfl_xor(v, 8, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 1, 64);
      const int it = wave * 16 + 4 * g + reg;
      if (c == 0 && it < cnt) spart[(size_t)s_gid[it] * ncb + cb] = v;
      if (two) {   // the s-corrupted negative (item npos + 2j) of positive j = s_gid
        float v2 = ps2[reg];
        v2 += __shfl_xor(v2, 8, 64);
        v2 += __shfl_xor(v2, 4, 64);
        v2 += __shfl_xor(v2, 2, 64);
        v2 += __shfl_xor(v2, 1, 64);
        if (c == 0 && it < cnt && s_es2[it] >= 0)
          spart[(size_t)(ws.npos + 2 * s_gid[it]) * ncb + cb] = v2;
      }
    }
  }
}

template <bool VEC>
__global__ __launch_bounds__(256) void k_rescal_gemm(const float* __restrict__ E,
                                                     const float* __restrict__ W, int d,
                                                     RescalWs ws) {
  __shared__ float sA[2][RT_ITEMS][KS + 4];
  __shared__ float sB[2][SBN];
  __shared__ int s_row[RT_ITEMS], s_gid[RT_ITEMS], s_es[RT_ITEMS], s_es2[RT_ITEMS];
  rescal_gemm_body<VEC>(E, W, d, ws, (int)blockIdx.x, sA, sB, s_row, s_gid, s_es, s_es2);
}

// ---------------------------------------------------------------------------
// margin test + entity contributions, one wave per pair (rescal.py:264-302)
// ---------------------------------------------------------------------------
template <int KM>
__global__ __launch_bounds__(256) void k_rescal_scatter(const int* __restrict__ pos,
                                                        const int* __restrict__ neg, int P, int d,
                                                        int af, float margin, RescalWs ws,
                                                        Accum accE, float* pscore, float* nscore,
                                                        int* nviol) {
  const int wpb = blockDim.x >> 6;
  int nv = 0;
  for (int i = blockIdx.x * wpb + (threadIdx.x >> 6); i < P; i += gridDim.x * wpb) {
    const int ix[6] = {__builtin_amdgcn_readfirstlane(pos[3 * i]),
                       __builtin_amdgcn_readfirstlane(pos[3 * i + 1]),
                       __builtin_amdgcn_readfirstlane(pos[3 * i + 2]),
                       __builtin_amdgcn_readfirstlane(neg[3 * i]),
                       __builtin_amdgcn_readfirstlane(neg[3 * i + 1]),
                       __builtin_amdgcn_readfirstlane(neg[3 * i + 2])};
    if (ix[2] < 0) {   // skipped pair: never bucketed (relation -1), no contribution
      commit_pair(accE, nullptr, false, ix, i);
      continue;
    }
    const int ncb = (d + GC - 1) / GC;
    const float praw = spart_sum(ws, i, ncb), nraw = spart_sum(ws, P + i, ncb);   // fixed order
    const float pf = af_f(af, praw), nf = af_f(af, nraw);
    const float gp = -af_g_given_f(af, pf);   // rescal.py:275 (all pairs)
    const float gn = af_g_given_f(af, nf);
    if (lane_id() == 0) {
      if (pscore) pscore[i] = praw;
      if (nscore) nscore[i] = nraw;
      ws.coef[ws.bpos[i]] = gp;
      ws.coef[ws.bpos[P + i]] = gn;
    }
    const bool viol = nf + margin > pf;   // rescal.py:269
    commit_pair(accE, nullptr, viol, ix, i);
    if (!viol) continue;
    ++nv;
    float wep[KM], wen[KM], ewp[KM], ewn[KM], x[KM], y[KM];
    load_row_gk<KM>(ws.WE, ws, i, d, wep);
    load_row_gk<KM>(ws.WE, ws, P + i, d, wen);
    load_row_gk<KM>(ws.EW, ws, i, d, ewp);
    load_row_gk<KM>(ws.EW, ws, P + i, d, ewn);
    // (sp, sn) <- (gp WEp, gn WEn)                    rescal.py:299-300
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      x[k] = gp * wep[k];
      y[k] = gn * wen[k];
    }
    acc_two<KM>(accE, ix[0], x, ix[3], y, d);
    // (op, on) <- (gp EWp, gn EWn)                    rescal.py:296-301
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      x[k] = gp * ewp[k];
      y[k] = gn * ewn[k];
    }
    acc_two<KM>(accE, ix[1], x, ix[4], y, d);
  }
  __shared__ int lds_nv;
  if (nviol) block_count_add(nviol, nv, &lds_nv);
}

// ---------------------------------------------------------------------------
// The device pair loop's form: one wave per POSITIVE and both of its pairs.
// The batch's triples are deduplicated -- list a holds each positive once
// (item j), list b its two negatives (items count + 2j: (s', o, p), count +
// 2j + 1: (s, o', p)) -- so the GEMMs and dW see 3 items per positive instead
// of the explicit pairs' 4 (the positive appears in both pairs).  Scores come
// from the same per-item partial sums (bitwise the pair path's); dW gets the
// positive once with coefficient gp (k0 + k1) (rescal.py:113-125 sums gp over
// every pair it is in); the entity rows get the two pairs' contributions
// (rescal.py:296-301) summed per row, with the occurrence counts of the
// lists (s: v0 + 2 v1, o: 2 v0 + v1, s': v0, o': v1; slots 4j..4j+3).
// ---------------------------------------------------------------------------
template <int KM>
__global__ __launch_bounds__(256) void k_rescal_pos_scatter(const int4* __restrict__ rec,
                                                            const int* __restrict__ rec_n1,
                                                            long long start, int count, int d,
                                                            int af, float margin, RescalWs ws,
                                                            Accum accE, int* nviol) {
  const int wpb = blockDim.x >> 6, l = lane_id(), ncb = (d + GC - 1) / GC;
  int nv = 0;
  for (int j = blockIdx.x * wpb + (threadIdx.x >> 6); j < count; j += gridDim.x * wpb) {
    const int4 r4 = rec[start + j];
    const int s = __builtin_amdgcn_readfirstlane(r4.x), o = __builtin_amdgcn_readfirstlane(r4.y);
    const int neg0 = __builtin_amdgcn_readfirstlane(r4.w);
    const int neg1 = __builtin_amdgcn_readfirstlane(rec_n1[start + j]);
    const int k0 = neg0 >= 0 ? 1 : 0, k1 = neg1 >= 0 ? 1 : 0;
    const int i0 = count + 2 * j, i1 = i0 + 1;   // the negatives' items
    // the contribution rows, loaded with the partial scores (one round trip; a
    // positive without a violation discards them): W E_o and E_s W of the
    // positive, E_s' W of (s', o, p), W E_o' of (s, o', p)
    float wep[KM], ewp[KM], ew0[KM], we1[KM];
    load_row_gk<KM>(ws.WE, ws, j, d, wep);
    load_row_gk<KM>(ws.EW, ws, j, d, ewp);
    load_row_gk<KM>(ws.EW, ws, i0, d, ew0);
    load_row_gk<KM>(ws.WE, ws, i1, d, we1);
    // fixed order: deterministic
    const float praw = spart_sum(ws, j, ncb), raw0 = spart_sum(ws, i0, ncb),
                raw1 = spart_sum(ws, i1, ncb);
    const float pf = af_f(af, praw), f0 = af_f(af, raw0), f1 = af_f(af, raw1);
    const float gp = -af_g_given_f(af, pf);   // rescal.py:275 (all pairs)
    const float g0 = af_g_given_f(af, f0), g1 = af_g_given_f(af, f1);
    if (l == 0 && k0 + k1 > 0 && ws.coef) {   // (null: dW was formed from ecoef already)
      ws.coef[ws.bpos[j]] = gp * (float)(k0 + k1);
      if (k0) ws.coef[ws.bpos[i0]] = g0;
      if (k1) ws.coef[ws.bpos[i1]] = g1;
    }
    const int v0 = (k0 && f0 + margin > pf) ? 1 : 0;   // rescal.py:269
    const int v1 = (k1 && f1 + margin > pf) ? 1 : 0;
    if (l < 4)
      commit_slot(accE, sel4(l, s, o, neg0, neg1), sel4(l, v0 + 2 * v1, 2 * v0 + v1, v0, v1),
                  4 * j + l);
    if (v0 + v1 == 0) continue;
    nv += v0 + v1;
    // (stale rows of absent negatives are not used; deduplicated GEMM rows: W
    // E_o of (s', o, p) is positive j's row, E_s W of (s, o', p) likewise --
    // bitwise the same values)
    float we0[KM], ew1[KM], x[KM];
    if (ws.npos > 0) {
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        we0[k] = wep[k];
        ew1[k] = ewp[k];
      }
    } else {
      load_row_gk<KM>(ws.WE, ws, i0, d, we0);
      load_row_gk<KM>(ws.EW, ws, i1, d, ew1);
    }
    const float fv0 = (float)v0, fv1 = (float)v1;
#pragma unroll
    for (int k = 0; k < KM; ++k) x[k] = fv0 * (gp * wep[k]) + fv1 * (gp * wep[k] + g1 * we1[k]);
    acc_row<KM>(accE, s, x, d);
#pragma unroll
    for (int k = 0; k < KM; ++k) x[k] = fv0 * (gp * ewp[k] + g0 * ew0[k]) + fv1 * (gp * ewp[k]);
    acc_row<KM>(accE, o, x, d);
    if (v0) {
#pragma unroll
      for (int k = 0; k < KM; ++k) x[k] = g0 * we0[k];
      acc_row<KM>(accE, neg0, x, d);
    }
    if (v1) {
#pragma unroll
      for (int k = 0; k < KM; ++k) x[k] = g1 * ew1[k];
      acc_row<KM>(accE, neg1, x, d);
    }
  }
  __shared__ int lds_nv;
  if (nviol) block_count_add(nviol, nv, &lds_nv);
}

// ---------------------------------------------------------------------------
// The device pair loop's entity update without the scatter (k_rescal_fold):
// one wave per work item of k_rs_rows_ep's grouping (two slots of a
// distinct entity row; a hub row's items merged by the last to arrive)
// takes the row's slots in slot order, recomputes each slot's pair tests
// from the partial scores and forms its contribution from the WE / EW rows
// exactly as k_rescal_pos_scatter does (rescal.py:264-302), sums them in
// registers (a fixed order: no float atomics, bitwise reproducible), then
// applies the segment mean and the updater's step (skge/param.py:115-174, as
// apply_row).  Workgroup 0 counts the batch's violations (the scatter's test
// for every positive: the gate) and makes the in-front W step current when
// there are any (WStep::cur; updateCounts of the relations present).
// ---------------------------------------------------------------------------
struct FoldTab {
  float* P;
  float* A;
  int* ucnt;
  int opt, post;
  float lr, rin, rout, fdiv;
  Accum acc;   // the entity accumulator: hub rows' sums (rows of more than RS_FOLD_MERGE items)
};
// a row of at most this many items (2 slots each) is merged from partial sums
// in item order (bitwise reproducible); a larger one (a hub of a skewed KG)
// adds its items into the entity accumulator (fp32 atomics, or exact
// fixed-point ones in the deterministic mode)
constexpr int RS_FOLD_MERGE = 8;

// slot `sl` of the batch in two halves, so a wave keeps several slots' loads
// in flight: fold_load issues the slot's WE / EW rows -- s: W E_o of the
// positive and of (s, o', p); o: E_s W of the positive and of (s', o, p);
// s' / o': the negative's own row (deduplicated: the positive's) -- and its
// three items' partial scores (lane q < 3 ncb: item q / ncb, column block
// q % ncb; K slices in sp2); fold_combine sums the scores in spart_sum's
// order, runs the pair tests and forms the contribution (x) exactly as
// k_rescal_pos_scatter does, returning the slot's count
template <int KM>
struct FoldLd {
  float ra[KM], rb[KM];
  float sp, sp2;
};

template <int KM>
__device__ __forceinline__ void fold_load(const RescalWs& ws, int count, int d, int sl,
                                          FoldLd<KM>& f) {
  const int l = lane_id(), ncb = (d + GC - 1) / GC;
  const int j = sl >> 4, role = sl & 3, i0 = count + 2 * j, i1 = i0 + 1;
  const bool dd = ws.npos > 0;
  const float* ta = (role & 1) ? ws.EW : ws.WE;
  load_row_gk<KM>(ta, ws, role < 2 ? j : (dd ? j : (role == 2 ? i0 : i1)), d, f.ra);
  if (role < 2) load_row_gk<KM>(ta, ws, role == 0 ? i1 : i0, d, f.rb);
  const int it = l / ncb, cb = l - it * ncb;
  const size_t at = (size_t)(it == 0 ? j : (it == 1 ? i0 : i1)) * ncb + cb;
  f.sp = l < 3 * ncb ? ws.spart[at] : 0.0f;
  f.sp2 = (ws.gks > 1 && l < 3 * ncb) ? ws.spart[ws.spart_stride + at] : 0.0f;
}

template <int KM>
__device__ __forceinline__ int fold_combine(const RescalWs& ws, int d, int af, float margin,
                                            int sl, const FoldLd<KM>& f, float (&x)[KM]) {
  const int ncb = (d + GC - 1) / GC;
  const int k1 = (sl >> 3) & 1, k0 = (sl >> 2) & 1, role = sl & 3;
  float raw[3];
#pragma unroll
  for (int it = 0; it < 3; ++it) {   // spart_sum's order
    float r = 0.0f;
    for (int q = 0; q < ncb; ++q) {
      r += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(f.sp), it * ncb + q));
      if (ws.gks > 1) r += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(f.sp2), it * ncb + q));
    }
    raw[it] = r;
  }
  const float pf = af_f(af, raw[0]), f0 = af_f(af, raw[1]), f1 = af_f(af, raw[2]);
  const float gp = -af_g_given_f(af, pf);   // rescal.py:275 (all pairs)
  const float g0 = af_g_given_f(af, f0), g1 = af_g_given_f(af, f1);
  const int v0 = (k0 && f0 + margin > pf) ? 1 : 0;   // rescal.py:269
  const int v1 = (k1 && f1 + margin > pf) ? 1 : 0;
  const float fv0 = (float)v0, fv1 = (float)v1;
  if (role == 0) {
#pragma unroll
    for (int k = 0; k < KM; ++k) x[k] = fv0 * (gp * f.ra[k]) + fv1 * (gp * f.ra[k] + g1 * f.rb[k]);
    return v0 + 2 * v1;
  }
  if (role == 1) {
#pragma unroll
    for (int k = 0; k < KM; ++k) x[k] = fv0 * (gp * f.ra[k] + g0 * f.rb[k]) + fv1 * (gp * f.ra[k]);
    return 2 * v0 + v1;
  }
  const int v = role == 2 ? v0 : v1;
  const float gg = role == 2 ? g0 : g1;
#pragma unroll
  for (int k = 0; k < KM; ++k) x[k] = v ? gg * f.ra[k] : 0.0f;
  return v;
}

template <int KM>
__global__ __launch_bounds__(256) void k_rescal_fold(const int4* __restrict__ rec,
                                                     const int* __restrict__ rec_n1,
                                                     long long start, int count, int d, int af,
                                                     float margin, RescalWs ws, FoldTab t,
                                                     WStep w, int* nviol, int nvw) {
  const int l = lane_id(), ncb = (d + GC - 1) / GC;
  if ((int)blockIdx.x < nvw) {
    // the first nvw workgroups: the batch's violations (the scatter's test,
    // one positive per thread); their counts and arrivals go into ONE 64-bit
    // word (one returned atomic per workgroup), so the last to arrive holds
    // the exact total -- the gate -- and makes the in-front W step current
    __shared__ int lds_nv, lds_tot;
    const int j = (int)blockIdx.x * (int)blockDim.x + (int)threadIdx.x;
    int nv = 0;
    if (j < count) {
      const int4 r4 = rec[start + j];
      const int n1 = rec_n1[start + j];
      const float pf = af_f(af, spart_sum(ws, j, ncb));
      const float f0 = af_f(af, spart_sum(ws, count + 2 * j, ncb));
      const float f1 = af_f(af, spart_sum(ws, count + 2 * j + 1, ncb));
      nv = ((r4.w >= 0 && f0 + margin > pf) ? 1 : 0) + ((n1 >= 0 && f1 + margin > pf) ? 1 : 0);
    }
    if (threadIdx.x == 0) lds_nv = 0;
    __syncthreads();
    nv = wave_sum_int(nv);
    if (l == 0 && nv) atomicAdd(&lds_nv, nv);
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long add = (1ull << 32) | (unsigned)lds_nv;
      const unsigned long long old = atomicAdd(ws.vword, add);
      // the last to arrive has every count: the batch's total
      lds_tot = (int)(old >> 32) == nvw - 1 ? (int)(unsigned)(old + add) : -1;
    }
    __syncthreads();
    const int tot = lds_tot;
    if (tot >= 0 && threadIdx.x < 64) {
      if (l == 0) *nviol = tot;
      if (w.cur && tot != 0) {   // the in-front W step becomes current (k_apply_wstep)
        if (l == 0) *w.cur ^= 1;
        if (w.opt == OPT_ADAGRAD && w.ucnt)   // updateCounts, skge/param.py:149-150 (lane p)
          for (int p = l; p < w.M; p += 64)
            if (w.rel_off[p + 1] > w.rel_off[p]) atomicAdd(w.ucnt + (p), 1);
      }
    }
    return;
  }
  // one wave per work item (two slots of a distinct row): its record in one
  // round trip, then the slots' rows and partial scores (and, for a row of one
  // item, the row's parameters and state)
  const int wi = ((int)blockIdx.x - nvw) * (int)(blockDim.x >> 6) + (int)(threadIdx.x >> 6);
  const int4 ur = ws.urec[wi];   // (wi < 4 count; row -1 past the batch's items)
  if (ur.x < 0) return;
  const int row = __builtin_amdgcn_readfirstlane(ur.x);
  const int sa0 = __builtin_amdgcn_readfirstlane(ur.y), sb0 = __builtin_amdgcn_readfirstlane(ur.z);
  const int info = __builtin_amdgcn_readfirstlane(ur.w);
  const int chunk = info >> 16, nch = info & 0xFFFF;
  const bool ada = t.opt == OPT_ADAGRAD;
  float* __restrict__ prow = t.P + (size_t)row * d;
  float* __restrict__ arow = ada ? t.A + (size_t)row * d : nullptr;
  float p[KM], a[KM], s[KM];
  if (nch == 1) {
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int e = l + 64 * k, ec = e < d ? e : d - 1;
      p[k] = prow[ec];
      a[k] = ada ? arow[ec] : 0.0f;
    }
  }
  int c;
  {   // every load issued, then the sums (slot order)
    FoldLd<KM> fa, fb;
    fold_load<KM>(ws, count, d, sa0, fa);
    if (sb0 >= 0) fold_load<KM>(ws, count, d, sb0, fb);
    float xa[KM], xb[KM];
    c = fold_combine<KM>(ws, d, af, margin, sa0, fa, xa);
    if (sb0 >= 0) c += fold_combine<KM>(ws, d, af, margin, sb0, fb, xb);
#pragma unroll
    for (int k = 0; k < KM; ++k) s[k] = sb0 >= 0 ? xa[k] + xb[k] : xa[k];
  }
  if (nch > 1) {
    // a row of several items: each item publishes its partial sum -- up to
    // RS_FOLD_MERGE items write-through into its own slot, more (a hub row)
    // into the entity accumulator with atomics -- drains, then adds to the
    // row's arrival counter; the last to arrive reads the partials in item
    // order (sc1 loads: every handed-off byte was stored sc1 or by an atomic
    // and drained before the counter add) or the accumulated row, and applies
    const bool hub = nch > RS_FOLD_MERGE;
    if (hub) {
      acc_row<KM>(t.acc, row, s, d);
      if (l == 0 && c) atomicAdd(t.acc.cnt + row, c);
    } else {
      float* pw = ws.part + (size_t)wi * d;
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const int e = l + 64 * k;
        if (e < d) __hip_atomic_store(pw + e, s[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (l == 0) __hip_atomic_store(ws.pcnt + wi, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int w0 = wi - chunk;
    int old = 0;
    if (l == 0) old = atomicAdd(ws.rowctr + w0, 1);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old != nch - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the loads below the add
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int e = l + 64 * k, ec = e < d ? e : d - 1;
      p[k] = prow[ec];
      a[k] = ada ? arow[ec] : 0.0f;
    }
    if (hub) {   // the accumulated row and count, then zeroed for the next batch
      const bool fx = t.acc.mode == ACC_FX64;
      float* srow = t.acc.sum + (size_t)row * t.acc.width;
      unsigned long long* xrow = reinterpret_cast<unsigned long long*>(t.acc.sum) +
                                 (size_t)row * t.acc.width;
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const int e = l + 64 * k, ec = e < d ? e : d - 1;
        s[k] = fx ? fx_dec((long long)__hip_atomic_load(xrow + ec, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT))
                  : __hip_atomic_load(srow + ec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      c = __hip_atomic_load(t.acc.cnt + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const int e = l + 64 * k;
        if (e < d) {
          if (fx)
            xrow[e] = 0ull;
          else
            srow[e] = 0.0f;
        }
      }
      if (l == 0) t.acc.cnt[row] = 0;
    } else {   // the items' partials, all loads in flight, summed in item order
      float v[RS_FOLD_MERGE][KM];
      int cv[RS_FOLD_MERGE];
#pragma unroll
      for (int q = 0; q < RS_FOLD_MERGE; ++q) {
        const int qq = q < nch ? q : 0;
        const float* pq = ws.part + (size_t)(w0 + qq) * d;
#pragma unroll
        for (int k = 0; k < KM; ++k) {
          const int e = l + 64 * k, ec = e < d ? e : d - 1;
          v[q][k] = __hip_atomic_load(pq + ec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        cv[q] = __hip_atomic_load(ws.pcnt + w0 + qq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      c = 0;
#pragma unroll
      for (int k = 0; k < KM; ++k) s[k] = 0.0f;
#pragma unroll
      for (int q = 0; q < RS_FOLD_MERGE; ++q) {
        if (q >= nch) break;
#pragma unroll
        for (int k = 0; k < KM; ++k) s[k] += v[q][k];
        c += cv[q];
      }
    }
  }
  if (c == 0) return;   // no violating occurrence: the row is not updated
  if (ada && t.ucnt && l == 0) atomicAdd(t.ucnt + (row), 1);   // param.py:149-150
  const float div = t.fdiv > 0.0f ? t.fdiv : (float)c;
  float ss = 0.0f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const bool in = l + 64 * k < d;
    const float pv0 = in ? p[k] : 0.0f;
    const float g = ((in ? s[k] : 0.0f) + t.rin * pv0) / div + t.rout * pv0;   // segment mean (+ rparam)
    float pv = pv0;
    if (ada) {
      const float av = (in ? a[k] : 0.0f) + g * g;      // p2[idx] += g*g           param.py:147
      a[k] = av;
      pv = pv - (t.lr * g) / fmaxf(sqrtf(av), 1e-7f);   // P -= lr*g/max(sqrt,1e-7) param.py:152-155
    } else {
      pv = pv - t.lr * g;                               // P -= lr*g                param.py:130
    }
    p[k] = pv;
    ss += pv * pv;
  }
  if (t.post != POST_NONE) {
    ss = wave_sum(ss);
    const float nrm = t.post == POST_NORMALIZE ? sqrtf(ss) : (ss < 1.0f ? 1.0f : ss);
#pragma unroll
    for (int k = 0; k < KM; ++k) p[k] = p[k] / nrm;   // param.py:165-166 / 171-173
  }
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int e = l + 64 * k;
    if (e < d) {
      prow[e] = p[k];
      if (ada) arow[e] = a[k];
    }
  }
}

// ---------------------------------------------------------------------------
// logistic loss + entity contributions, one wave per labelled triple
// (rescal.py:37-76): fs = -y sigmoid(-y f); E[s] += fs WE, E[o] += fs EW
// ---------------------------------------------------------------------------
template <int KM>
__global__ __launch_bounds__(256) void k_rescal_logistic(const int* __restrict__ trip,
                                                         const float* __restrict__ ys, int T,
                                                         int d, RescalWs ws, Accum accE,
                                                         float* score_out, float* loss) {
  const int wpb = blockDim.x >> 6, ncb = (d + GC - 1) / GC;
  float lsum = 0.0f;
  for (int i = blockIdx.x * wpb + (threadIdx.x >> 6); i < T; i += gridDim.x * wpb) {
    const int s = __builtin_amdgcn_readfirstlane(trip[3 * i]);
    const int o = __builtin_amdgcn_readfirstlane(trip[3 * i + 1]);
    const float score = spart_sum(ws, i, ncb);   // fixed order
    const float y = ys[i];
    const float ysc = y * score;
    const float li = fmaxf(-ysc, 0.0f) + log1pf(expf(-fabsf(ysc)));   // logaddexp(0, -ys)
    const float fs = -(y * (1.0f / (1.0f + expf(ysc))));                 // -(y sigmoid(-ys))
    if (lane_id() == 0) {
      if (score_out) score_out[i] = score;
      ws.coef[ws.bpos[i]] = fs;
    }
    {
      const int l = lane_id();   // entity occurrences (s, o): slots 2i, 2i+1
      if (l < 2) commit_slot(accE, l == 0 ? s : o, s == o ? (l == 0 ? 2 : 0) : 1, 2 * i + l);
    }
    float we[KM], ew[KM], x[KM], yv[KM];
    load_row_gk<KM>(ws.WE, ws, i, d, we);
    load_row_gk<KM>(ws.EW, ws, i, d, ew);
#pragma unroll
    for (int k = 0; k < KM; ++k) {   // rescal.py:65-66 (fs WE over ss, fs EW over os)
      x[k] = fs * we[k];
      yv[k] = fs * ew[k];
    }
    acc_two<KM>(accE, s, x, o, yv, d);
    lsum += li;
  }
  __shared__ float lds_loss;
  if (loss) block_sum_add(loss, lsum, &lds_loss);
}

// ---------------------------------------------------------------------------
// dW[p] = sum_items coef_i E[s_i] (x) E[o_i]: one workgroup per (relation,
// 16-row strip, 4 x 16-column tiles); K = the relation's triples in bucket order
// ---------------------------------------------------------------------------
// the W updater, applied by the workgroup that owns each dW tile (APPLY):
// the same g = (sum + rin W)/div + rout W, AdaGrad / SGD step as k_apply_wide
// (skge/param.py:115-155), with sum = the tile's dW straight from registers
struct WApply {
  float* W;
  float* A;          // AdaGrad state or nullptr
  int opt;
  float lr, rin, rout, fdiv;
  const int* gate;   // skip the update when *gate == 0 (no violations)
  int* ucnt;         // optional updateCounts
};

// dW[p] = sum_i coef_i E[s_i]^T E[o_i] over relation p's items.  One
// workgroup per (relation, 64-row tile, 64-col tile); wave w owns rows
// 16w..16w+15 and all 64 columns (four 16x16 accumulators); items are staged
// 64 at a time (coef-scaled E[s] and E[o] row segments, one memory round
// trip per chunk) and contracted with v_mfma_f32_16x16x4_f32.
constexpr int WG_T = 64;    // rows / columns of a dW tile
constexpr int WG_CH = 64;   // items staged per step
constexpr int WG_TPI = 256 / WG_CH;       // threads per item
constexpr int WG_FPT = WG_T / WG_TPI;     // row floats per thread and operand
constexpr int WG_PF = SKGE_RS_WG_PF;      // chunks of items loaded together

template <bool APPLY, bool VEC>
__global__ __launch_bounds__(256) void k_rescal_wgrad_mfma(const float* __restrict__ E, int d,
                                                           RescalWs ws, Accum accW, WApply wa) {
  const int nt = (d + WG_T - 1) / WG_T;
  const int blk = blockIdx.x;
  const int p = blk / (nt * nt);
  const int rem = blk - p * nt * nt;
  const int rt = rem / nt, ct = rem - (rem / nt) * nt;
  const int tid = threadIdx.x, l = lane_id(), wave = tid >> 6;
  const int off = ws.rel_off[p], cnt = ws.rel_off[p + 1] - off;
  const int gv = APPLY && wa.gate != nullptr ? *wa.gate : 1;   // (loaded with rel_off)
  if (!APPLY && rem == 0 && tid == 0) {   // slot p (skge_hip.h slot map)
    if (accW.touched) accW.touched[p] = cnt > 0 ? p : -1;
    accW.cnt[p] = cnt;
  }
  if (cnt == 0) return;
  const bool upd = gv != 0;
  if (APPLY && !upd) return;   // the model returned None: no update
  if (APPLY && rem == 0 && tid == 0 && wa.opt == OPT_ADAGRAD && wa.ucnt)
    atomicAdd(wa.ucnt + (p), 1);   // updateCounts, skge/param.py:149-150
  __shared__ float sEs[2][WG_CH][WG_T + 4];
  __shared__ float sEo[2][WG_CH][WG_T + 4];
  const int r0 = rt * WG_T, c0 = ct * WG_T;
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  // thread -> item it of a chunk, WG_FPT columns from h of its E[s] segment
  // (rows r0..) and E[o] segment (columns c0..).  The items are loaded WG_PF
  // chunks at a time, every load of the group in flight together (one round
  // trip for the ids, one for the rows, per group -- at the reference's batch
  // size a relation's items fit one group), then staged chunk by chunk
  // through the double-buffered LDS and contracted.
  const int it = tid / WG_TPI, h = (tid % WG_TPI) * WG_FPT;
  // the W updater's operands do not depend on dW: in flight from the start
  size_t os[16];
  bool in[16];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int r = r0 + 16 * wave + 4 * (l >> 4) + reg, cc = c0 + 16 * j + (l & 15);
      in[4 * j + reg] = r < d && cc < d;
      os[4 * j + reg] = (size_t)p * d * d + (size_t)(r < d ? r : 0) * d + (cc < d ? cc : 0);
    }
  float pv[16], av[16];
  if (APPLY) {
    const bool ada = wa.opt == OPT_ADAGRAD;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      pv[e] = wa.W[os[e]];
      av[e] = ada ? wa.A[os[e]] : 0.0f;
    }
  }
  const int nch = (cnt + WG_CH - 1) / WG_CH;
  for (int g0 = 0; g0 < nch; g0 += WG_PF) {
    int ns[WG_PF], no[WG_PF];
    float nc[WG_PF];
#pragma unroll
    for (int q = 0; q < WG_PF; ++q) {   // the group's item ids (clamped in-range addresses)
      const int i = (g0 + q) * WG_CH + it;
      const int at = off + (i < cnt ? i : cnt - 1);
      ns[q] = ws.sorted_s[at];
      no[q] = ws.sorted_o[at];
      nc[q] = i < cnt ? ws.coef[at] : 0.0f;
    }
    float4 es[WG_PF][WG_FPT / 4], eo[WG_PF][WG_FPT / 4];
#pragma unroll
    for (int q = 0; q < WG_PF; ++q) {   // the group's row segments
      const float* srow = E + (size_t)ns[q] * d;
      const float* orow = E + (size_t)no[q] * d;
#pragma unroll
      for (int m = 0; m < WG_FPT / 4; ++m) {
        const int cs = r0 + h + 4 * m, co = c0 + h + 4 * m;
        if (VEC) {
          es[q][m] = *reinterpret_cast<const float4*>(srow + (cs < d ? cs : 0));
          eo[q][m] = *reinterpret_cast<const float4*>(orow + (co < d ? co : 0));
        } else {
          es[q][m] = make_float4(srow[cs < d ? cs : 0], srow[cs + 1 < d ? cs + 1 : 0],
                                 srow[cs + 2 < d ? cs + 2 : 0], srow[cs + 3 < d ? cs + 3 : 0]);
          eo[q][m] = make_float4(orow[co < d ? co : 0], orow[co + 1 < d ? co + 1 : 0],
                                 orow[co + 2 < d ? co + 2 : 0], orow[co + 3 < d ? co + 3 : 0]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < WG_PF; ++q) {
      const int b = g0 + q;
      if (b >= nch) break;
      const int buf = b & 1;
#pragma unroll
      for (int m = 0; m < WG_FPT / 4; ++m) {   // coef-scaled E[s], E[o]; zero past d
        const int cs = r0 + h + 4 * m, co = c0 + h + 4 * m;
        float4 a = es[q][m], o = eo[q][m];
        const float cur_c = nc[q];
        a.x = cs + 0 < d ? cur_c * a.x : 0.0f;
        a.y = cs + 1 < d ? cur_c * a.y : 0.0f;
        a.z = cs + 2 < d ? cur_c * a.z : 0.0f;
        a.w = cs + 3 < d ? cur_c * a.w : 0.0f;
        o.x = co + 0 < d ? o.x : 0.0f;
        o.y = co + 1 < d ? o.y : 0.0f;
        o.z = co + 2 < d ? o.z : 0.0f;
        o.w = co + 3 < d ? o.w : 0.0f;
        *reinterpret_cast<float4*>(&sEs[buf][it][h + 4 * m]) = a;
        *reinterpret_cast<float4*>(&sEo[buf][it][h + 4 * m]) = o;
      }
      __syncthreads();   // (also: every wave is done with buf's use two chunks ago)
      const int mm = min(WG_CH, cnt - b * WG_CH);   // items past mm are zero (coef 0)
      // A[row i][k = item] = coef Es[item][i], B[k = item][col j] = Eo[item][j]
      for (int k0 = 0; k0 < mm; k0 += 4) {
        const int ik = k0 + (l >> 4);
        const float av_ = sEs[buf][ik][16 * wave + (l & 15)];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av_, sEo[buf][ik][16 * j + (l & 15)],
                                                        acc[j], 0, 0, 0);
      }
    }
  }
  // D[row 4g + reg][col] of accumulator j (os / in above: out-of-range
  // elements read a clamped in-range address and are not stored)
  if (!APPLY) {
#pragma unroll
    for (int e = 0; e < 16; ++e)
      if (in[e]) accW.sum[os[e]] = acc[e >> 2][e & 3];
    return;
  }
  // same step as k_apply_wide (skge/param.py:115-155); every load of the
  // tile issued before any of it is used
  const float div = wa.fdiv > 0.0f ? wa.fdiv : (float)cnt;
  const bool ada = wa.opt == OPT_ADAGRAD;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const float g = (acc[e >> 2][e & 3] + wa.rin * pv[e]) / div + wa.rout * pv[e];
    float w;
    if (ada) {
      av[e] = av[e] + g * g;
      w = pv[e] - (wa.lr * g) / fmaxf(sqrtf(av[e]), 1e-7f);
    } else {
      w = pv[e] - wa.lr * g;
    }
    if (in[e]) {
      wa.W[os[e]] = w;
      if (ada) wa.A[os[e]] = av[e];
    }
  }
}

// ---- split-K dW (rs_wsplit > 1) ----
// k_rescal_wgrad_part: one workgroup per (relation, 64 x 64 tile, split s);
// the tile's item groups g = s, s + splits, ... (WG_PF chunks of WG_CH items
// each, every load of a group in flight together), contracted as in
// k_rescal_wgrad_mfma but through one LDS buffer (a workgroup walks one group
// at the reference's batch size, so double buffering buys nothing and halving
// the LDS lets more workgroups be resident); the partial tile is stored whole.
static_assert(WS_TILE == WG_T && WS_GROUP == WG_PF * WG_CH, "split-K group geometry");
// workgroup `bid` of the split-K dW grid (k_rescal_wgrad_part,
// k_rescal_front_fused); coef: the items' dW coefficients in bucket order
constexpr int WPART_LDS_FLOATS = 2 * WG_CH * (WG_T + 4);
// COMB: the combined dW of deduplicated buckets (RescalWs::o2): items are
// product 1's rows, A = E_s unscaled, B = coef E_o + E_o2
// IF: one split, and the tile's W step written into the other buffer (WFront)
// instead of the partial tile; a relation without items copies its tile over
template <bool VEC, bool COMB = false, bool IF = false>
__device__ __forceinline__ void rescal_wgrad_part_body(const float* __restrict__ E, int d,
                                                       const RescalWs& ws,
                                                       const float* __restrict__ coef, int splits,
                                                       int bid, float (*sEs)[WG_T + 4],
                                                       float (*sEo)[WG_T + 4],
                                                       const WFront& wf = WFront{}) {
  const int nt = (d + WG_T - 1) / WG_T;
  const int blk = bid / splits, sp = bid - (bid / splits) * splits;
  const int p = blk / (nt * nt);
  const int rem = blk - p * nt * nt;
  const int rt = rem / nt, ct = rem - (rem / nt) * nt;
  const int tid = threadIdx.x, l = lane_id(), wave = tid >> 6;
  const int off = ws.rel_off[p], cntb = ws.rel_off[p + 1] - off;
  const int cnt = COMB ? ws.n01[p] : cntb;
  const int nch = (cnt + WG_CH - 1) / WG_CH, ngr = (nch + WG_PF - 1) / WG_PF;
  const int r0 = rt * WG_T, c0 = ct * WG_T;
  // IF: the W updater's operands, element e = 4 j + reg of the tile: row r0 +
  // 16 wave + 4 (l >> 4) + reg, column c0 + 16 j + (l & 15) (as
  // k_rescal_wgrad_mfma); loaded after the contraction (held across it they
  // would cost the launch a wave per SIMD)
  const bool ada = wf.opt == OPT_ADAGRAD;
  auto w_elem = [&](int e, size_t& o) {
    const int r = r0 + 16 * wave + 4 * (l >> 4) + (e & 3), cc = c0 + 16 * (e >> 2) + (l & 15);
    o = (size_t)p * d * d + (size_t)(r < d ? r : 0) * d + (cc < d ? cc : 0);
    return r < d && cc < d;
  };
  if (sp >= ngr) {   // no group for this split (the finishing kernel knows)
    if (IF && cnt == 0) {   // relation not in the batch: W_{b+1}[p] = W_b[p]
      const int cur = *wf.cur;
      const float* Wr = cur ? wf.W1 : wf.W0;
      const float* Ar = cur ? wf.A1 : wf.A0;
      float* Ww = cur ? wf.W0 : wf.W1;
      float* Aw = cur ? wf.A0 : wf.A1;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        size_t o;
        if (w_elem(e, o)) {
          Ww[o] = Wr[o];
          if (ada) Aw[o] = Ar[o];
        }
      }
    }
    return;
  }
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  const int it = tid / WG_TPI, h = (tid % WG_TPI) * WG_FPT;
  for (int gr = sp; gr < ngr; gr += splits) {
    const int g0 = gr * WG_PF;
    int ns[WG_PF], no[WG_PF], no2[WG_PF];
    float nc[WG_PF];
#pragma unroll
    for (int q = 0; q < WG_PF; ++q) {
      const int i = (g0 + q) * WG_CH + it;
      const int at = off + (i < cnt ? i : cnt - 1);
      ns[q] = ws.sorted_s[at];
      no[q] = ws.sorted_o[at];
      nc[q] = i < cnt ? coef[at] : 0.0f;
      if (COMB) no2[q] = i < cnt ? ws.o2[at] : -1;
    }
    float4 es[WG_PF][WG_FPT / 4], eo[WG_PF][WG_FPT / 4], eo2[WG_PF][WG_FPT / 4];
#pragma unroll
    for (int q = 0; q < WG_PF; ++q) {
      const float* srow = E + (size_t)ns[q] * d;
      const float* orow = E + (size_t)no[q] * d;
      const float* o2row = E + (size_t)(COMB && no2[q] >= 0 ? no2[q] : 0) * d;
#pragma unroll
      for (int m = 0; m < WG_FPT / 4; ++m) {
        const int cs = r0 + h + 4 * m, co = c0 + h + 4 * m;
        if (VEC) {
          es[q][m] = *reinterpret_cast<const float4*>(srow + (cs < d ? cs : 0));
          eo[q][m] = *reinterpret_cast<const float4*>(orow + (co < d ? co : 0));
          if (COMB) eo2[q][m] = *reinterpret_cast<const float4*>(o2row + (co < d ? co : 0));
        } else {
          es[q][m] = make_float4(srow[cs < d ? cs : 0], srow[cs + 1 < d ? cs + 1 : 0],
                                 srow[cs + 2 < d ? cs + 2 : 0], srow[cs + 3 < d ? cs + 3 : 0]);
          eo[q][m] = make_float4(orow[co < d ? co : 0], orow[co + 1 < d ? co + 1 : 0],
                                 orow[co + 2 < d ? co + 2 : 0], orow[co + 3 < d ? co + 3 : 0]);
          if (COMB)
            eo2[q][m] = make_float4(o2row[co < d ? co : 0], o2row[co + 1 < d ? co + 1 : 0],
                                    o2row[co + 2 < d ? co + 2 : 0], o2row[co + 3 < d ? co + 3 : 0]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < WG_PF; ++q) {
      const int b = g0 + q;
      if (b >= nch) break;
      __syncthreads();   // every wave is done with the buffer's previous chunk
#pragma unroll
      for (int m = 0; m < WG_FPT / 4; ++m) {   // coef-scaled E[s], E[o]; zero past d
        const int cs = r0 + h + 4 * m, co = c0 + h + 4 * m;
        float4 a = es[q][m], o = eo[q][m];
        const float cur_c = nc[q];
        if (COMB) {   // A = E_s, B = coef E_o + E_o2
          const bool two = no2[q] >= 0;
          const float4 o2 = eo2[q][m];
          a.x = cs + 0 < d ? a.x : 0.0f;
          a.y = cs + 1 < d ? a.y : 0.0f;
          a.z = cs + 2 < d ? a.z : 0.0f;
          a.w = cs + 3 < d ? a.w : 0.0f;
          o.x = co + 0 < d ? cur_c * o.x + (two ? o2.x : 0.0f) : 0.0f;
          o.y = co + 1 < d ? cur_c * o.y + (two ? o2.y : 0.0f) : 0.0f;
          o.z = co + 2 < d ? cur_c * o.z + (two ? o2.z : 0.0f) : 0.0f;
          o.w = co + 3 < d ? cur_c * o.w + (two ? o2.w : 0.0f) : 0.0f;
        } else {
          a.x = cs + 0 < d ? cur_c * a.x : 0.0f;
          a.y = cs + 1 < d ? cur_c * a.y : 0.0f;
          a.z = cs + 2 < d ? cur_c * a.z : 0.0f;
          a.w = cs + 3 < d ? cur_c * a.w : 0.0f;
          o.x = co + 0 < d ? o.x : 0.0f;
          o.y = co + 1 < d ? o.y : 0.0f;
          o.z = co + 2 < d ? o.z : 0.0f;
          o.w = co + 3 < d ? o.w : 0.0f;
        }
        *reinterpret_cast<float4*>(&sEs[it][h + 4 * m]) = a;
        *reinterpret_cast<float4*>(&sEo[it][h + 4 * m]) = o;
      }
      __syncthreads();
      const int mm = min(WG_CH, cnt - b * WG_CH);
      for (int k0 = 0; k0 < mm; k0 += 4) {
        const int ik = k0 + (l >> 4);
        const float av_ = sEs[ik][16 * wave + (l & 15)];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av_, sEo[ik][16 * j + (l & 15)], acc[j], 0,
                                                        0, 0);
      }
    }
  }
  if (IF) {   // the W updater's step (skge/param.py:115-155) into the other buffer
    const int cur = *wf.cur;
    const float* Wr = cur ? wf.W1 : wf.W0;
    const float* Ar = cur ? wf.A1 : wf.A0;
    float* Ww = cur ? wf.W0 : wf.W1;
    float* Aw = cur ? wf.A0 : wf.A1;
    float pv[16], av[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {   // every load of the tile issued before any use
      size_t o;
      w_elem(e, o);
      pv[e] = Wr[o];
      av[e] = ada ? Ar[o] : 0.0f;
    }
    const float div = wf.fdiv > 0.0f ? wf.fdiv : (float)cntb;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float g = (acc[e >> 2][e & 3] + wf.rin * pv[e]) / div + wf.rout * pv[e];
      float w, a2 = av[e];
      if (ada) {
        a2 = av[e] + g * g;
        w = pv[e] - (wf.lr * g) / fmaxf(sqrtf(a2), 1e-7f);
      } else {
        w = pv[e] - wf.lr * g;
      }
      size_t o;
      if (w_elem(e, o)) {
        Ww[o] = w;
        if (ada) Aw[o] = a2;
      }
    }
    return;
  }
  // D[row 16 wave + 4 (l >> 4) + reg][col 16 j + (l & 15)] -> the partial tile
  float* out = ws.wpart + ((size_t)blk * splits + sp) * (WG_T * WG_T);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg)
      out[(16 * wave + 4 * (l >> 4) + reg) * WG_T + 16 * j + (l & 15)] = acc[j][reg];
}

template <bool VEC>
__global__ __launch_bounds__(256) void k_rescal_wgrad_part(const float* __restrict__ E, int d,
                                                           RescalWs ws, int splits) {
  __shared__ float sEs[WG_CH][WG_T + 4];
  __shared__ float sEo[WG_CH][WG_T + 4];
  rescal_wgrad_part_body<VEC>(E, d, ws, ws.coef, splits, (int)blockIdx.x, sEs, sEo);
}

// ---------------------------------------------------------------------------
// The device pair loop's fused front (Linear activation): with g = 1 the dW
// coefficients do not depend on the scores (gp = -1 per pair the positive is
// in, gn = +1; rescal.py:113-125, 275), so they are written when the epoch's
// buckets are built (ws.ecoef) and batch b's dW contraction needs only E --
// the same operand the GEMMs read.  ONE launch runs both: the first nwg
// workgroups are the split-K dW grid (partial tiles into ws.wpart), the rest
// the GEMM grid; the W step (k_rescal_wgrad_fin, gated on the batch's
// violations) follows the scatter.  The LDS is one buffer carved per role.
// Same arithmetic, same k order as the unfused kernels: bitwise the same W.
// ---------------------------------------------------------------------------
constexpr int front_lds_floats(int ks) {
  return gemm_lds_floats(ks) > WPART_LDS_FLOATS ? gemm_lds_floats(ks) : WPART_LDS_FLOATS;
}
template <bool VEC, bool COMB, bool IF, int KS>
__global__ __launch_bounds__(256) void k_rescal_front_fused(const float* __restrict__ E,
                                                            const float* __restrict__ W, int d,
                                                            RescalWs ws, int splits, int nwg,
                                                            int order, WFront wf) {
  __shared__ __attribute__((aligned(16))) float lds[front_lds_floats(KS)];
  const int bid = (int)blockIdx.x, ng = (int)gridDim.x - nwg;
  // role of workgroup bid: order 0 = the dW grid first, 1 = the GEMM grid
  // first, r >= 2 = one dW workgroup every r workgroups (while they last)
  int wid = -1, gid;
  if (order == 0) {
    if (bid < nwg) wid = bid;
    gid = bid - nwg;
  } else if (order == 1) {
    if (bid >= ng) wid = bid - ng;
    gid = bid;
  } else {
    const int k = bid / order;
    if (bid - k * order == 0 && k < nwg) wid = k;
    gid = bid - min((bid + order - 1) / order, nwg);
  }
  if (wid >= 0) {
    rescal_wgrad_part_body<VEC, COMB, IF>(E, d, ws, ws.ecoef, splits, wid,
                                reinterpret_cast<float(*)[WG_T + 4]>(lds),
                                reinterpret_cast<float(*)[WG_T + 4]>(lds + WG_CH * (WG_T + 4)), wf);
  } else {
    float* sb = lds + 2 * RT_ITEMS * (KS + 4);
    int* si = reinterpret_cast<int*>(sb + 2 * rs_sbn(KS));
    const float* Wb = IF && *wf.cur ? wf.W1 : W;   // W_b's buffer
    rescal_gemm_body<VEC, KS>(E, Wb, d, ws, gid,
                              reinterpret_cast<float(*)[RT_ITEMS][KS + 4]>(lds),
                              reinterpret_cast<float(*)[rs_sbn(KS)]>(sb), si, si + RT_ITEMS,
                              si + 2 * RT_ITEMS, si + 3 * RT_ITEMS);
  }
}

// k_rescal_wgrad_fin: one workgroup per (relation, 64 x 64 tile): the tile's
// partials summed in split order, then the accumulator write (slot map as
// k_rescal_wgrad_mfma) or the W updater's step (the same arithmetic as its
// APPLY epilogue)
template <bool APPLY>
__global__ __launch_bounds__(256) void k_rescal_wgrad_fin(int d, RescalWs ws, Accum accW,
                                                          WApply wa, int splits) {
  const int nt = (d + WG_T - 1) / WG_T;
  const int blk = blockIdx.x;
  const int p = blk / (nt * nt);
  const int rem = blk - p * nt * nt;
  const int rt = rem / nt, ct = rem - (rem / nt) * nt;
  const int tid = threadIdx.x;
  const int off = ws.rel_off[p], cnt = ws.rel_off[p + 1] - off;
  const int gv = APPLY && wa.gate != nullptr ? *wa.gate : 1;   // (loaded with rel_off)
  if (!APPLY && rem == 0 && tid == 0) {   // slot p (skge_hip.h slot map)
    if (accW.touched) accW.touched[p] = cnt > 0 ? p : -1;
    accW.cnt[p] = cnt;
  }
  if (cnt == 0) return;
  const bool upd = gv != 0;
  if (APPLY && !upd) return;   // the model returned None: no update
  if (APPLY && rem == 0 && tid == 0 && wa.opt == OPT_ADAGRAD && wa.ucnt)
    atomicAdd(wa.ucnt + (p), 1);   // updateCounts, skge/param.py:149-150
  const int nch = (cnt + WG_CH - 1) / WG_CH, ngr = (nch + WG_PF - 1) / WG_PF;
  const int nsp = min(splits, ngr);
  const float* part = ws.wpart + (size_t)blk * splits * (WG_T * WG_T);
  const bool ada = wa.opt == OPT_ADAGRAD;
  const float div = wa.fdiv > 0.0f ? wa.fdiv : (float)cnt;
  constexpr int EPT = WG_T * WG_T / 256;   // 16 elements per thread, 4 float4
  float sum[EPT], pw[EPT], aw[EPT];
  size_t os[EPT];
  bool in[EPT];
#pragma unroll
  for (int k = 0; k < EPT / 4; ++k) {   // elements 4 (tid + 256 k) + m: row e / 64, col e % 64
    const int e = 4 * (tid + 256 * k), r = rt * WG_T + e / WG_T, c = ct * WG_T + e % WG_T;
    const float4 v = *reinterpret_cast<const float4*>(part + e);
    sum[4 * k] = v.x;
    sum[4 * k + 1] = v.y;
    sum[4 * k + 2] = v.z;
    sum[4 * k + 3] = v.w;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      in[4 * k + m] = r < d && c + m < d;
      os[4 * k + m] = (size_t)p * d * d + (size_t)(r < d ? r : 0) * d + (c + m < d ? c + m : 0);
    }
  }
  if (APPLY) {   // the W updater's operands, in flight with the partials
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      pw[e] = wa.W[os[e]];
      aw[e] = ada ? wa.A[os[e]] : 0.0f;
    }
  }
  for (int q = 1; q < nsp; ++q) {   // split order: deterministic sums
#pragma unroll
    for (int k = 0; k < EPT / 4; ++k) {
      const float4 v = *reinterpret_cast<const float4*>(part + (size_t)q * (WG_T * WG_T) +
                                                        4 * (tid + 256 * k));
      sum[4 * k] += v.x;
      sum[4 * k + 1] += v.y;
      sum[4 * k + 2] += v.z;
      sum[4 * k + 3] += v.w;
    }
  }
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    if (!in[e]) continue;
    if (!APPLY) {
      accW.sum[os[e]] = sum[e];
      continue;
    }
    // same step as k_rescal_wgrad_mfma's APPLY epilogue (skge/param.py:115-155)
    const float g = (sum[e] + wa.rin * pw[e]) / div + wa.rout * pw[e];
    if (ada) {
      const float a2 = aw[e] + g * g;
      wa.W[os[e]] = pw[e] - (wa.lr * g) / fmaxf(sqrtf(a2), 1e-7f);
      wa.A[os[e]] = a2;
    } else {
      wa.W[os[e]] = pw[e] - wa.lr * g;
    }
  }
}

}  // namespace skge

using namespace skge;

size_t skge_rescal_mfma_ws_bytes(int n, int M, int d) {
  return rescal_ws_layout(n, M, d, nullptr, nullptr);
}

bool skge_rescal_mfma_ok(int d, int M) {
  return d >= 1 && d <= RS_MAX_D && M >= 1 && M <= RS_MAX_M;
}

// bucket the n = na + nb triples (list a, then list b) by relation and run the
// two GEMMs (WE^T, EW, partial scores)
static int rescal_front(hipStream_t st, const skge_table_t* ent, const skge_table_t* rel, int d,
                        const int* a, int na, const int* b, int n, const RescalWs& ws,
                        bool bucketed = false) {
  const int M = rel->rows;
  if (bucketed) {
    // the epoch's buckets were built up front (rescal_epoch_bucket)
  } else if (M <= SB_MAXM && n <= SB_MAXN) {
    hipLaunchKernelGGL(k_rs_bucket_small, dim3(1), dim3(1024), 0, st, a, b, na, n, M, ws);
  } else {
    const int nchunks = (n + 63) / 64;
    if (M > 64)   // (k_rs_count writes whole rows itself for M <= 64)
      SKGE_CHECK_HIP(hipMemsetAsync(ws.chunk, 0, (size_t)nchunks * M * sizeof(int), st));
    const int cblocks = (nchunks + 3) / 4;
    hipLaunchKernelGGL(k_rs_count, dim3(cblocks), dim3(256), 0, st, a, b, na, n, M, ws);
    hipLaunchKernelGGL(k_rs_scan, dim3(1), dim3(1024), (size_t)(2 * M + 1) * sizeof(int), st, n,
                       M, ws);
    hipLaunchKernelGGL(k_rs_scatter, dim3(cblocks), dim3(256), 0, st, a, b, na, n, M, ws);
  }
  const int ncb = (d + GC - 1) / GC;
  const dim3 ggrid((unsigned)((ws.npos > 0 ? rs_tmax_dedup(ws.npos, M) * ncb
                                           : rs_tmax(n, M) * 2 * ncb) * ws.gks));
  if ((d & 3) == 0)
    hipLaunchKernelGGL((k_rescal_gemm<true>), ggrid, dim3(256), 0, st, ent->param, rel->param, d,
                       ws);
  else
    hipLaunchKernelGGL((k_rescal_gemm<false>), ggrid, dim3(256), 0, st, ent->param, rel->param,
                       d, ws);
  SKGE_CHECK_LAUNCH("rescal mfma front");
  return SKGE_OK;
}

// dW per relation; apply_gate != nullptr: also the W update of rel's updater
// (fused apply, gated on *apply_gate unless it points at a constant 1 --
// pass rel->gate semantics through `gate`)
static void rescal_wgrad_launch(hipStream_t st, const skge_table_t* ent,
                                const skge_table_t* rel, int d, const RescalWs& ws, bool apply,
                                const int* gate, int n) {
  const int nt = (d + WG_T - 1) / WG_T;
  const dim3 grid((unsigned)((long long)rel->rows * nt * nt));
  WApply wa = {};
  if (apply) {
    wa.W = rel->param;
    wa.A = rel->state;
    wa.opt = rel->opt;
    wa.lr = rel->lr;
    wa.rin = rel->rin;
    wa.rout = rel->rout;
    wa.fdiv = rel->fixed_div;
    wa.gate = gate;
    wa.ucnt = rel->upd_count;
  }
  const int splits = ws.wpart ? rs_wsplit(n, rel->rows, d) : 1;
  if (splits > 1) {   // split-K: partial tiles, then the sum + accumulator write / W step
    const dim3 pgrid(grid.x * (unsigned)splits);
    if ((d & 3) == 0)
      hipLaunchKernelGGL((k_rescal_wgrad_part<true>), pgrid, dim3(256), 0, st, ent->param, d, ws,
                         splits);
    else
      hipLaunchKernelGGL((k_rescal_wgrad_part<false>), pgrid, dim3(256), 0, st, ent->param, d, ws,
                         splits);
    if (apply)
      hipLaunchKernelGGL((k_rescal_wgrad_fin<true>), grid, dim3(256), 0, st, d, ws, accum_of(rel),
                         wa, splits);
    else
      hipLaunchKernelGGL((k_rescal_wgrad_fin<false>), grid, dim3(256), 0, st, d, ws,
                         accum_of(rel), wa, splits);
    return;
  }
  if (apply) {
    if ((d & 3) == 0)
      hipLaunchKernelGGL((k_rescal_wgrad_mfma<true, true>), grid, dim3(256), 0, st, ent->param, d,
                         ws, accum_of(rel), wa);
    else
      hipLaunchKernelGGL((k_rescal_wgrad_mfma<true, false>), grid, dim3(256), 0, st, ent->param,
                         d, ws, accum_of(rel), wa);
  } else {
    if ((d & 3) == 0)
      hipLaunchKernelGGL((k_rescal_wgrad_mfma<false, true>), grid, dim3(256), 0, st, ent->param,
                         d, ws, accum_of(rel), wa);
    else
      hipLaunchKernelGGL((k_rescal_wgrad_mfma<false, false>), grid, dim3(256), 0, st, ent->param,
                         d, ws, accum_of(rel), wa);
  }
}

#define SKGE_KM_SWITCH(KERNEL, ...)                                             \
  switch (km_for(d)) {                                                          \
    case 1: hipLaunchKernelGGL((KERNEL<1>), __VA_ARGS__); break;                \
    case 2: hipLaunchKernelGGL((KERNEL<2>), __VA_ARGS__); break;                \
    case 3: hipLaunchKernelGGL((KERNEL<3>), __VA_ARGS__); break;                \
    case 4: hipLaunchKernelGGL((KERNEL<4>), __VA_ARGS__); break;                \
    case 8: hipLaunchKernelGGL((KERNEL<8>), __VA_ARGS__); break;                \
    case 16: hipLaunchKernelGGL((KERNEL<16>), __VA_ARGS__); break;              \
    default: set_error("d=%d unsupported on the MFMA path", d); return SKGE_ENOTSUP; \
  }

// the RESCAL pairwise gradient (entity accumulator, W accumulator) on MFMA
int skge_rescal_pair_grad_mfma(hipStream_t st, int af, const skge_table_t* ent,
                               const skge_table_t* rel, int d, const int* pos, const int* neg,
                               int P, float margin, void* workspace, size_t ws_bytes,
                               float* pscore, float* nscore, int* nviol, bool apply_w) {
  RescalWs ws;
  const size_t need = rescal_ws_layout(2 * P, rel->rows, d, workspace, &ws);
  SKGE_CHECK_ARG(workspace && ws_bytes >= need, "RESCAL workspace needs %zu bytes", need);
  SKGE_CHECK_ARG(apply_w || (rel->acc_sum && rel->acc_cnt), "W accumulator missing");
  SKGE_CHECK_ARG(!apply_w || nviol, "the fused W update is gated on nviol");
  int rc = rescal_front(st, ent, rel, d, pos, P, neg, 2 * P, ws);
  if (rc) return rc;
  const int blocks = std::max(1, std::min((P + 3) / 4, 16384));
  const Accum aE = accum_of(ent);
  SKGE_KM_SWITCH(k_rescal_scatter, dim3(blocks), dim3(256), 0, st, pos, neg, P, d, af, margin, ws,
                 aE, pscore, nscore, nviol)
  rescal_wgrad_launch(st, ent, rel, d, ws, apply_w, nviol, 2 * P);
  SKGE_CHECK_LAUNCH("rescal mfma pair grad");
  return SKGE_OK;
}

// the device pair loop's RESCAL batch (k_rescal_pos_scatter): lists a = the
// count positives, b = their 2 count negatives (k_pairs_of_epoch's RESCAL
// form), records for the scatter; W updated in place, entity rows accumulated
int skge_rescal_pos_grad_mfma(hipStream_t st, int af, const skge_table_t* ent,
                              const skge_table_t* rel, int d, const int* pos, const int* neg,
                              const int4* rec, const int* rec_n1, long long start, int count,
                              float margin, void* workspace, size_t ws_bytes, int* nviol) {
  int rc;
  if ((rc = check_table(ent, "ent", true)) || (rc = check_table(rel, "rel", false)) ||
      (rc = check_f32(ent, "ent")) || (rc = check_f32(rel, "rel")) ||
      (rc = check_single(ent, "ent")) || (rc = check_single(rel, "rel")) ||
      (rc = check_slots(ent, 4ll * count, "ent")) || (rc = check_slots(rel, rel->rows, "W")))
    return rc;
  SKGE_CHECK_ARG(ent->width == d && rel->width == d * d, "RESCAL table widths");
  SKGE_CHECK_ARG(af >= 0 && af <= 3, "unknown activation %d", af);
  SKGE_CHECK_ARG(rel->opt == SKGE_SGD || rel->state, "AdaGrad needs state");
  SKGE_CHECK_ARG(nviol, "the fused W update is gated on nviol");
  RescalWs ws;
  const size_t need = rescal_ws_layout(3 * count, rel->rows, d, workspace, &ws);
  SKGE_CHECK_ARG(workspace && ws_bytes >= need, "RESCAL workspace needs %zu bytes", need);
  rc = rescal_front(st, ent, rel, d, pos, count, neg, 3 * count, ws);
  if (rc) return rc;
  const int blocks = std::max(1, std::min((count + 3) / 4, 16384));
  SKGE_KM_SWITCH(k_rescal_pos_scatter, dim3(blocks), dim3(256), 0, st, rec, rec_n1, start, count,
                 d, af, margin, ws, accum_of(ent), nviol)
  rescal_wgrad_launch(st, ent, rel, d, ws, true, nviol, 3 * count);
  SKGE_CHECK_LAUNCH("rescal positive grad");
  return SKGE_OK;
}

// ---- epoch-level bucketing for the device pair loop ----
// workspace: the shared part (spart, coef, WE, EW for one batch of n = 3 bs
// items) once, then nb bucket slices of `stride` bytes (chunk counts,
// offsets, items, tiles, sorted rows, positions), batch b at slice b
static size_t rescal_epoch_layout(int bs, int nb, int M, int d, void* base, RescalWs* ws0,
                                  long long* stride) {
  // (sized for both enumerations: deduplicated blocks start on chunk boundaries)
  const int n = 3 * bs, nchunks = 3 * ((bs + 63) / 64);
  const int tmax = std::max(rs_tmax(n, M), rs_tmax_dedup(bs, M));
  size_t off = 0;
  char* p = (char*)base;
  auto take = [&](size_t bytes) {
    char* q = p ? p + off : nullptr;
    off += al256(bytes);
    return q;
  };
  RescalWs w;
  const int gks = rs_gks(d);
  w.gks = gks;
  w.part_stride = (long long)n * d;
  w.spart_stride = (long long)n * ((d + GC - 1) / GC);
  w.spart = (float*)take((size_t)gks * n * ((d + GC - 1) / GC) * 4);
  w.coef = (float*)take((size_t)n * 4);
  w.WE = (float*)take((size_t)gks * n * d * 4);
  w.EW = (float*)take((size_t)gks * n * d * 4);
  // batches of fewer items use fewer splits; the fused front (Linear) needs
  // partial tiles even at one split
  const size_t wpb = std::max(rs_wpart_bytes(n, M, d), rs_front_wpart_bytes(n, M, d));
  w.wpart = wpb ? (float*)take(wpb) : nullptr;
  // the row-grouped apply's partial sums of multi-chunk rows (k_rescal_fold)
  w.part = (float*)take((size_t)4 * bs * d * 4);
  w.pcnt = (int*)take((size_t)4 * bs * 4);
  // the in-front W step's second buffers (up to 256 MB)
  const bool wb = (size_t)M * d * d * 8 <= (256u << 20);
  w.W1 = wb ? (float*)take((size_t)M * d * d * 4) : nullptr;
  w.A1 = wb ? (float*)take((size_t)M * d * d * 4) : nullptr;
  w.wcur = wb ? (int*)take(4) : nullptr;
  const size_t s0 = off;
  w.chunk = (int*)take((size_t)nchunks * M * 4);
  w.rel_off = (int*)take((size_t)(M + 1) * 4);
  w.items = (int*)take((size_t)n * 4);
  w.tile_rel = (int*)take((size_t)tmax * 4);
  w.tile_start = (int*)take((size_t)tmax * 4);
  w.tile_cnt = (int*)take((size_t)tmax * 4);
  w.ntiles = (int*)take(8);   // tiles; deduplicated: also the product-0 tiles
  w.sorted_s = (int*)take((size_t)n * 4);
  w.sorted_o = (int*)take((size_t)n * 4);
  w.bpos = (int*)take((size_t)n * 4);
  w.ecoef = (float*)take((size_t)n * 4);
  w.s2 = (int*)take((size_t)n * 4);
  w.o2 = (int*)take((size_t)n * 4);
  w.n01 = (int*)take((size_t)M * 4);
  // the row grouping of the batch's 4 bs entity slots (k_rs_rows_ep)
  w.urec = (int4*)take((size_t)4 * bs * 16);
  w.rowctr = (int*)take((size_t)4 * bs * 4);
  w.nuniq = (int*)take(4);
  w.vword = (unsigned long long*)take(8);
  w.npos = 0;   // (set per batch: rs_batch_view)
  const size_t slice = off - s0;
  if (ws0) *ws0 = w;
  if (stride) *stride = (long long)slice;
  return s0 + (size_t)nb * slice;
}

bool rescal_epoch_ok(int M) { return M <= 64; }

size_t rescal_epoch_ws_bytes(int bs, int nb, int M, int d) {
  return rescal_epoch_layout(bs, nb, M, d, nullptr, nullptr, nullptr);
}

static RescalEpoch rescal_epoch_view(void* ws, long long T, int bs, int nb, int M, int d) {
  RescalEpoch e;
  rescal_epoch_layout(bs, nb, M, d, ws, &e.ws0, &e.stride);
  e.T = T;
  e.bs = bs;
  e.nb = nb;
  e.M = M;
  e.dedup = rs_dedup_on() ? 1 : 0;
  e.cpb = e.dedup ? 3 * ((bs + 63) / 64) : (3 * bs + 63) / 64;
  return e;
}

// every batch's buckets of the epoch, three launches (dedup lists: pos [T][3],
// neg [T][2][3], k_pairs_of_epoch's RESCAL form)
bool rs_rows_ok(int bs) { return 4ll * bs <= RS_ROWS_MAX; }

int rescal_epoch_bucket(hipStream_t st, const int* pos, const int* neg, long long T, int bs, int nb,
                        int M, int d, void* ws, const int4* rec, const int* rec_n1) {
  SKGE_CHECK_ARG(rescal_epoch_ok(M), "epoch bucketing needs M <= 64");
  const RescalEpoch e = rescal_epoch_view(ws, T, bs, nb, M, d);
  const long long waves = (long long)nb * e.cpb;
  const unsigned blocks = (unsigned)((waves + 3) / 4);
  hipLaunchKernelGGL(k_rs_count_ep, dim3(blocks), dim3(256), 0, st, pos, neg, e);
  hipLaunchKernelGGL(k_rs_scan_ep, dim3((unsigned)nb), dim3(1024),
                     (size_t)(e.dedup ? 8 * M + 2 : 2 * M + 1) * sizeof(int), st, e);
  hipLaunchKernelGGL(k_rs_scatter_ep, dim3(blocks), dim3(256), 0, st, pos, neg, e);
  if (rec && rec_n1 && rs_rows_ok(bs))   // the batches' entity rows grouped (k_rescal_fold)
    hipLaunchKernelGGL(k_rs_rows_ep, dim3((unsigned)nb), dim3(1024), 0, st, rec, rec_n1, e);
  SKGE_CHECK_LAUNCH("rescal epoch bucketing");
  return SKGE_OK;
}

// the device pair loop's RESCAL batch b on pre-built buckets
int skge_rescal_pos_grad_mfma_ep(hipStream_t st, int af, const skge_table_t* ent,
                                 const skge_table_t* rel, int d, const int4* rec,
                                 const int* rec_n1, long long T, int bs, int nb, int b,
                                 float margin, void* ws, int* nviol, WStep* wstep) {
  int rc;
  if (wstep) wstep->part = nullptr;
  const long long start = (long long)b * bs;
  const int count = (int)(start + bs <= T ? bs : T - start);
  if ((rc = check_table(ent, "ent", true)) || (rc = check_table(rel, "rel", false)) ||
      (rc = check_f32(ent, "ent")) || (rc = check_f32(rel, "rel")) ||
      (rc = check_single(ent, "ent")) || (rc = check_single(rel, "rel")) ||
      (rc = check_slots(ent, 4ll * count, "ent")) || (rc = check_slots(rel, rel->rows, "W")))
    return rc;
  SKGE_CHECK_ARG(ent->width == d && rel->width == d * d, "RESCAL table widths");
  SKGE_CHECK_ARG(af >= 0 && af <= 3, "unknown activation %d", af);
  SKGE_CHECK_ARG(rel->opt == SKGE_SGD || rel->state, "AdaGrad needs state");
  SKGE_CHECK_ARG(nviol, "the fused W update is gated on nviol");
  SKGE_CHECK_ARG(rescal_epoch_ok(rel->rows), "epoch bucketing needs M <= 64");
  const RescalEpoch e = rescal_epoch_view(ws, T, bs, nb, rel->rows, d);
  RescalWs w = e.ws0;   // host-side batch view (same arithmetic as rs_batch_view)
  const long long o = e.stride * b;
  auto sh = [o](auto* p) { return reinterpret_cast<decltype(p)>(reinterpret_cast<char*>(p) + o); };
  w.chunk = sh(w.chunk);
  w.rel_off = sh(w.rel_off);
  w.items = sh(w.items);
  w.tile_rel = sh(w.tile_rel);
  w.tile_start = sh(w.tile_start);
  w.tile_cnt = sh(w.tile_cnt);
  w.ntiles = sh(w.ntiles);
  w.sorted_s = sh(w.sorted_s);
  w.sorted_o = sh(w.sorted_o);
  w.bpos = sh(w.bpos);
  w.ecoef = sh(w.ecoef);
  w.s2 = sh(w.s2);
  w.o2 = sh(w.o2);
  w.n01 = sh(w.n01);
  w.urec = sh(w.urec);
  w.rowctr = sh(w.rowctr);
  w.nuniq = sh(w.nuniq);
  w.vword = sh(w.vword);
  w.npos = e.dedup ? count : 0;
  const int n = 3 * count, M = rel->rows;
  const int fsplits = af == AF_LINEAR ? rs_front_splits(n, M, d) : 0;
  const int blocks = std::max(1, std::min((count + 3) / 4, 16384));
  if (fsplits > 0) {   // k_rescal_front_fused: dW contraction and GEMMs in one launch
    const int nt = (d + WG_T - 1) / WG_T, ncb = (d + GC - 1) / GC;
    const int nwg = M * nt * nt * fsplits;
    const dim3 grid((unsigned)(nwg + (w.npos > 0 ? rs_tmax_dedup(count, M) * ncb
                                                  : rs_tmax(n, M) * 2 * ncb) * w.gks));
    // workgroup order of the two roles (k_rescal_front_fused): the GEMM grid
    // first (A/B on WN18 d = 200: 29.25 M vs 29.0 M triples/s with the dW
    // grid first, 29.2 M interleaving one dW workgroup in three)
    const RsForm form = rs_form();
    int order = form.order;
    if (order >= 2) {   // every dW workgroup needs a slot: order * nwg <= grid
      order = std::min<long long>(order, (long long)grid.x / nwg);
      if (order < 2) order = 0;
    }
    // combined dW: a positive's two outer products over E_s as one (form
    // "dw3": three items; the separate finishing kernel counts a relation's
    // items by its bucket)
    const bool wstep_in_apply = wstep != nullptr;
    const bool comb = w.npos > 0 && wstep_in_apply && !form.dw3;
    // the W step inside the front when every batch of the epoch has one dW
    // split (form "wapply": in the apply, from partial tiles)
    const long long last = T - (long long)(nb - 1) * bs;
    const bool infront = comb && w.wcur && !form.wapply &&
                         rs_front_splits(3 * bs, M, d) == 1 &&
                         rs_front_splits((int)(3 * last), M, d) == 1;
    WFront wf = {};
    if (infront)
      wf = WFront{w.wcur, rel->param, rel->state, w.W1, w.A1, rel->opt, rel->lr, rel->rin,
                  rel->rout, rel->fixed_div};
    const bool ks_small = bs < RS_KS_SMALL_BS;
#define SKGE_FRONT(V, C, I)                                                                  \
  do {                                                                                       \
    if (ks_small)                                                                            \
      hipLaunchKernelGGL((k_rescal_front_fused<V, C, I, KS_SMALL>), grid, dim3(256), 0, st,  \
                         ent->param, rel->param, d, w, fsplits, nwg, order, wf);             \
    else                                                                                     \
      hipLaunchKernelGGL((k_rescal_front_fused<V, C, I, KS>), grid, dim3(256), 0, st,        \
                         ent->param, rel->param, d, w, fsplits, nwg, order, wf);             \
  } while (0)
    if ((d & 3) == 0) {
      if (infront) SKGE_FRONT(true, true, true);
      else if (comb) SKGE_FRONT(true, true, false);
      else SKGE_FRONT(true, false, false);
    } else {
      if (infront) SKGE_FRONT(false, true, true);
      else if (comb) SKGE_FRONT(false, true, false);
      else SKGE_FRONT(false, false, false);
    }
#undef SKGE_FRONT
    RescalWs wsc = w;
    wsc.coef = nullptr;   // dW was formed from the bucketing's coefficients
    const WStep wstp{w.wpart, w.rel_off, comb ? w.n01 : nullptr, rel->param, rel->state,
                     rel->upd_count, nviol, M, d, fsplits, rel->opt, rel->lr, rel->rin, rel->rout,
                     rel->fixed_div, infront ? w.wcur : nullptr, w.W1, w.A1};
    // the entity rows updated by the row-grouped apply (k_rescal_fold: no
    // scatter launch, no entity atomics) where the W step is in the front and
    // the epoch's row grouping exists (form "scatter": the scatter + apply)
    if (infront && !form.scatter && w.nuniq && rs_rows_ok(bs)) {
      const FoldTab ft{ent->param, ent->state, ent->upd_count, ent->opt, ent->post, ent->lr,
                       ent->rin, ent->rout, ent->fixed_div, accum_of(ent)};
      const int nvw = (count + 255) / 256;   // violation-count workgroups, then one wave per row
      SKGE_KM_SWITCH(k_rescal_fold, dim3((unsigned)(nvw + count)), dim3(256), 0, st, rec, rec_n1,
                     start, count, d, af, margin, wsc, ft, wstp, nviol, nvw)
      *wstep = wstp;
      wstep->applied = 1;   // the caller's apply launch is not needed
      SKGE_CHECK_LAUNCH("rescal positive grad (fused front, row-grouped apply)");
      return SKGE_OK;
    }
    SKGE_KM_SWITCH(k_rescal_pos_scatter, dim3(blocks), dim3(256), 0, st, rec, rec_n1, start,
                   count, d, af, margin, wsc, accum_of(ent), nviol)
    if (wstep_in_apply) {   // the caller's entity apply runs the W step
      *wstep = wstp;
    } else {
      WApply wa = {rel->param, rel->state, rel->opt, rel->lr, rel->rin, rel->rout,
                   rel->fixed_div, nviol, rel->upd_count};
      hipLaunchKernelGGL((k_rescal_wgrad_fin<true>), dim3((unsigned)(M * nt * nt)), dim3(256), 0,
                         st, d, w, accum_of(rel), wa, fsplits);
    }
    SKGE_CHECK_LAUNCH("rescal positive grad (fused front)");
    return SKGE_OK;
  }
  rc = rescal_front(st, ent, rel, d, nullptr, count, nullptr, 3 * count, w, true);
  if (rc) return rc;
  SKGE_KM_SWITCH(k_rescal_pos_scatter, dim3(blocks), dim3(256), 0, st, rec, rec_n1, start, count,
                 d, af, margin, w, accum_of(ent), nviol)
  rescal_wgrad_launch(st, ent, rel, d, w, true, nviol, 3 * count);
  SKGE_CHECK_LAUNCH("rescal positive grad (epoch buckets)");
  return SKGE_OK;
}

// the in-front W step's epoch end: W / state back into the caller's buffers
// when the other buffer is current (k_rescal_w_sync), then cur = 0.  n = M d^2
// elements: float4 body + a scalar tail (M d^2 need not be a multiple of 4,
// e.g. d = 25, M = 7)
__global__ __launch_bounds__(256) void k_rescal_w_sync(const int* __restrict__ cur, float* W0,
                                                       float* A0, const float* __restrict__ W1,
                                                       const float* __restrict__ A1, long long n) {
  if (*cur == 0) return;
  const long long n4 = n >> 2;
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (long long i = tid; i < n4; i += (long long)gridDim.x * blockDim.x) {
    reinterpret_cast<float4*>(W0)[i] = reinterpret_cast<const float4*>(W1)[i];
    if (A0) reinterpret_cast<float4*>(A0)[i] = reinterpret_cast<const float4*>(A1)[i];
  }
  const long long t = 4 * n4 + tid;   // <= 3 tail elements, threads 0..2 of block 0
  if (t < n) {
    W0[t] = W1[t];
    if (A0) A0[t] = A1[t];
  }
}
__global__ void k_rescal_w_reset(int* cur) { *cur = 0; }

int skge::rescal_w_sync(hipStream_t st, const WStep& w) {
  if (!w.cur) return SKGE_OK;
  const long long n = (long long)w.M * w.d * w.d;
  const long long blocks = std::max<long long>(1, std::min<long long>((n / 4 + 255) / 256, 2048));
  hipLaunchKernelGGL(k_rescal_w_sync, dim3((unsigned)blocks), dim3(256), 0, st, w.cur, w.W,
                     w.A, w.W1, w.A1, n);
  hipLaunchKernelGGL(k_rescal_w_reset, dim3(1), dim3(1), 0, st, w.cur);
  SKGE_CHECK_LAUNCH("rescal W sync");
  return SKGE_OK;
}

// the RESCAL logistic gradient (rescal.py:37-76) on MFMA
int skge_rescal_triple_grad_mfma(hipStream_t st, const skge_table_t* ent,
                                 const skge_table_t* rel, int d, const int* trip,
                                 const float* ys, int T, void* workspace, size_t ws_bytes,
                                 float* score, float* loss, bool apply_w) {
  RescalWs ws;
  const size_t need = rescal_ws_layout(T, rel->rows, d, workspace, &ws);
  SKGE_CHECK_ARG(workspace && ws_bytes >= need, "RESCAL workspace needs %zu bytes", need);
  SKGE_CHECK_ARG(apply_w || (rel->acc_sum && rel->acc_cnt), "W accumulator missing");
  int rc = rescal_front(st, ent, rel, d, trip, T, trip, T, ws);
  if (rc) return rc;
  const int blocks = std::max(1, std::min((T + 3) / 4, 16384));
  const Accum aE = accum_of(ent);
  SKGE_KM_SWITCH(k_rescal_logistic, dim3(blocks), dim3(256), 0, st, trip, ys, T, d, ws, aE, score,
                 loss)
  rescal_wgrad_launch(st, ent, rel, d, ws, apply_w, rel->gate, T);
  SKGE_CHECK_LAUNCH("rescal mfma triple grad");
  return SKGE_OK;
}
