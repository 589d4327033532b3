// k_screen_valu.hip — kernel 11: the exact two-pass scan for a lone question or a handful (nq <= 8;
// BASELINE config 2: 100k × 768 f32, nq 1, k 10, and the adapter's un-batched questions), in ONE
// launch: int8 screen of the index's int8 copy on v_dot4_i32_i8, exact re-score of the rows that can
// still reach the top-k, the final merge in the last block.  When the screen cannot prove its answer
// the exact one-launch VALU search (k_scan_valu.h) rewrites it: for a lone question inside this same
// launch (round 5, below), otherwise as a gated launch that follows.
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551).
// The int8 copy and the exactness argument are kernel 10's (k_scan_screen.h): per
// 32-row tile scale s_t, per query s_y and e2 = 2 E_q / s_y (rounded up), screen score A = s_t D;
// every row of the exact top-k has A >= a_k - e2 (a_k: the k-th best A over live rows).  Here:
//   * each wave keeps the 16 best A of its rows per query (WaveList) and the best A it had to drop
//     (rejected or evicted); the block merges its four wave lists and writes a record per query:
//     its 15 best (A, row) and, in entry 15, its drop bound (everything it did not keep is <= it);
//   * the last block to finish (agent-scope arrival counter) takes a_k' = the k-th best A over the
//     records' best entries (a lower bound of a_k: distinct live rows).  If some drop bound
//     reaches a_k' - e2 a dropped row might belong to the top-k: not proven, and the exact search
//     rewrites the answer.  Otherwise every row with
//     A >= a_k' - e2 (the top-k among them, as a_k' <= a_k) is in a record, and it ranks those
//     survivors by their exact scores (f64 sum of the exact products, rounded to f32, 16 lanes per
//     row; score desc, row asc).  The exact scores come with the records: each block re-scores the
//     entries that can still survive before it arrives (its own k-th best A and the best such bound
//     other blocks posted so far bound a_k' from below; step 3), so the re-score's memory round trip
//     leaves the last block's critical path (round 5).
// No atomics on shared addresses besides the arrival counter: the bound travels in the records.
// The fallback inside the launch (lone question): the blocks that arrived before the last one wait, for
// a bounded time, for its verdict; on "not proven" every block still there, and the last block itself,
// CLAIMS virtual blocks of the exact search from a counter (scan_valu_body over vb) until none is left.
// A block that stops waiting simply exits, so the fallback is complete whichever blocks take part —
// no co-residency of the grid is needed (round 4 withdrew a version that split the search statically
// over the waiting blocks: two launches on one device could fill every CU with waiting blocks).
// Algorithmic bytes: N·d codes + ⌈N/32⌉·16 tile records + the re-scored rows (a few per query).
#include "k_scan_valu.h"

namespace rfx {
namespace {

constexpr int kK = 16;           // A-list length (k <= 16)
constexpr int kDropRow = -2;     // record entry 15: the block's drop bound, not a row
constexpr int kSurvCap = 1024;   // survivors re-scored by the last block; more -> the exact fallback

template <int DT>
__device__ __forceinline__ float qelem(const void* Q, int64_t i) {
  if constexpr (DT == RFX_F32)
    return ((const float*)Q)[i];
  else if constexpr (DT == RFX_BF16)
    return bf16_to_f32(((const uint16_t*)Q)[i]);
  else
    return f16_to_f32(((const uint16_t*)Q)[i]);
}

__device__ __forceinline__ float f32_up(double v) {
  float f = (float)v;
  if ((double)f < v) f = nextafterf(f, __builtin_inff());
  return f;
}

__device__ __forceinline__ float unord_f32(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// D / 16 bytes of int8 codes per lane of a 16-lane row group: chunk c = j + 16 i (16 B each)
template <int D>
struct Codes {
  static constexpr int C = D / 256;  // 16-B chunks per lane (3 at d 768, 4 at d 1024)
  uint4 v[C];
  uint4 md;  // the row's tile record {scale, live word}, loaded with the codes (prefetched alike)
};

// The two-pass score rule's exact dot of one row against one question, 16 lanes of a DPP row (chunk
// gl + 16 u of each): the f64 sum of the exact products, lane 0 of the row holding the row's sum.  One
// function for the blocks' re-score and the last block's, so their keys are bit-identical.
template <int DT, int VPL>
__device__ __forceinline__ double exact_dot16(const uint4 (&xv)[VPL], const uint4 (&yv)[VPL]) {
  constexpr int EPV = DT == RFX_F32 ? 4 : 8;
  double acc = 0.0;
#pragma unroll
  for (int u = 0; u < VPL; ++u)
#pragma unroll
    for (int ee = 0; ee < EPV; ++ee) acc += (double)elem<DT>(xv[u], ee) * (double)elem<DT>(yv[u], ee);
  return row16_sum_f64(acc);  // (DPP; lane 0's sum = the xor butterfly's)
}

#ifdef RFX_DEBUG_BUILD
// debug library only: the 100-MHz wall clock per block (< 1024) at 0 start, 1 query quantised, 2 row
// stream done, 3 record written; and for the last block 4 records loaded, 5 bound + drop check,
// 6 survivors, 7 re-scored + ranked (query 0), 8 end (tools/k11_phases.py via rfx_dbg_k11_times)
__device__ unsigned long long g_k11_t[1024][4];
__device__ unsigned long long g_k11_last[8];
#define RFX_K11_T(i) \
  do {                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_k11_t[blockIdx.x][i] = wall_clock64(); \
  } while (0)
#define RFX_K11_L(i) \
  do {                                                   \
    if (threadIdx.x == 0) g_k11_last[i] = wall_clock64(); \
  } while (0)
#else
#define RFX_K11_T(i) \
  do {               \
  } while (0)
#define RFX_K11_L(i) \
  do {               \
  } while (0)
#endif

// The exact fallback inside kernel 11's launch (a lone question): claim virtual blocks of the one-launch
// VALU search (K slot 16) until all are taken.  Every branch around a barrier here is on a readfirstlane
// value (uniform to the compiler): with the claimed unit read as a plain LDS value the compiler structurised
// the loop as a divergent one — lanes 1-63 of wave 0 went back to the barrier before lane 0 claimed the
// next unit, and the block re-ran one unit forever (round 5, a 120-s test timeout).  Bounded: a block
// claims at most gridDim.x units.
template <int DT, int D, int VPLV>
__device__ __attribute__((noinline)) void k11_fallback(const void* X, int nrows, const void* Q, int nq, int rows_per_wave,
                                                       float* cand_s, int* cand_r, const uint32_t* mask, uint32_t* vtau,
                                                       uint32_t* vctr, uint32_t* clm, int k_out, float* out_s,
                                                       int64_t* out_r) {
  __shared__ int unit;
  const int tid = threadIdx.x;
  for (int it = 0; it <= (int)gridDim.x; ++it) {
    if (tid == 0) unit = (int)__hip_atomic_fetch_add(clm, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int u = __builtin_amdgcn_readfirstlane(unit);
    __syncthreads();
    if (u >= (int)gridDim.x) break;
    scan_valu_body<DT, 1, 16, VPLV, true>((const uint8_t*)X, nrows, D, Q, nq, rows_per_wave, cand_s, cand_r,
                                          (int)gridDim.x, mask, vtau, FusedOut{vctr, k_out, out_s, out_r, nullptr}, u,
                                          (int)gridDim.x);
  }
}

constexpr int kKeepChunks = 2;  // the kept-score waves' chunks of 64 rows (KEEP below)

template <int DT, int D, int NQT, bool KEEP>
__global__ __launch_bounds__(256) void screen_valu_kernel(const int8_t* __restrict__ X8, const uint4* __restrict__ tmeta,
                                                          const uint32_t* __restrict__ stats, int nrows,
                                                          const void* __restrict__ X, const void* __restrict__ Q, int nq,
                                                          int rows_per_wave, const uint32_t* __restrict__ mask,
                                                          uint32_t* __restrict__ state, float* __restrict__ cand_s,
                                                          int* __restrict__ cand_r, uint32_t* __restrict__ cand_x,
                                                          int k_out, float* __restrict__ out_s,
                                                          int64_t* __restrict__ out_r, int force,
                                                          uint32_t* __restrict__ vtau, uint32_t* __restrict__ vctr) {
  constexpr int C = D / 256;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, j = lane & 15;
  const int n_lists = gridDim.x;
  // state (per index and stream): [0] the arrival counter (zero on entry, left zero), [24] the
  // fallback gate (written by the last block, read by the gated exact search)
  uint32_t* const ctr = state;
  uint32_t* const gate = state + 24;
  // The in-launch fallback's words, each on a cache line of its own (the waiting blocks poll the
  // verdict; polling the arrival counter's line slowed every block's arrival, round 4): [32] the launch
  // generation g (read by every block at its start, advanced by the last block once all have arrived),
  // [64] the verdict 4 g + 1 (proven) / 4 g + 2 (not proven), [96] the claim counter (reset by the last
  // block before a "not proven" verdict).  A verdict names its launch, so nothing is reset after it;
  // launches sharing this state are ordered on one stream, so no block of launch g runs beside g + 1.
  uint32_t* const genw = state + 32;
  uint32_t* const dec = state + 64;
  uint32_t* const clm = state + 96;
  constexpr int ESZV = DT == RFX_F32 ? 4 : 2;
  constexpr int VPR0 = D * ESZV / 16;
  constexpr int VPLV = (VPR0 + 15) / 16 <= 4 ? 4 : (VPR0 + 15) / 16 <= 8 ? 8 : (VPR0 + 15) / 16 <= 12 ? 12 : 16;
  constexpr bool INL = screen_valu_inline_fallback(NQT, DT, D);
  // the exact fallback: claim virtual blocks of the one-launch VALU search (K slot 16) until all are taken
  // (a call, not inlined: the fallback's registers stay out of the screen's allocation — inlined, kernel 11
  // went from 256 to 256 + 57 AGPR registers and its screen from 41.6 to 49.8 us at config 2, round 5)
  auto fallback = [&]() {
    if constexpr (INL)
      k11_fallback<DT, D, VPLV>(X, nrows, Q, nq, rows_per_wave, cand_s, cand_r, mask, vtau, vctr, clm, k_out, out_s,
                                out_r);
  };
  RFX_K11_T(0);
  const uint32_t gen0 = INL ? __hip_atomic_load(genw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;

  // The int8 row stream (step 2): iteration t scores rows wb + 64 (t >> 4) + 4 (t & 15) + g.  Its first
  // NB - 1 iterations of loads are issued here, before the query quantiser, so their latency overlaps
  // it (the rows do not depend on the query).
  const int wave_g = blockIdx.x * 4 + w;
  const int wb = (int)min((int64_t)wave_g * rows_per_wave, (int64_t)nrows);
  const int we = (int)min((int64_t)wb + rows_per_wave, (int64_t)nrows);
  // force bits 2/4/8/16/32/64 (RFX_K11_ABLATE, timing only, wrong results): no row stream / no query
  // quantiser / no last-block work / no re-score and rank / no LB over the records / no list offers
  const int T = (force & 2) ? 0 : we > wb ? (we - wb + 15) / 16 * 4 : 0;
  auto load_row = [&](int t, Codes<D>& v) {
    const int row = wb + 64 * (t >> 4) + 4 * (t & 15) + g;
    const int rr = row < we ? row : wb;
    const int8_t* rp = X8 + (int64_t)rr * D;
#pragma unroll
    for (int i = 0; i < C; ++i) v.v[i] = *(const uint4*)(rp + 16 * (j + 16 * i));
    v.md = tmeta[rr >> 5];  // cache hits after the first row of a tile
  };
  // NB row buffers: NB - 1 iterations of loads in flight ahead of the one being scored (one wave per
  // SIMD has nothing else to hide the latency; 3 in flight measured latency-bound at 2.6 TB/s)
  constexpr int NB = NQT == 1 ? 8 : 4;
  static_assert(NB % 4 == 0, "the offer step takes whole 4-iteration groups (64-row chunks)");
  Codes<D> buf[NB];
  // The quantiser's inputs are requested first (the store maxima and this wave's first query, loaded
  // unconditionally: a load under a wave-uniform condition becomes a branch around it, and the join after
  // it a vmcnt(0) wait on everything in flight) and its max |y| is reduced before the row prefetch is
  // issued: that wait covers the query loads only.  The codes and e2 are then computed while the rows
  // are in flight.
  constexpr int PL = D / 64;  // query elements per lane
  const uint32_t st0 = stats[0], st1 = stats[1];
  const int wq = w < nq ? w : nq - 1;
  const float wmf = w < nq ? 1.f : 0.f;  // a multiply, not a select: no branch around the loads
  float y0[PL];
#pragma unroll
  for (int e = 0; e < PL; ++e) y0[e] = qelem<DT>(Q, (int64_t)wq * D + lane + 64 * e);
  float am0 = 0.f;
#pragma unroll
  for (int e = 0; e < PL; ++e) {
    y0[e] *= wmf;
    am0 = fmaxf(am0, fabsf(y0[e]));
  }
  am0 = wave_max_f32(am0);
  if (T > 0) {
#pragma unroll
    for (int p = 0; p < NB - 1; ++p) load_row(p, buf[p]);
  }

  // ---- 1. query codes and e2 (every block, identically): wave w quantises queries w, w + 4 ------
  __shared__ __attribute__((aligned(16))) int8_t qc_lds[NQT][D];
  __shared__ float e2_lds[NQT];
  const double xm = (double)__uint_as_float(st0), em = (double)__uint_as_float(st1);
  // codes c = rint(y / s) clamped to +-127 (s = max|y| / 127), and e2 from the codes themselves; no
  // branches (s = 0: codes 0, e2 0)
  auto quant = [&](int qi, const float* y, float am) {
    const float s = am > 0.f ? __fdiv_rn(am, 127.f) : 0.f;
    const float sd = s > 0.f ? s : 1.f;
    double ey = 0.0;
    int cc = 0;  // <= 64 PL 127^2 < 2^31
#pragma unroll
    for (int e = 0; e < PL; ++e) {
      int c = (int)fminf(fmaxf(rintf(__fdiv_rn(y[e], sd)), -127.f), 127.f);
      c = s > 0.f ? c : 0;
      qc_lds[qi][lane + 64 * e] = (int8_t)c;
      const double dd = (double)y[e] - (double)s * (double)c;
      ey += dd * dd;
      cc += c * c;
    }
    ey = wave_sum_f64(ey);
    cc = wave_sum_i32(cc);
    if (lane == 0) {
      const double yh = (double)s * sqrt((double)cc);
      const double eq = xm * sqrt(ey) + em * yh;
      const float e2 = f32_up((2.0 * eq + 4e-7 * (xm + em) * yh + 2.4e-7 * xm * (yh + sqrt(ey))) * (1.0 + 1e-5) /
                              (double)sd);  // (the e2 rule of k_screen.hip)
      e2_lds[qi] = s > 0.f ? e2 : 0.f;
    }
  };
  if (!(force & 4)) {
    if (w < NQT) quant(w, y0, am0);
    for (int qi = w + 4; qi < NQT; qi += 4) {  // nq 5..8 only
      const int qq = qi < nq ? qi : nq - 1;
      const float qm = qi < nq ? 1.f : 0.f;
      float y[PL];
      float am = 0.f;
#pragma unroll
      for (int e = 0; e < PL; ++e) {
        y[e] = qelem<DT>(Q, (int64_t)qq * D + lane + 64 * e) * qm;
        am = fmaxf(am, fabsf(y[e]));
      }
      am = wave_max_f32(am);
      quant(qi, y, am);
    }
  }
  __syncthreads();
  RFX_K11_T(1);
  Codes<D> qv[NQT];
#pragma unroll
  for (int qi = 0; qi < NQT; ++qi)
#pragma unroll
    for (int i = 0; i < C; ++i) qv[qi].v[i] = *(const uint4*)(&qc_lds[qi][16 * (j + 16 * i)]);

  // ---- 2. the int8 row stream (set up and first loads issued above) -----------------------------
  WaveList<kK> L[NQT];
  float dm[NQT];  // per lane: the best A this wave dropped (rejected at offer time or evicted)
  float cand[NQT];
#pragma unroll
  for (int qi = 0; qi < NQT; ++qi) {
    L[qi].init();
    dm[qi] = -__builtin_inff();
    cand[qi] = __builtin_nanf("");
  }
  auto score_row = [&](int t, const Codes<D>& v) {
    const int row = wb + 64 * (t >> 4) + 4 * (t & 15) + g;
    const uint4 md = v.md;
    const float st = __uint_as_float(md.x);
#pragma unroll
    for (int qi = 0; qi < NQT; ++qi) {
      int acc = 0;
#pragma unroll
      for (int i = 0; i < C; ++i) {
        acc = __builtin_amdgcn_sdot4((int)v.v[i].x, (int)qv[qi].v[i].x, acc, false);
        acc = __builtin_amdgcn_sdot4((int)v.v[i].y, (int)qv[qi].v[i].y, acc, false);
        acc = __builtin_amdgcn_sdot4((int)v.v[i].z, (int)qv[qi].v[i].z, acc, false);
        acc = __builtin_amdgcn_sdot4((int)v.v[i].w, (int)qv[qi].v[i].w, acc, false);
      }
      const float dsum = row16_sum((float)acc);  // |partial sums| < 2^24: exact in f32
      const float a = dsum * st;                 // A = s_t D, one rounding (as kernel 10)
      // the tile's live bit only: the row mask is read once per chunk at offer time (a load under a
      // condition here would end in a vmcnt(0) drain of the row stream at every row)
      const bool live = row < we && ((md.y >> (row & 31)) & 1u);
      if (j == (t & 15)) cand[qi] = live ? a : __builtin_nanf("");
    }
  };
  auto offer = [&](int qi, float a, int row) {
    // offer one candidate per lane; record in dm what the list does not keep
    WaveList<kK>& l = L[qi];
    const bool valid = a == a;  // NaN = dead / masked / past the end
    if (valid && !better(a, row, l.ts, l.tr)) dm[qi] = fmaxf(dm[qi], a);
    uint64_t m = __ballot(valid && better(a, row, l.ts, l.tr));
    while (m) {
      const int src = __builtin_ctzll(m);
      m &= m - 1;
      const float s = readlane_f(a, src);
      const int r = readlane_i(row, src);
      if (!better(s, r, l.ts, l.tr)) {  // the threshold rose meanwhile: dropped
        if (lane == src) dm[qi] = fmaxf(dm[qi], s);
        continue;
      }
      const float ev = readlane_f(l.ls, kK - 1);  // evicted (-inf while the list is not full)
      if (lane == 0) dm[qi] = fmaxf(dm[qi], ev);
      const bool b = (lane < kK) && better(l.ls, l.lr, s, r);
      const int pos = __popcll(__ballot(b));
      const float us = lane_shr1(l.ls);
      const int ur = lane_shr1(l.lr);
      if (lane > pos && lane < kK) {
        l.ls = us;
        l.lr = ur;
      }
      if (lane == pos) {
        l.ls = s;
        l.lr = r;
      }
      l.ts = readlane_f(l.ls, kK - 1);
      l.tr = readlane_i(l.lr, kK - 1);
    }
  };
  // Round 6 (KEEP: at most kKeepChunks 64-row chunks per wave, config 2: 100 rows): the waves keep every
  // score in registers (one per lane, chunk and question) and pick their 16 best per question once, after
  // the stream, instead of inserting into the sorted lists chunk by chunk: the inserts' serial pop loop was
  // ~12 of config 2's 39 us and ~85-115 of 124-179 us at 2-8 questions (RFX_K11_ABLATE=64,
  // profiles/r06/k11_offer/, k11_nq8/).  The block record needs a wave's best 16 as a set (step 3 ranks all
  // 64 entries) and the best score it did not keep.
  constexpr bool keepall = KEEP;
  // a lone question's list path (> kKeepChunks chunks per wave) seeds its sorted list by one selection over
  // its first kKeepChunks kept chunks (300k rows: 60.8 -> 53.4 us, 1M: 147.5 -> 140.0 us); with 8 query
  // slots the seeded lists measured slower at 1M rows (0.59 against 0.39 ms) and are not used
  constexpr bool seeded = !KEEP && NQT == 1;
  float ka[NQT][kKeepChunks];
  int kr[kKeepChunks];
#pragma unroll
  for (int c = 0; c < kKeepChunks; ++c) {
#pragma unroll
    for (int qi = 0; qi < NQT; ++qi) ka[qi][c] = __builtin_nanf("");
    kr[c] = kEmptyRow;
  }
  // Per question, the wave's 16 best kept scores as a set: v = the 16th largest orderable score (bitwise
  // search on the counts of keys >= v; 0 = fewer than 16 rows), keep every key > v and ties at v in (chunk,
  // lane) order up to 16, into lanes 0..15 of the list; dm = the best score not kept (every row the wave
  // drops is <= it, as the list's drop bound).  sort: also order the 16 (score desc, row asc; a bitonic
  // network over lanes) and set the list's threshold, for the list inserts of later chunks.  Wave-local:
  // the compaction goes through this wave's LDS rows only (no block barrier: waves stream different counts).
  auto select_kept = [&](bool sort) {
    __shared__ float ksa[4][NQT][kK];
    __shared__ int ksr[4][NQT][kK];
    int nk[NQT];
#pragma unroll
    for (int qi = 0; qi < NQT; ++qi) {
      uint32_t key[kKeepChunks];
      int nvalid = 0;
#pragma unroll
      for (int c = 0; c < kKeepChunks; ++c) {
        key[c] = ka[qi][c] == ka[qi][c] ? ord_f32(ka[qi][c]) : 0u;  // (a valid score's key is > 0)
        nvalid += (int)__popcll(__ballot(key[c] != 0u));
      }
      uint32_t v = 0u;
      if (nvalid > kK) {
        for (int bit = 31; bit >= 0; --bit) {
          const uint32_t c1 = v | (1u << bit);
          int cnt = 0;
#pragma unroll
          for (int c = 0; c < kKeepChunks; ++c) cnt += (int)__popcll(__ballot(key[c] >= c1));
          v = cnt >= kK ? c1 : v;
        }
      }
      int room = kK;
#pragma unroll
      for (int c = 0; c < kKeepChunks; ++c) room -= (int)__popcll(__ballot(key[c] > v));
      int base = 0;
      float d = -__builtin_inff();
#pragma unroll
      for (int c = 0; c < kKeepChunks; ++c) {
        const uint64_t tie = __ballot(v != 0u && key[c] == v);
        const int ti =
            (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(tie >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)tie, 0u));
        const bool keep = key[c] > v || (v != 0u && key[c] == v && ti < room);
        room -= min((int)__popcll(tie), max(room, 0));
        if (key[c] != 0u && !keep) d = fmaxf(d, ka[qi][c]);
        const uint64_t kb = __ballot(keep);
        const int p =
            base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(kb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)kb, 0u));
        if (keep) {
          ksa[w][qi][p] = ka[qi][c];
          ksr[w][qi][p] = kr[c];
        }
        base += (int)__popcll(kb);
        ka[qi][c] = __builtin_nanf("");
      }
      dm[qi] = fmaxf(dm[qi], d);
      nk[qi] = base;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int qi = 0; qi < NQT; ++qi) {
      float ls = lane < nk[qi] ? ksa[w][qi][lane] : -__builtin_inff();
      int lr = lane < nk[qi] ? ksr[w][qi][lane] : kEmptyRow;
      if (sort) {
#pragma unroll
        for (int kk = 2; kk <= kK; kk <<= 1)
#pragma unroll
          for (int jj = kk >> 1; jj > 0; jj >>= 1) {
            const float ps = __shfl_xor(ls, jj);
            const int pr = __shfl_xor(lr, jj);
            const bool lower = (lane & jj) == 0, desc = (lane & kk) == 0;
            const bool mine = better(ls, lr, ps, pr);
            if (lower == desc ? !mine : mine) {
              ls = ps;
              lr = pr;
            }
          }
        L[qi].ts = readlane_f(ls, kK - 1);
        L[qi].tr = readlane_i(lr, kK - 1);
      }
      L[qi].ls = ls;
      L[qi].lr = lr;
    }
    __builtin_amdgcn_wave_barrier();  // (this wave's LDS rows are read before any later rewrite)
  };
  for (int t = 0; t < T; t += NB) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      load_row(t + b + NB - 1, buf[(b + NB - 1) % NB]);  // past T: re-reads of row wb, never offered
      score_row(t + b, buf[b]);
      if ((b & 3) == 3 && (((t + b + 1) & 15) == 0 || t + b + 1 >= T)) {
        // a 64-row chunk scored (or the last, partial one): every lane holds one row
        const int crow = wb + 64 * ((t + b) >> 4) + j * 4 + g;
        const bool ok = crow < we && (mask == nullptr || row_allowed(mask, crow));
        // (the loop runs whole groups of NB iterations: a chunk end past T re-offers the last chunk's slot
        // with nothing in it, which the list ignores; kept, it would overwrite the kept chunk)
        const int ch = t + b < T ? (t + b) >> 4 : 1 << 20;
        if (keepall || (seeded && ch < kKeepChunks)) {
          // KEEP: every chunk; a seeded list: the first kKeepChunks, then one selection seeds the sorted
          // list (most inserts happen in the first chunks, before a list's threshold has risen)
#pragma unroll
          for (int c = 0; c < kKeepChunks; ++c)
            if (c == ch) {
#pragma unroll
              for (int qi = 0; qi < NQT; ++qi) ka[qi][c] = ok ? cand[qi] : __builtin_nanf("");
              kr[c] = crow;
            }
#pragma unroll
          for (int qi = 0; qi < NQT; ++qi) cand[qi] = __builtin_nanf("");
          if (seeded && ch == kKeepChunks - 1) select_kept(true);
        } else {
#pragma unroll
          for (int qi = 0; qi < NQT; ++qi) {
            if (!(force & 64)) offer(qi, ok ? cand[qi] : __builtin_nanf(""), crow);
            cand[qi] = __builtin_nanf("");
          }
        }
      }
    }
  }
  // KEEP: every chunk was kept; a seeded list of at most one chunk has not selected yet
  if (keepall || (seeded && T <= 16)) select_kept(false);

  RFX_K11_T(2);
  // ---- 3. block record per query: the 15 best A of the block (rows), and its drop bound ----------
  // The four wave lists (sorted, best first, empty entries at the tail) as rank keys (orderable A << 32
  // | ~row; 0 = empty); the merging wave holds one of the 64 entries per lane and counts the entries
  // better than its own — a one-compare-per-entry rank, no serial insert loop.
  __shared__ uint64_t mk[NQT][4 * kK];
  __shared__ float wdm[4][NQT];
  __shared__ int xrow[NQT][kK];  // per query: the rows this block re-scores early (record entries 0..nxl-1)
  __shared__ int nxl[NQT];
#pragma unroll
  for (int qi = 0; qi < NQT; ++qi) {
    if (lane < kK) {
      const bool v = L[qi].lr != kEmptyRow;
      mk[qi][w * kK + lane] = v ? ((uint64_t)ord_f32(L[qi].ls) << 32) | (uint32_t)(~(uint32_t)L[qi].lr) : 0ull;
    }
    float d = dm[qi];
    d = wave_max_f32(d);
    if (lane == 0) wdm[w][qi] = d;
  }
  __syncthreads();
  for (int qi = w; qi < nq; qi += 4) {
    const uint64_t mine = mk[qi][lane];
    int rank = 0;
#pragma unroll 16
    for (int i = 0; i < 4 * kK; ++i) rank += mk[qi][i] > mine ? 1 : 0;
    const bool v = mine != 0ull;
    const float ms_ = unord_f32((uint32_t)(mine >> 32));
    // dropped: the waves' drops and every entry from the 16th on (the record keeps 15; entry 15 carries
    // the drop bound instead)
    float d = fmaxf(fmaxf(wdm[0][qi], wdm[1][qi]), fmaxf(wdm[2][qi], wdm[3][qi]));
    if (v && rank >= kK - 1) d = fmaxf(d, ms_);
    d = wave_max_f32(d);
    const int nv = (int)__popcll(__ballot(v));
    const int64_t o0 = ((int64_t)qi * n_lists + blockIdx.x) * kK;
    if (v && rank < kK - 1) {
      __hip_atomic_store((uint32_t*)cand_s + o0 + rank, __float_as_uint(ms_), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(cand_r + o0 + rank, (int)(~(uint32_t)mine), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane >= nv && lane < kK - 1) {  // empty tail of the record
      __hip_atomic_store((uint32_t*)cand_s + o0 + lane, __float_as_uint(-__builtin_inff()), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(cand_r + o0 + lane, kEmptyRow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == kK - 1) {
      __hip_atomic_store((uint32_t*)cand_s + o0 + lane, __float_as_uint(d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(cand_r + o0 + lane, kDropRow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // Early re-score (round 5).  LB_b = the block's k-th best A (record entry k - 1) is a lower bound of
    // a_k (distinct live rows); the last block's bound LB* includes every record's entry k - 1 (k <= 15),
    // so an entry it keeps has A >= LB* - e2 >= LB_b - e2 (f32 subtraction is monotone).  Those entries (a
    // prefix of the ranks: A falls with the rank) are re-scored exactly by this block AFTER it arrives (off
    // the critical path; step 4), their keys going to cand_x, which holds 0 for every entry until then.
    // The last block takes a survivor's key from there, and re-scores a survivor whose key is still 0
    // itself (its own entries, a block not done yet): no answer depends on the timing.
    const uint64_t kb = __ballot(v && rank == k_out - 1);
    const uint32_t lbb = kb ? ord_f32(readlane_f(ms_, (int)__builtin_ctzll(kb))) : 0u;
    const float cutb = lbb ? unord_f32(lbb) - e2_lds[qi] : -__builtin_inff();
    const bool rx = v && rank < kK - 1 && ms_ >= cutb;
    if (v && rank < kK - 1) __hip_atomic_store(cand_x + o0 + rank, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane >= nv && lane < kK - 1) __hip_atomic_store(cand_x + o0 + lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (rx) xrow[qi][rank] = (int)(~(uint32_t)mine);
    const int nx = (int)__popcll(__ballot(rx));
    if (lane == 0) nxl[qi] = nx;
  }
  // the early re-score (a block that is not the last, after it arrived): the entries above, 16 lanes each
  // (the last block's layout), all queries' entries in a row
  auto early_rescore = [&]() {
    int tot = 0;
    for (int qi = 0; qi < nq; ++qi) tot += nxl[qi];
    tot = __builtin_amdgcn_readfirstlane(tot);
    constexpr int ESZ = DT == RFX_F32 ? 4 : 2;
    constexpr int VPL = D * ESZ / 256;
    const int grp = tid >> 4, gl = tid & 15;
    for (int p0 = 0; p0 < tot; p0 += 16) {
      const int p = p0 + grp < tot ? p0 + grp : 0;  // (clamped: whole 16-lane rows take part in the sum)
      int qi = 0, e = p;
      while (qi < nq - 1 && e >= nxl[qi]) {
        e -= nxl[qi];
        ++qi;
      }
      const int r = xrow[qi][e];
      uint4 yv[VPL], xv[VPL];
#pragma unroll
      for (int u = 0; u < VPL; ++u) {
        yv[u] = *(const uint4*)((const uint8_t*)Q + (int64_t)qi * D * ESZ + (int64_t)(gl + 16 * u) * 16);
        xv[u] = *(const uint4*)((const uint8_t*)X + (int64_t)r * D * ESZ + (int64_t)(gl + 16 * u) * 16);
      }
      const double acc = exact_dot16<DT, VPL>(xv, yv);
      if (gl == 0 && p0 + grp < tot)
        __hip_atomic_store(cand_x + ((int64_t)qi * n_lists + blockIdx.x) * kK + e, ord_f32((float)acc),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };

  // ---- 4. the last block: a_k from the records, the drop check, survivors, exact re-score, top-k --
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const uint32_t old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == gridDim.x - 1;
  }
  __syncthreads();
  RFX_K11_T(3);
  const bool lastu = __builtin_amdgcn_readfirstlane(last) != 0;  // (uniform: see fallback above)
  if (!lastu && !(force & 16)) early_rescore();
  if (!INL && !lastu) return;
  if (!lastu) {
    // wait for the last block's verdict on this launch, at most kVerdictWait of wall clock (100 MHz):
    // a block that stops waiting exits, and the fallback completes without it.  Round 6: every
    // 8th poll also reads the arrival counter; while blocks are still to arrive and none has for kStallWait,
    // the grid is not all running (another launch holds CUs: a kernel-10 batch, a second kernel-11 launch) and
    // this block leaves at once, so the late blocks find a CU.  The counter reads 0 only once the last block
    // has reset it, right before its verdict.  Worst case a waiting block holds its CU for kVerdictWait when
    // every block has arrived and the last block's check runs long; for kStallWait + one poll (~6 us) when
    // arrivals stall.
    constexpr uint64_t kVerdictWait = 5000;  // 50 us
    constexpr uint64_t kStallWait = 500;     // 5 us
    __shared__ uint32_t verdict;
    if (tid == 0) {
      const uint64_t t0 = wall_clock64();
      uint64_t t_seen = t0;
      uint32_t d = 0u, seen = 0xffffffffu;
      for (int i = 1;; ++i) {
        d = __hip_atomic_load(dec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t now = wall_clock64();
        if (((d >> 2) == (gen0 & 0x3fffffffu) && (d & 3u)) || now - t0 > kVerdictWait) break;
        if ((i & 7) == 0) {
          const uint32_t c = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (c != seen) {
            seen = c;
            t_seen = now;
          } else if (c != 0u && c < gridDim.x && now - t_seen > kStallWait) {
            break;
          }
        }
        __builtin_amdgcn_s_sleep(8);
      }
      verdict = (d >> 2) == (gen0 & 0x3fffffffu) ? (d & 3u) : 0u;
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(verdict) == 2u) fallback();
    return;
  }
  RFX_K11_L(0);
  if (force & 8) {
    if (tid == 0) {
      *gate = 0u;
      *ctr = 0u;
      if (INL) {
        __hip_atomic_store(dec, ((gen0 & 0x3fffffffu) << 2) | 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(genw, gen0 + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  const int n = n_lists * kK;  // <= kFusedLdsCand (host check)
  __shared__ float bs[kFusedLdsCand];
  __shared__ int br[kFusedLdsCand];
  __shared__ int sv[kSurvCap];    // survivor -> record index
  __shared__ int mv[kSurvCap];    // survivors without an exact key (re-scored here)
  // its rank key: (orderable fl32 of the exact f64 sum) << 32 | ~row, larger = better under (score
  // desc, row asc): the rank is one 64-bit compare per survivor (no branches, no dependent LDS loads)
  __shared__ uint64_t skey[kSurvCap];
  __shared__ float red[4];
  __shared__ uint32_t redg[4];
  __shared__ int n_sv, n_mv, fail;
  __shared__ float cut;
  __shared__ uint32_t fin[4 * kK];
  if (tid == 0) fail = force & 1;
  for (int qi = 0; qi < nq; ++qi) {
    // bulk copy into LDS with all loads of a thread in flight (agent-scope loads are not batched by the
    // compiler: one at a time they cost a memory round trip each — measured 55 us for this select)
    // (16 per thread: config 2's 250 records of 16 in one round trip; the loads are unconditional, on a
    // clamped index, so no branch and no drain sits between them)
    constexpr int UL = 16;
    for (int base = 0; base < n; base += 256 * UL) {
      uint32_t sv8[UL];
      int rv8[UL];
#pragma unroll
      for (int u = 0; u < UL; ++u) {
        const int i = base + u * 256 + tid;
        const int ic = i < n ? i : n - 1;
        sv8[u] = __hip_atomic_load((const uint32_t*)cand_s + (int64_t)qi * n + ic, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        rv8[u] = __hip_atomic_load(cand_r + (int64_t)qi * n + ic, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int u = 0; u < UL; ++u) {
        const int i = base + u * 256 + tid;
        if (i < n) {
          bs[i] = __uint_as_float(sv8[u]);
          br[i] = rv8[u];
        }
      }
    }
    if (tid == 0) {
      n_sv = 0;
      n_mv = 0;
    }
    __syncthreads();
    if (qi == 0) RFX_K11_L(1);
    // The largest drop bound (entry 15 of each record), and LB, a lower bound of a_k: the k-th largest
    // key (with multiplicity; 0 = fewer than k) of the records' best entries (every entry when the
    // records are few) — distinct live rows either way.  Each wave extracts the k best of its 256 keys
    // (4 per lane, sorted in registers) by k rounds of a wave max; wave 0 ranks the 4k finalists (the
    // union of the waves' top-k holds the top-k values with their multiplicity).
    float dmax = -__builtin_inff();
    uint32_t gk = 0u;  // the largest block bound LB_b (record entry k - 1; k <= 15)
    for (int c = tid; c < n_lists; c += 256) {
      const int i = c * kK + kK - 1;
      if (br[i] == kDropRow) dmax = fmaxf(dmax, bs[i]);
      const int i2 = c * kK + k_out - 1, r2 = br[i2];
      if (k_out < kK && r2 != kEmptyRow && r2 != kDropRow) gk = max(gk, ord_f32(bs[i2]));
    }
    dmax = wave_max_f32(dmax);
    gk = wave_max_u32(gk);
    if (lane == 0) {
      red[w] = dmax;
      redg[w] = gk;
    }
    const bool every = n <= 1024;
    const int m = (force & 32) ? 0 : every ? n : n_lists;  // <= 1024
    uint32_t a0, a1, a2, a3;  // this lane's keys, sorted
    {
      uint32_t ak[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = w * 256 + u * 64 + lane;
        uint32_t key = 0u;
        if (c < m) {
          const int i = every ? c : c * kK;
          const int r = br[i];
          key = r != kEmptyRow && r != kDropRow ? ord_f32(bs[i]) : 0u;
        }
        ak[u] = key;
      }
      // sort the lane's four keys descending (five compare-exchanges)
      auto cx = [](uint32_t& x, uint32_t& y) {
        const uint32_t hi = max(x, y), lo = min(x, y);
        x = hi;
        y = lo;
      };
      cx(ak[0], ak[1]);
      cx(ak[2], ak[3]);
      cx(ak[0], ak[2]);
      cx(ak[1], ak[3]);
      cx(ak[1], ak[2]);
      a0 = ak[0], a1 = ak[1], a2 = ak[2], a3 = ak[3];
      if (m > 256) {  // (several waves hold keys: each extracts its k best, wave 0 ranks the 4 k)
        if (lane < kK) fin[w * kK + lane] = 0u;
        for (int it = 0; it < k_out; ++it) {
          const uint32_t mx = wave_max_u32(a0);
          const bool win = lane == (int)__builtin_ctzll(__ballot(a0 == mx));
          a0 = win ? a1 : a0;
          a1 = win ? a2 : a1;
          a2 = win ? a3 : a2;
          a3 = win ? 0u : a3;
          if (lane == 0) fin[w * kK + it] = mx;
        }
      }
    }
    __syncthreads();
    if (w == 0) {
      uint32_t lb = 0u;
      if (m <= 256) {
        // every key is wave 0's (config 2: 250 record heads): the k-th largest with multiplicity by a
        // bitwise search on ballot counts (round 6; 0 when fewer than k keys), no finalists, no barrier
        uint32_t v = 0u;
        for (int bit = 31; bit >= 0; --bit) {
          const uint32_t c1 = v | (1u << bit);
          const int cnt = (int)(__popcll(__ballot(a0 >= c1)) + __popcll(__ballot(a1 >= c1)) +
                                __popcll(__ballot(a2 >= c1)) + __popcll(__ballot(a3 >= c1)));
          v = cnt >= k_out ? c1 : v;
        }
        lb = v;
      } else {
        const uint32_t x = fin[lane];  // 4 kK = 64 finalists, one per lane
        int ge = 0, gt = 0;
#pragma unroll 16
        for (int i = 0; i < 4 * kK; ++i) {
          const uint32_t v = fin[i];
          ge += v >= x ? 1 : 0;
          gt += v > x ? 1 : 0;
        }
        lb = x && gt < k_out && ge >= k_out ? x : 0u;
      }
      // LB* = the larger of the two lower bounds of a_k: >= every LB_b the blocks re-scored against
      lb = max(wave_max_u32(lb), max(max(redg[0], redg[1]), max(redg[2], redg[3])));
      if (lane == 0) {
        const float dm_all = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
        cut = lb ? unord_f32(lb) - e2_lds[qi] : -__builtin_inff();
        // a dropped row at or above LB - e2 could belong to the top-k: not proven
        if (dm_all > -__builtin_inff() && dm_all >= cut) fail = 1;
      }
    }
    __syncthreads();
    if (qi == 0) RFX_K11_L(2);
    // survivors: the entries at or above the cut; a record is sorted best first, so its scan ends at
    // the first entry below the cut (most records: at their best entry)
    for (int c = tid; c < n_lists; c += 256) {
      const int i0 = c * kK;
      for (int e = 0; e < kK - 1; ++e) {
        const int r = br[i0 + e];
        if (r == kEmptyRow || !(bs[i0 + e] >= cut)) break;
        const int j2 = atomicAdd(&n_sv, 1);
        if (j2 < kSurvCap) sv[j2] = i0 + e;
      }
    }
    __syncthreads();
    if (n_sv > kSurvCap && tid == 0) fail = 1;
    __syncthreads();
    if (qi == 0) RFX_K11_L(3);
    if (!fail && !(force & 16)) {
      const int ns = n_sv;
      // the survivors' exact keys from the blocks' early re-score (one round of loads), read now, when
      // the blocks that arrived before this one have had the bound, drop check and survivors' time to
      // write them; a key still 0 (this block's own entries, a block not done yet) is re-scored here
      for (int e = tid; e < ns; e += 256) {
        const int i = sv[e];
        const uint32_t x = __hip_atomic_load(cand_x + (int64_t)qi * n + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (x)
          skey[e] = ((uint64_t)x << 32) | (uint32_t)(~(uint32_t)br[i]);
        else
          mv[atomicAdd(&n_mv, 1)] = e;
      }
      __syncthreads();
      // exact re-score of those: 16 lanes per survivor (16-B chunks gl + 16 u of the row), UR survivors per group
      // in flight, 32 per round; the query's chunks are loaded once per query, not per survivor
      const int nm = __builtin_amdgcn_readfirstlane(n_mv);
#ifdef RFX_DEBUG_BUILD
      if (qi == 0 && tid == 0) {  // survivors, and those without a key from the blocks (tools/k11_phases.py)
        g_k11_last[6] = (unsigned long long)ns;
        g_k11_last[7] = (unsigned long long)nm;
      }
#endif
      if (nm > 0) {
        constexpr int ESZ = DT == RFX_F32 ? 4 : 2;
        constexpr int VPL = D * ESZ / 256;
        constexpr int UR = 2;
        const int grp = tid >> 4, gl = tid & 15;
        uint4 yv[VPL];
#pragma unroll
        for (int u = 0; u < VPL; ++u)
          yv[u] = *(const uint4*)((const uint8_t*)Q + (int64_t)qi * D * ESZ + (int64_t)(gl + 16 * u) * 16);
        for (int e0 = 0; e0 < nm; e0 += 16 * UR) {
          uint4 xv[UR][VPL];
#pragma unroll
          for (int ur = 0; ur < UR; ++ur) {
            const int e = e0 + grp + 16 * ur;
            const int r = br[sv[mv[e < nm ? e : 0]]];
#pragma unroll
            for (int u = 0; u < VPL; ++u)
              xv[ur][u] = *(const uint4*)((const uint8_t*)X + (int64_t)r * D * ESZ + (int64_t)(gl + 16 * u) * 16);
          }
#pragma unroll
          for (int ur = 0; ur < UR; ++ur) {
            const int e = e0 + grp + 16 * ur;
            const double acc = exact_dot16<DT, VPL>(xv[ur], yv);
            if (gl == 0 && e < nm) {
              const int jj = mv[e];
              skey[jj] = ((uint64_t)ord_f32((float)acc) << 32) | (uint32_t)(~(uint32_t)br[sv[jj]]);
            }
          }
        }
      }
      __syncthreads();
      // top-k of the survivors by (exact score desc, row asc): each survivor counts those ahead of it
      for (int e = tid; e < ns; e += 256) {
        const uint64_t ke = skey[e];
        int rank = 0;
#pragma unroll 8
        for (int f = 0; f < ns; ++f) rank += skey[f] > ke ? 1 : 0;
        if (rank < k_out) {
          const uint32_t o = (uint32_t)(ke >> 32);
          out_s[(int64_t)qi * k_out + rank] = __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
          out_r[(int64_t)qi * k_out + rank] = (int)(~(uint32_t)ke);
        }
      }
      for (int i = ns + tid; i < k_out; i += 256) {  // fewer survivors than k: padding
        out_s[(int64_t)qi * k_out + i] = -__builtin_inff();
        out_r[(int64_t)qi * k_out + i] = -1;
      }
    }
    __syncthreads();
    if (qi == 0) RFX_K11_L(4);
  }
  RFX_K11_L(5);
  const bool fb = __builtin_amdgcn_readfirstlane(fail) != 0;
  if (tid == 0) {
    // the gate: read by the gated exact search that follows on the stream (several questions)
    __hip_atomic_store(gate, fb ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *ctr = 0u;
    if (INL) {
      // the claim counter is zero before any block can read a "not proven" verdict
      if (fb) __hip_atomic_store(clm, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(dec, ((gen0 & 0x3fffffffu) << 2) | (fb ? 2u : 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(genw, gen0 + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (INL && fb) {
    __syncthreads();
    fallback();
  }
}

}  // namespace

#ifdef RFX_DEBUG_BUILD
int dbg_k11_times(unsigned long long* blocks_h, unsigned long long* last_h) {
  if (hipMemcpyFromSymbol(blocks_h, HIP_SYMBOL(g_k11_t), sizeof(g_k11_t)) != hipSuccess) return -1;
  return hipMemcpyFromSymbol(last_h, HIP_SYMBOL(g_k11_last), sizeof(g_k11_last)) == hipSuccess ? 0 : -1;
}
#endif

// One launch: grid (blocks) × 256 threads, one query slice of up to 8 queries.  The in-launch fallback
// (a lone question) is the one-launch VALU search's K slot 16 over the same plan (k 5..16; its state
// vstate: bounds, then counters).
int launch_screen_valu(const ValuPlan& p, const int8_t* X8, const void* tmeta, const uint32_t* stats, int nrows, int D,
                       int dtype, const void* X, const void* Q, int nq, const uint32_t* mask, uint32_t* state,
                       uint32_t* vstate, float* cs, int* cr, uint32_t* cx, int k, float* out_s, int64_t* out_r,
                       int force, hipStream_t st) {
  if (!cx) return -1;
  if (nq < 1 || nq > 8 || k < 1 || k > kK || (D != 768 && D != 1024)) return -1;
  if ((int64_t)p.blocks * kK > (int64_t)1 << 30) return -1;
  if (screen_valu_inline_fallback(nq == 1 ? 1 : 8, dtype, D) && (!vstate || p.q_slices != 1 || valu_k_slot(k) != 16))
    return -1;
  const dim3 grid((unsigned)p.blocks);
  uint32_t* const vtau = vstate;
  uint32_t* const vctr = vstate ? vstate + kValuFusedMaxNq : nullptr;
  // the kept-score waves (KEEP) when every wave streams at most kKeepChunks 64-row chunks
  const bool keep = p.rows_per_wave <= 64 * kKeepChunks;
#define RFX_SV(DTV, DV, NQ)                                                                                         \
  do {                                                                                                              \
    if (keep)                                                                                                       \
      hipLaunchKernelGGL((screen_valu_kernel<DTV, DV, NQ, true>), grid, dim3(256), 0, st, X8, (const uint4*)tmeta,    \
                         stats, nrows, X, Q, nq, p.rows_per_wave, mask, state, cs, cr, cx, k, out_s, out_r, force,    \
                         vtau, vctr);                                                                               \
    else                                                                                                            \
      hipLaunchKernelGGL((screen_valu_kernel<DTV, DV, NQ, false>), grid, dim3(256), 0, st, X8, (const uint4*)tmeta,   \
                         stats, nrows, X, Q, nq, p.rows_per_wave, mask, state, cs, cr, cx, k, out_s, out_r, force,    \
                         vtau, vctr);                                                                               \
  } while (0)
  // (2 and 4 query slots for the kept-score waves: a batch of 2 paid the stream work of 8 slots — 32 of its
  // 54 us, profiles/r06/k11_nq8_ablate/; the list path keeps 1 or 8)
#define RFX_SV_KEEP(DTV, DV, NQ)                                                                                  \
  hipLaunchKernelGGL((screen_valu_kernel<DTV, DV, NQ, true>), grid, dim3(256), 0, st, X8, (const uint4*)tmeta, stats, \
                     nrows, X, Q, nq, p.rows_per_wave, mask, state, cs, cr, cx, k, out_s, out_r, force, vtau, vctr)
#define RFX_SV_D(DTV)                            \
  if (D == 768) {                                \
    if (nq == 1)                                 \
      RFX_SV(DTV, 768, 1);                       \
    else if (keep && nq <= 2)                    \
      RFX_SV_KEEP(DTV, 768, 2);                  \
    else if (keep && nq <= 4)                    \
      RFX_SV_KEEP(DTV, 768, 4);                  \
    else                                         \
      RFX_SV(DTV, 768, 8);                       \
  } else {                                       \
    if (nq == 1)                                 \
      RFX_SV(DTV, 1024, 1);                      \
    else if (keep && nq <= 2)                    \
      RFX_SV_KEEP(DTV, 1024, 2);                 \
    else if (keep && nq <= 4)                    \
      RFX_SV_KEEP(DTV, 1024, 4);                 \
    else                                         \
      RFX_SV(DTV, 1024, 8);                      \
  }
  if (dtype == RFX_F32) {
    RFX_SV_D(RFX_F32)
  } else if (dtype == RFX_BF16) {
    RFX_SV_D(RFX_BF16)
  } else {
    RFX_SV_D(RFX_F16)
  }
#undef RFX_SV_D
#undef RFX_SV_KEEP
#undef RFX_SV
  return 0;
}

}  // namespace rfx
