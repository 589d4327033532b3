// k_scan_screen.h — kernel 10, the int8 screen of the exact two-pass scan (BASELINE config 3:
// 10M×768 bf16, nq 256, k 10; config 4's shard at d 1024).
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551).
// The screen reads an int8 copy of the store (half the bytes of the bf16 rows) on
// v_mfma_i32_16x16x64_i8 (twice the bf16 rate) and keeps, per query, every row whose exact score
// can still reach the query's k-th best; k_screen.hip re-scores those rows exactly from the bf16
// rows and returns the same top-k as the exact scan (kernel 6 / 8).  DESIGN §4.10.
//
// Why the result is exact.  Rows are quantised per 32-row tile (scale s_t = amax_t / 127, codes
// c = rint(x / s_t)), queries per query (s_y).  For a row x and query y with reconstructions
// x^ = s_t c_x, y^ = s_y c_y:   x·y − x^·y^ = x·(y − y^) + (x − x^)·y^, so by Cauchy-Schwarz
//     |x·y − s_t s_y D| <= ||x|| ||y − y^|| + ||x − x^|| ||y^|| =: E_q      (D = c_x·c_y, exact i32)
// with ||x|| and ||x − x^|| replaced by their maxima over the store (the `stats` of the
// quantiser, rounded up).  In units of s_y the screen score is A = s_t D (one f32 rounding,
// covered by the slack in e2 = 2 E_q / s_y rounded up, k_screen.hip quantize_queries_kernel).
// Let a_k be the k-th best A over live rows.  The k rows that reach it have exact scores
// >= a_k − E_q, so the true k-th best exact score is too, and a row of the true top-k has
// A >= a_k − 2 E_q / s_y = a_k − e2.  The kernel keeps every such row:
//   * pruning.  The bound max(own list's KL-th best, KL-th largest of the query's 16 cross-workgroup
//     slots; tau_kth below) is a lower bound of a_k (KL >= k); a row is looked at only when
//     A >= bound − e2;
//   * lists.  Each lane keeps the KL best A of the rows it looked at (LDS, as kernel 6) and the
//     best A it had to drop (`drop`: not inserted, or evicted).  k_screen.hip's select kernel
//     finds a_k from the lists' union, and takes the fallback (the exact kernel on the whole
//     batch) when a dropped A reaches a_k − e2 or the survivors overflow its buffer.
// Dead rows (tombstones, the NaN tail, rows a metadata filter excludes) carry code 0 and a clear
// bit in the tile's live word; the slow path skips them, so they never raise a_k.
//
// Layout and schedule follow kernel 6 (k_scan_mfma6.h) at half the bytes: workgroup = 8 waves ×
// 32 resident queries (B fragments: D / 64 k-steps × 2 query blocks × 16 B = 96 VGPRs at d 768),
// 32-row tiles (block b takes tiles b, b + B, ...), a stage = 32 rows × 256 codes (8 KB) by LDS-DMA
// into a RING-slot ring (one 1-KB piece per wave per stage), LDS image with chunk c of row r at
// c ^ (r & 15), counted vmcnt + s_barrier per stage, v_permlane16_swap epilogue.
// Algorithmic bytes per tile: 32 * D (codes) + 16 (the tile's metadata record).
#pragma once
#include "k_mfma_common.h"

namespace rfx {
namespace k10 {

using namespace mfc;

constexpr int kWaves = 8;
constexpr int kTM = 32;                   // rows per tile
constexpr int kQW = 32;                   // queries per wave
constexpr int kQG = kWaves * kQW;         // 256 queries per workgroup
constexpr int kQGSmall = 2 * kQW;         // the 2-wave kernel's 64 (batches of <= 64 questions)
constexpr int kSK = 256;                  // codes (bytes) per row per stage
constexpr int kRowB = kSK;                // 256 B per row per stage
constexpr int kSlot = kTM * kRowB;        // 8 KB: 32 rows × 256 codes
#ifndef RFX_K10_RING
#define RFX_K10_RING 8
#endif
constexpr int kRing = RFX_K10_RING;       // slots; RING - 1 stages in flight
constexpr int kGPW = 1;                   // LDS-DMA pieces per wave per stage (8 KB / 1 KB / 8 waves)
constexpr int kTauW = 16;                 // u32 per query in the threshold table: 16 slots (tau_kth)
constexpr int kTauBytes = kQG * kTauW * 4;  // 16 KB
constexpr int kTauGPW = kTauBytes / 1024 / kWaves;
constexpr int kMR = 8;  // tile-metadata slots (1 KB each: 64 lane copies of the 16-B record)
constexpr int kXbWords = 8;  // after the slot table: the XCD split's weight snapshot for this launch
#ifdef RFX_K10_BLOCK_TIMES
// debug build only (k10_dbg.hip): MODE 65536 records each block's 100-MHz wall clock when it starts
// and when all its waves are done ([0], [1]), and its shader clock (s_memtime) at the same points ([2], [3]):
// the in-kernel clock = d(memtime) / d(realtime) x 100 MHz (tools/k10_block_times.py)
__device__ unsigned long long g_k10_bt[1024][4];
// MODE 8192: per tile index (capped at 63) the wave-tiles that enter the slow path and the pop-loop
// trips they make (max over the wave's lanes of the passing values), summed over all waves
__device__ unsigned int g_k10_trips[2][64];
#endif
// NW: waves per workgroup (kWaves = 8: 256 queries, config 3's batches; 2: 64 queries, the micro-batches of
// 9..64 questions, two workgroups per CU).  A workgroup's slot table is NW * 32 queries x 16 slots.
template <int NW>
constexpr int tau_bytes_nw() { return NW * kQW * kTauW * 4; }
template <int RING>
constexpr int meta_off() { return RING * kSlot; }
template <int RING>
constexpr int tau_off() { return meta_off<RING>() + kMR * 1024; }
template <int RING, int NW = kWaves>
constexpr int list_off() { return tau_off<RING>() + tau_bytes_nw<NW>(); }
// per-slot arrival counters of the barrier-free ring (debug MODE 32768): ready[16], done[16], in the
// first 128 B of the debug MODE 1024 list area (never both; both are zeroed before the first barrier)
template <int KL, int RING, int NW = kWaves>
constexpr int ctr_off() { return list_off<RING, NW>(); }
// the list area (debug MODE 1024's LDS lists) exists in the 8-wave kernel; the 2-wave kernel keeps only the
// 128 B of counters, so two workgroups fit a CU's LDS
template <int KL, int RING, int NW = kWaves>
constexpr int lds_bytes() { return list_off<RING, NW>() + (NW == kWaves ? kWaves * KL * 64 * 8 : 128); }
static_assert(lds_bytes<10, 12>() <= 163840, "LDS budget");
static_assert(2 * lds_bytes<16, 8, 2>() <= 163840, "two 2-wave workgroups per CU");

// spin (s_sleep) until the LDS counter reaches target; bounded, so a counting error can never hang the
// GPU (the result would be wrong, and the tests would say so)
__device__ __forceinline__ void lds_spin_ge(const uint32_t* p, uint32_t target) {
  for (int guard = 0; guard < (1 << 20); ++guard) {
    if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) break;
    __builtin_amdgcn_s_sleep(1);
  }
}
__device__ __forceinline__ void lds_arrive(uint32_t* p) {
  __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
static_assert(kSlot / 1024 == kWaves * kGPW && kTauGPW == 2, "DMA pieces per wave");

// the slot table is re-read at the end of these tiles (used two tiles later); debug MODE 16: at every one
// of the first 16 tiles (the bound's warm-up), then every 4th
template <int MODE>
__device__ __forceinline__ bool tau_refresh_tile(int it) {
  return it < ((MODE & 16) != 0 ? 16 : 2) || (it & 3) == 3;
}

// The pruning bound from a query's kTauW = 16 slots: list j publishes its best A to slot j % 16, so
// the slots hold the A of 16 distinct rows (lists are disjoint row sets) and the KL-th largest slot is
// a lower bound of the query's KL-th best A.  Against kernel 6's min over KL slots it sits much closer
// to the KL-th best (simulated on 10M Gaussian scores, 512 lists: 14.6 rows above the bound against
// 26.2 for k = 10), so fewer rows reach bound - e2 and fewer tiles take the slow path.  Bitonic sort of
// the 16 values, descending (80 compare-exchanges; the refresh runs every 4th tile).
template <int KL>
__device__ __forceinline__ uint32_t kth16(uint32_t (&v)[16]) {
#pragma unroll
  for (int k = 2; k <= 16; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int l = i ^ j;
        if (l > i) {
          const uint32_t a = v[i], b = v[l];
          const bool desc = (i & k) == 0;
          v[i] = desc ? max(a, b) : min(a, b);
          v[l] = desc ? min(a, b) : max(a, b);
        }
      }
  return v[KL - 1];
}
template <int KL>
__device__ __forceinline__ uint32_t tau_kth(const uint8_t* p) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint4 a = *(const uint4*)(p + 16 * i);
    v[4 * i] = a.x;
    v[4 * i + 1] = a.y;
    v[4 * i + 2] = a.z;
    v[4 * i + 3] = a.w;
  }
  return kth16<KL>(v);
}

__device__ __forceinline__ v4i32 mfma_i8(const uint4& a, const uint4& b, const v4i32& c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(v4i32, a), __builtin_bit_cast(v4i32, b), c, 0, 0, 0);
}
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }

// Fold one tile's 16 values of this lane (rows rbase + (r & 7) + 16 (r >> 3), ROWMAP 1 of
// k_mfma_common.h) into its list.  thr_o: the pruning bound (orderable A, 0 = none); rows are
// looked at from thr − e2 on.  drop_o: the best A this lane looked at and did not keep.
// Production: the 16 pass tests make a bit mask first (fold_mask); the list (L) lives in registers for
// the whole scan, and each lane inserts its passing values one per trip (fold_trip: KL independent
// compares, no memory); fold_end tightens the own bound and publishes the list's best.  The
// serial LDS insert (one dependent LDS round trip per shifted entry) is debug MODE 1024: a wave in this
// slow path holds the whole workgroup at the next stage barrier.
// The pass mask: bit r set = value r is live and reaches thr − e2; pub = the tile's best reaches it (the
// lane then publishes its list's best, fold_end).
__device__ __forceinline__ uint32_t fold_mask(const v4i32 (&a)[4], float st, uint32_t bits, uint32_t thr_o, float e2,
                                              bool& pub) {
  int mx = max3i(a[0][0], a[0][1], a[0][2]);
  mx = max3i(mx, a[0][3], a[1][0]);
  mx = max3i(mx, a[1][1], a[1][2]);
  mx = max3i(mx, a[1][3], a[2][0]);
  mx = max3i(mx, a[2][1], a[2][2]);
  mx = max3i(mx, a[2][3], a[3][0]);
  mx = max3i(mx, a[3][1], a[3][2]);
  mx = max(mx, a[3][3]);
  const float thr = thr_o ? unord(thr_o) - e2 : -__builtin_inff();
  pub = (float)mx * st >= thr;  // s_t >= 0: the tile's best A bounds every row's
  uint32_t pm = 0;
  if (pub) {
    // which of the 16 values pass (live bits applied once, re-ordered to r: bit r <- row bit
    // (r & 7) + 16 (r >> 3)), without branching on each one
#pragma unroll
    for (int r = 0; r < 16; ++r) pm |= (float)a[r >> 2][r & 3] * st >= thr ? (1u << r) : 0u;
    pm &= (bits & 0xffu) | ((bits >> 8) & 0xff00u);
  }
  return pm;
}
// Production pass mask (round 5): one INTEGER threshold per lane instead of 16 float scale-and-compare
// steps.  t is at or below the smallest D with fl(fl(D) s_t) >= thr - e2 (the passing D form an up-set:
// the product's rounding is monotone in D), so the mask is a superset of the float test's: a value it adds
// lies below thr - e2 <= a_k - e2, is looked at like any other (kept, or recorded in drop) and can never
// reach the select's a_k - e2 (the records hold the true top-k, so the select's a_k' is a_k).  The margin:
// c = tf * rcp(s_t) is within 2^-22 |c| of tf / s_t, and fl(D s_t) >= tf needs D >= tf / s_t (1 - 2^-24);
// |c| 2^-19 + 2 covers both.  The 16 bits are shifted in by v_alignbit (the sign of t - 1 - D, which
// is set iff D >= t; |D| < 2^24, |t| <= 2^30: no overflow): 2 VALU per value against the float test's 4.
// (debug kModeFloatMask: the float test, fold_mask above)
__device__ __forceinline__ uint32_t fold_mask_int(const v4i32 (&a)[4], float st, uint32_t bits, uint32_t thr_o, float e2,
                                                  bool& pub) {
  int mx = max3i(a[0][0], a[0][1], a[0][2]);
  mx = max3i(mx, a[0][3], a[1][0]);
  mx = max3i(mx, a[1][1], a[1][2]);
  mx = max3i(mx, a[1][3], a[2][0]);
  mx = max3i(mx, a[2][1], a[2][2]);
  mx = max3i(mx, a[2][3], a[3][0]);
  mx = max3i(mx, a[3][1], a[3][2]);
  mx = max(mx, a[3][3]);
  const float tf = thr_o ? unord(thr_o) - e2 : -__builtin_inff();
  constexpr int kBig = 1 << 30;
  int t;
  if (!(tf > -__builtin_inff())) {
    t = -kBig;  // no bound yet: every value
  } else if (!(st > 0.f)) {
    t = 0.f >= tf ? -kBig : kBig;  // every A of the tile is 0
  } else {
    const float c = tf * __builtin_amdgcn_rcpf(st);
    const float cl = floorf(c - fabsf(c) * 0x1p-19f) - 2.f;
    t = (int)fminf(fmaxf(cl, -1073741824.f), 1073741824.f);
  }
  pub = mx >= t;
  uint32_t pm = 0;
  if (pub) {
    const int tm1 = t - 1;
#pragma unroll
    for (int r = 15; r >= 0; --r)  // MSB first: value r ends at bit r
      pm = __builtin_amdgcn_alignbit(pm, (uint32_t)(tm1 - a[r >> 2][r & 3]), 31);
    pm &= (bits & 0xffu) | ((bits >> 8) & 0xff00u);
  }
  return pm;
}
// One passing value of this lane (the lowest bit of pm, cleared) into its list.
template <int KL>
__device__ __forceinline__ void fold_trip(const v4i32 (&a)[4], float st, int rbase, uint32_t& pm, uint64_t (&L)[KL],
                                          uint32_t& drop_o) {
  const int r = __builtin_ctz(pm);
  pm &= pm - 1;
  // value r: a select tree on r's bits as bit-field inserts (15 v_bfi_b32); the masks go through
  // an empty asm so the compiler cannot turn the tree back into an indexed (scratch) read of a
  int m3 = -((r >> 3) & 1), m2 = -((r >> 2) & 1), m1 = -((r >> 1) & 1), m0 = -(r & 1);
  asm volatile("" : "+v"(m3), "+v"(m2), "+v"(m1), "+v"(m0));
  int v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (a[(j + 8) >> 2][j & 3] & m3) | (a[j >> 2][j & 3] & ~m3);
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = (v[j + 4] & m2) | (v[j] & ~m2);
#pragma unroll
  for (int j = 0; j < 2; ++j) v[j] = (v[j + 2] & m1) | (v[j] & ~m1);
  const int av = (v[1] & m0) | (v[0] & ~m0);
  const float s = (float)av * st;
  const int row = rbase + (r & 7) + 16 * (r >> 3);
  // insert, unconditionally and without a dependency chain: with c_i = (L_i > key) and the list
  // sorted, the new entry i is c_{i-1} ? (c_i ? L_i : key) : L_{i-1} (c_{-1} = true), and the
  // smallest of L and the key falls out — the evicted entry when the key goes in, the key itself
  // when it does not; either way a value this lane looked at and did not keep (an empty entry
  // falls out as 0, which max ignores).  KL independent compares, no branch: the list stays in
  // the same registers from trip to trip.
  const uint64_t key = ((uint64_t)ord(s) << 32) | (uint32_t)(~(uint32_t)row);
  bool c[KL];
#pragma unroll
  for (int i = 0; i < KL; ++i) c[i] = L[i] > key;
  const uint64_t k = c[KL - 1] ? key : L[KL - 1];
#pragma unroll
  for (int i = KL - 1; i > 0; --i) L[i] = c[i - 1] ? (c[i] ? L[i] : key) : L[i - 1];
  L[0] = c[0] ? L[0] : key;
  drop_o = max(drop_o, (uint32_t)(k >> 32));
}
// PUBCH (kModePubOnChange, production since round 5): the list's best is published only when it rose above what this lane
// published last (the slot table holds the same values either way: an atomic max with a value already
// published is a no-op), so a slow-path entry that does not raise the list's best issues no atomic.
template <int KL, bool PUBCH = false>
__device__ __forceinline__ void fold_end(const uint64_t (&L)[KL], uint32_t& thr_o, bool pub, v4i32 tau_rsrc,
                                         uint32_t slot_voff, uint32_t& pubd) {
  if (pub) {
    const uint32_t own = (uint32_t)(L[KL - 1] >> 32);
    thr_o = own > thr_o ? own : thr_o;
    const uint32_t best = (uint32_t)(L[0] >> 32);
    if (!PUBCH || best > pubd) {
      batomic_umax(tau_rsrc, slot_voff, best);
      pubd = best;
    }
  }
}
// Debug kModeSortMerge (round 5): a wave whose lanes pass many values at once (the first tiles, where
// every value passes: 16 pop-loop trips each) folds them as one sorted merge instead of one trip per
// value: the lane's 16 keys (orderable A << 32 | ~row, 0 = not passing) are sorted by a bitonic network,
// and the top KL of the union with the list come out of a bitonic split (max(L[i], K[KL-1-i]): the
// top KL of the union, as a bitonic sequence) re-sorted; the best key not kept is
// max(min(L[i], K[KL-1-i]), K[KL]) — what the trips would have recorded in drop, and the same list.
__device__ __forceinline__ void cx_desc64(uint64_t& a, uint64_t& b) {
  const bool sw = a < b;
  const uint64_t hi = sw ? b : a, lo = sw ? a : b;
  a = hi;
  b = lo;
}
template <int N>
__device__ __forceinline__ void bitonic_desc64(uint64_t (&v)[N]) {
#pragma unroll
  for (int k = 2; k <= N; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int l = i ^ j;
        if (l > i) {
          if ((i & k) == 0)
            cx_desc64(v[i], v[l]);
          else
            cx_desc64(v[l], v[i]);
        }
      }
}
template <int KL>
__device__ __forceinline__ void fold_sorted(const v4i32 (&a)[4], float st, int rbase, uint32_t pm, uint64_t (&L)[KL],
                                            uint32_t& drop_o) {
  static_assert(KL <= 16, "one 16-key merge");
  uint64_t K[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float s = (float)a[r >> 2][r & 3] * st;
    const int row = rbase + (r & 7) + 16 * (r >> 3);
    const uint64_t key = ((uint64_t)ord(s) << 32) | (uint32_t)(~(uint32_t)row);
    K[r] = (pm >> r) & 1u ? key : 0ull;
  }
  bitonic_desc64<16>(K);
  uint64_t M[16];
  uint32_t d = KL < 16 ? (uint32_t)(K[KL] >> 32) : 0u;
#pragma unroll
  for (int i = 0; i < KL; ++i) {
    const uint64_t x = L[i], y = K[KL - 1 - i];
    M[i] = x > y ? x : y;
    const uint64_t lo = x > y ? y : x;
    d = max(d, (uint32_t)(lo >> 32));
  }
#pragma unroll
  for (int i = KL; i < 16; ++i) M[i] = 0ull;  // (constant: the network folds them away)
  bitonic_desc64<16>(M);
#pragma unroll
  for (int i = 0; i < KL; ++i) L[i] = M[i];
  drop_o = max(drop_o, d);
}
constexpr int kSortMergeTrips = 8;  // (a merge costs about as much VALU as 8 trips)
template <int KL, bool REG = true, bool FMASK = false, bool SORTM = false, bool PUBCH = false>
__device__ __forceinline__ void fold_screen(const v4i32 (&a)[4], float st, uint32_t bits, uint64_t* Ls, uint64_t (&L)[KL],
                                            uint32_t& thr_o,
                                            float e2, uint32_t& drop_o, int rbase, v4i32 tau_rsrc, uint32_t slot_voff,
                                            uint32_t& pubd) {
  if constexpr (REG) {
    bool pub;
    uint32_t pm = FMASK ? fold_mask(a, st, bits, thr_o, e2, pub) : fold_mask_int(a, st, bits, thr_o, e2, pub);
    int many = 0;
    if constexpr (SORTM) {  // the wave's largest pass count: one sorted merge when it is high
      int c = __popc(pm);
#pragma unroll
      for (int off = 32; off; off >>= 1) c = max(c, __shfl_xor(c, off));
      many = c >= kSortMergeTrips;
    }
    if (SORTM && many) {
      fold_sorted<KL>(a, st, rbase, pm, L, drop_o);
    } else {
      // one passing value per lane per trip: the wave makes max-over-lanes(popcount) trips, not one
      // trip per position some lane passes at
      while (pm) fold_trip<KL>(a, st, rbase, pm, L, drop_o);
    }
    fold_end<KL, PUBCH>(L, thr_o, pub, tau_rsrc, slot_voff, pubd);
  } else {
    const float thr = thr_o ? unord(thr_o) - e2 : -__builtin_inff();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float s = (float)a[r >> 2][r & 3] * st;
      if (((bits >> ((r & 7) + 16 * (r >> 3))) & 1u) && s >= thr) {
        const int row = rbase + (r & 7) + 16 * (r >> 3);
        const uint64_t key = ((uint64_t)ord(s) << 32) | (uint32_t)(~(uint32_t)row);
        const uint64_t last = Ls[(KL - 1) * 64];
        if (key > last) {
          if (last) drop_o = max(drop_o, (uint32_t)(last >> 32));  // evicted
          int i = KL - 1;
          for (; i > 0; --i) {
            const uint64_t prev = Ls[(i - 1) * 64];
            if (prev >= key) break;
            Ls[i * 64] = prev;
          }
          Ls[i * 64] = key;
        } else {
          drop_o = max(drop_o, ord(s));  // looked at, not kept
        }
      }
    }
    const uint32_t own = (uint32_t)(Ls[(KL - 1) * 64] >> 32);
    thr_o = own > thr_o ? own : thr_o;
    batomic_umax(tau_rsrc, slot_voff, (uint32_t)(Ls[0] >> 32));
  }
}

// ---- round-5 fold (debug MODE kModeFold2; measured SLOWER than round 4's 64-bit list, which production keeps:
// 0.407 against 0.340 ms at the 8-GPU shard, 2.327 against 2.104 ms at 10M rows, one box, interleaved,
// profiles/r05/k10_fold2_tb_ab_*.txt — the fewer VALU ops per insert did not pay for the larger code and
// register footprint, 251 against 229 VGPRs) ------------------------------------------------------------
// The lane's list as KL orderable scores S (best first, 0 = empty) beside their rows R.  An insert is
// S'_i = max(S_i, min(S_{i-1}, key)) (the median of three for a sorted list) and, for the rows, with
// c_i = (S_i >= key): R'_i = c_i ? R_i : (c_{i-1} ? row : R_{i-1}) — one compare, two selects and a
// min/max pair per entry against round 4's 64-bit compare and four selects.  Equal scores keep their
// order (the older, lower row ahead); which of two equal-score rows a full list keeps does not matter:
// the select ranks survivors by their exact scores, and what falls out (min of the last entry and the
// key) is the score `drop` records either way.  key 0 (an empty entry, below every real score) is a
// no-op insert.
template <int KL>
__device__ __forceinline__ void insert_s(uint32_t (&S)[KL], uint32_t (&R)[KL], uint32_t key, uint32_t row,
                                         uint32_t& drop_o) {
  bool c[KL];
#pragma unroll
  for (int i = 0; i < KL; ++i) c[i] = S[i] >= key;
  drop_o = max(drop_o, min(S[KL - 1], key));
#pragma unroll
  for (int i = KL - 1; i > 0; --i) {
    R[i] = c[i] ? R[i] : (c[i - 1] ? row : R[i - 1]);
    S[i] = max(S[i], min(S[i - 1], key));
  }
  R[0] = c[0] ? R[0] : row;
  S[0] = max(S[0], key);
}
// The pass test of the slow path, (float)D * s_t >= tf, as ONE integer threshold per lane: t = min{D :
// fl(fl(D) s_t) >= tf} (fl(D) exact: |D| < 2^24; the product's rounding is monotone in D, so the
// passing D form an up-set).  From c = tf / s_t (v_rcp: |c - tf/s_t| < 1 for |c| <= 2^22) two steps
// down while P(t - 1) and two up while !P(t) reach it exactly; `ok` verifies P(t) && !P(t - 1) (false
// only for |c| > 2^22, where the wave takes the float mask instead).
__device__ __forceinline__ int pass_threshold(float st, float tf, bool& ok) {
  auto P = [&](int d) { return (float)d * st >= tf; };
  if (!(tf > -__builtin_inff())) {
    ok = true;
    return INT_MIN;  // no bound yet: every value passes
  }
  if (!(st > 0.f)) {
    ok = true;
    return 0.f >= tf ? INT_MIN : INT_MAX;  // every A of the tile is 0
  }
  const float c = tf * __builtin_amdgcn_rcpf(st);
  ok = fabsf(c) <= 4194304.f;
  int t = ok ? (int)ceilf(c) : 0;
  t -= P(t - 1) ? 1 : 0;
  t -= P(t - 1) ? 1 : 0;
  t += P(t) ? 0 : 1;
  t += P(t) ? 0 : 1;
  ok = ok && P(t) && !P(t - 1);
  return t;
}
// The pass mask of the round-5 fold: bit r set = value r (acc[r >> 2][r & 3], row (r & 7) + 16 (r >> 3) of
// the lane's half-tile) reaches the threshold; `all` before the live bits (pub: the lane publishes its
// list's best), the return value after them.
__device__ __forceinline__ uint32_t pass_mask_int(const v4i32 (&a)[4], int t, uint32_t bits, uint32_t& all) {
  uint32_t pm = 0;
#pragma unroll
  for (int r = 0; r < 16; ++r) pm |= a[r >> 2][r & 3] >= t ? (1u << r) : 0u;
  all = pm;
  return pm & ((bits & 0xffu) | ((bits >> 8) & 0xff00u));
}

// X: int8 codes [ntiles * 32][D]; tmeta: per tile {f32 scale, u32 live word, 0, 0}; stats: the
// quantiser's maxima (stats[2] = max tile scale); Qc: int8 query codes [nq_pad][D];
// qe2: [nq_pad] e2 per query (units of the query's scale).  Outputs per (query, list): KL
// candidates (A, row) sorted best first, empty tail (-inf, kEmptyRow), and the list's drop.
// MODE: 0 production; debug-build ablations (k10_dbg.hip): 1 = no top-k fold (accumulators kept
// live), 2 = resident fragments NOT laundered (hipcc's own vmcnt waits stay in the loop), 4 = A
// fragments prefetched 2 k-steps ahead (d 768 only), 8 = no corpus stream after the prologue (MFMA +
// LDS only; wrong scores, timing only), 32 = count slow-path entries (threshold slot 15 of each
// wave's first query), 64 = the fast path on the store-wide integer bound (max tile scale) instead
// of the tile's own scale, 128 = the epilogue in place at each tile's end (no alternating accumulators),
// 256 = kernel 6's slot-table bound (min over KL slots) instead of the KL-th largest of 16, 512 = the
// slow path compiled in but never taken (wrong results; separates its cost from the code's presence),
// 1024 = the slow path's serial LDS list insert instead of the register-resident list, 16 = the slot
// table re-read at every one of the first 16 tiles, 2048 = issue priority for a wave in the slow path,
// 32768 = the ring without stage barriers (DEC below).
// debug MODE bits of round 5 (k10_dbg.hip; variant = 10^7 * RING + MODE)
constexpr int kModeEpiLate = 131072;
constexpr int kModeStagger = 262144;
constexpr int kModePermBounds = 524288;
constexpr int kModeFold2 = 1048576;  // the round-5 u32-score fold (debug; slower, see above)
constexpr int kModeTileBarrier = 2097152;  // one wait + barrier per tile (TB below; RING 12)
constexpr int kModeFloatMask = 4194304;  // the slow path's float pass mask (fold_mask) instead of fold_mask_int
constexpr int kModePubOnChange = 8388608;  // publish a list's best only when it rose (production; variant encoding 10^8 RING + MODE)
constexpr int kModeSortMerge = 16384;  // a wave with >= 8 passes in some lane folds by one sorted merge (debug)
// round 6 (debug A/B): only wave 0 DMAs each tile's 16-B record (1 KB: 64 lane copies) instead of all 8 waves
// (the per-tile barrier makes it visible to every wave); the other waves' counted waits drop the records
constexpr int kModeMetaOne = 33554432;
template <int KL, int D, bool MASK, int RING = kRing, int MODE = 0, int NW = kWaves>
__global__ __launch_bounds__(64 * NW, 1) void scan_screen_kernel(const int8_t* __restrict__ X, const uint4* __restrict__ tmeta,
                                                             const uint32_t* __restrict__ stats,
                                                             const int8_t* __restrict__ Qc, const float* __restrict__ qe2,
                                                             int nq, int ntiles, uint32_t* __restrict__ tau,
                                                             float* __restrict__ cand_s, int* __restrict__ cand_r,
                                                             uint32_t* __restrict__ drops, int64_t n_lists,
                                                             const uint32_t* __restrict__ mask, uint32_t* __restrict__ xb,
                                                             uint32_t* __restrict__ xw) {
  constexpr int NKS = D / 64;    // 64-deep k-steps per tile
  constexpr int NST = D / kSK;   // stages per tile
  constexpr int KPS = kSK / 64;  // k-steps per stage (4)
  static_assert(D % kSK == 0, "D must be a multiple of 256");
  static_assert(KL <= 16, "the bound is the KL-th largest of 16 slots");
  static_assert(NW == 8 || NW == 2, "8 waves (256 queries) or 2 waves (64 queries) per workgroup");
  constexpr int NT = 64 * NW;          // threads
  constexpr int QG = NW * kQW;         // queries per workgroup
  constexpr int GPW = 8 / NW;          // LDS-DMA pieces per wave per stage (8 KB / 1 KB / NW)
  constexpr int TAUB = tau_bytes_nw<NW>();
  static_assert(TAUB / 1024 / NW == kTauGPW, "slot-table DMA pieces per wave");
  __shared__ __attribute__((aligned(1024))) uint8_t lds[lds_bytes<KL, RING, NW>()];
  constexpr int kTauOff = tau_off<RING>();
  constexpr int kMetaOff = meta_off<RING>();
  constexpr int kListOff = list_off<RING, NW>();

  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int half = lane >> 5;
  const int range = blockIdx.x;
  const int qg = blockIdx.y * QG;
  const int q = qg + w * kQW + 16 * ((lane >> 4) & 1) + (lane & 15);  // after the pair swap
  const int nblk = gridDim.x;
  // The tiles of this block: tb0 + i * tstride, i < nt.  Static split: tiles range, range + nblk, ...
  // XCD-balanced split (production; debug MODE 4096 keeps the static one): block b runs on XCD b % 8, and
  // the XCDs do not run at one speed under the power limit (2.10 to 2.20 ms per block at
  // 10M rows, the slow XCD's blocks last in every launch).  XCD x takes the tile range
  // [T_x, T_x+1) in proportion to its weight (the speed it measured in earlier launches, a snapshot
  // the query quantiser took for this launch, so every block computes the same split), its 32 blocks
  // interleaved in it.  Any split of the tiles into disjoint lists is exact.
  // (>= 64 tiles per block on average: with weights in [0.5, 2] every block keeps >= 2 tiles)
  const bool bal = (MODE & 4096) == 0 && xb != nullptr && xw != nullptr && (nblk & 7) == 0 && ntiles >= 64 * nblk;
  const int xc = range & 7;
  int tb0 = range, tstride = nblk, nt = range < ntiles ? (ntiles - range + nblk - 1) / nblk : 0;
  if (bal) {
    uint64_t pre = 0, tot = 0;
    uint32_t wx = 1;
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      const uint32_t wv = xb[x];  // (1024 = 1.0, clamped by the quantiser to [512, 2048])
      pre += x < xc ? wv : 0u;
      wx = x == xc ? wv : wx;
      tot += wv;
    }
    const int t_lo = (int)((uint64_t)ntiles * pre / tot), t_hi = (int)((uint64_t)ntiles * (pre + wx) / tot);
    const int bpx = nblk >> 3;
    tb0 = t_lo + (range >> 3);
    tstride = bpx;
    nt = tb0 < t_hi ? (t_hi - tb0 + bpx - 1) / bpx : 0;
  }
  auto tile_of = [&](int i) -> int { return tb0 + i * tstride; };
  const int S = nt * NST;
  const uint64_t t_start = wall_clock64();
  if (S == 0) return;
#ifdef RFX_K10_BLOCK_TIMES
  if constexpr ((MODE & 65536) != 0)
    if (tid == 0 && range < 1024 && blockIdx.y == 0) {
      g_k10_bt[range][0] = wall_clock64();
      g_k10_bt[range][2] = __builtin_amdgcn_s_memtime();
    }
#endif
  const int lst = range * 2 + half;
  const float e2 = qe2[q];
  const float smax = __uint_as_float(stats[2]);  // max tile scale of the store

  {
    uint4* tz = (uint4*)(lds + kTauOff);
#pragma unroll
    for (int i = 0; i < TAUB / 16 / NT; ++i) tz[tid + NT * i] = uint4{0u, 0u, 0u, 0u};
  }
  uint64_t* const Ls = (uint64_t*)(lds + kListOff) + (w * KL) * 64 + lane;  // debug MODE 1024's list
  if constexpr (NW == kWaves)
#pragma unroll
    for (int i = 0; i < KL; ++i) Ls[i * 64] = 0ull;
  uint32_t* const ready = (uint32_t*)(lds + ctr_off<KL, RING, NW>());  // MODE 32768: [RING] pieces landed
  uint32_t* const done = ready + 16;                                  // [RING] waves done reading
  if (tid < 32) ready[tid] = 0u;  // (the same zeros as the list init above)
  constexpr bool F2 = (MODE & kModeFold2) != 0 && (MODE & 1024) == 0;  // the round-5 fold (debug)
  // (d 1024 holds 128 resident fragment registers: the unrolled per-position inserts would spill there)
  constexpr bool SWEEP = D == 768;
  uint64_t Lr[KL];  // production: the lane's 64-bit list in registers for the whole scan
  uint32_t LS[KL], LR[KL];  // debug kModeFold2: scores and rows (insert_s)
#pragma unroll
  for (int i = 0; i < KL; ++i) {
    Lr[i] = 0ull;
    LS[i] = 0u;
    LR[i] = 0u;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // resident query codes (B[k][col] of 16x16x64 i8): query block qb, lane holds col 16 qb + (lane & 15),
  // k = 64 ks + 16 (lane >> 4) + j; the A fragments below use the same k map, so the i32 dot is exact
  uint4 bq[2 * NKS];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int8_t* qa = Qc + (int64_t)(qg + w * kQW + 16 * qb + (lane & 15)) * D + 16 * (lane >> 4);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) bq[2 * ks + qb] = *(const uint4*)(qa + 64 * ks);
  }

  // LDS-DMA piece p of a stage: slot bytes [1024 p, +1024) = rows 4p .. 4p+3 (256 B each); lane ->
  // (row 4p + (lane >> 4), position lane & 15) <- source chunk position ^ (row & 15).  Wave w issues pieces
  // w + NW u, u < GPW (one piece per wave in the 8-wave kernel, four in the 2-wave kernel).
  uint32_t laneoff[GPW];
#pragma unroll
  for (int u = 0; u < GPW; ++u) {
    const int pr = 4 * (w + NW * u) + (lane >> 4);
    laneoff[u] = (uint32_t)(pr * D + (((lane & 15) ^ (pr & 15)) * 16));
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  // The tile metadata (scale, live word) rides the same counted stream: with the piece of a tile's
  // first stage, every wave also DMAs the tile's 16-B record (64 lane copies, identical bytes from
  // every wave) into meta slot (tile % kMR), read by the epilogue's slow path from LDS.
  const v4i32 meta_rsrc = make_rsrc(tmeta);
  // (per-tile barrier schedule only: see kModeMetaOne)
  constexpr bool META1 = (MODE & kModeMetaOne) != 0 && (MODE & kModeTileBarrier) != 0 && (MODE & 32768) == 0 &&
                         (MODE & 8) == 0;
  auto issue_piece = [&](int gi, int slot) {
    const bool first = gi % NST == 0;  // (counted on the unclamped index: the waits stay exact)
    gi = gi < S ? gi : S - 1;  // tail: harmless duplicate loads keep the counted waits exact
    const int ti = gi / NST;
    const int si = gi - ti * NST;
    const int8_t* tbase = X + (int64_t)tile_of(ti) * kTM * D + si * kSK;
    const v4i32 rs = make_rsrc(tbase);
#pragma unroll
    for (int u = 0; u < GPW; ++u) {
      const uint32_t dst =
          __builtin_amdgcn_readfirstlane(lds_base + (uint32_t)(slot * kSlot) + (uint32_t)((w + NW * u) * 1024));
      bdma_nt(rs, laneoff[u], dst);  // codes are read once per batch
    }
    if (first && (!META1 || w == 0)) {
      const uint32_t mdst = __builtin_amdgcn_readfirstlane(lds_base + kMetaOff + (uint32_t)((ti % kMR) * 1024));
      bdma(meta_rsrc, (uint32_t)tile_of(ti) * 16u, mdst);
    }
  };
  const v4i32 tau_rsrc = make_rsrc(tau);
  auto issue_tau = [&]() {
#pragma unroll
    for (int u = 0; u < kTauGPW; ++u) {
      const int i = w + NW * u;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + kTauOff + i * 1024);
      bdma_sc1(tau_rsrc, (uint32_t)(qg * kTauW * 4 + tid * 16 + u * NW * 1024), dst);
    }
  };

  uint32_t thr = 0u, drop = 0u;
  uint32_t pubd = 0u;  // the list's best this lane published last (kModePubOnChange)
  // Debug MODE 64's fast path, bounds on the raw i32 dot D (no per-tile data): every tile scale s_t <= smax, so a
  // lane value with D < ibound(thr) has fl(D s_t) < thr - e2 and is never looked at (proof in
  // DESIGN §4.10).  ti_own: this lane's query (after the pair swap); ti_oth: the query the partner
  // lane (lane ^ 16) owns, whose values this lane also holds before the swap.
  auto ibound = [&](uint32_t t_o) -> int {
    if (!t_o) return INT_MIN;
    const float tf = unord(t_o) - e2;
    if (!(tf > 0.f)) return INT_MIN;
    if (!(smax > 0.f)) return INT_MAX;  // every A is 0 < tf
    const float qv = __fdiv_rn(tf, smax) * 0.999999f;
    return qv >= 2.0e9f ? INT_MAX : (int)floorf(qv);
  };
  int ti_own = INT_MIN, ti_oth = INT_MIN;
  // Production fast path: the slow path's own test, (float)D * s_t >= thr - e2, on the lane's max D
  // per query with the tile's scale from the LDS metadata slot (one ds_read per tile).  Float
  // multiplication by s_t >= 0 is monotone, so the max passes whenever any value would.  Against
  // the store-wide smax bound it skips the tiles whose scale lies below smax (measured: 17 % of
  // wave-tiles entered the slow path with the smax bound).
  const bool odd = ((lane >> 4) & 1) != 0;
  // a padded query (q >= nq: code 0, every A = 0) never enters the slow path: its bound is +inf and its
  // live bits are cleared (otherwise every one of its A = 0 values would reach bound - e2 = 0 - 0 forever)
  const bool qlive = q < nq;
  float tf_own = qlive ? -__builtin_inff() : __builtin_inff();
  float tf_oth = (odd ? q - 16 : q + 16) < nq ? -__builtin_inff() : __builtin_inff();  // the partner lane's query
  auto set_bounds = [&]() {
    if constexpr ((MODE & 64) != 0) {
      ti_own = ibound(thr);
      ti_oth = __shfl_xor(ti_own, 16);
    } else {
      tf_own = !qlive ? __builtin_inff() : thr ? unord(thr) - e2 : -__builtin_inff();
      if constexpr ((MODE & kModePermBounds) != 0) {
        // the partner lane's (lane ^ 16) bound by one v_permlane16_swap: no ds_bpermute round trip
        const uint32_t b = __float_as_uint(tf_own);
        const auto r = __builtin_amdgcn_permlane16_swap(b, b, false, false);
        tf_oth = __uint_as_float(odd ? r[0] : r[1]);
      } else {
        tf_oth = __shfl_xor(tf_own, 16);
      }
    }
  };
  // the quantiser's seed bound for the lane's query (k_screen.hip kSeedRows: a lower bound of a_k, 0 = none),
  // in the words after the XCD split's
  if (xb != nullptr) {
    thr = xb[kXbWords + q];
    set_bounds();
  }
  // MODE 32 (debug) counts slow-path entries in slot 15 of each wave's first query: 15 slots then;
  // MODE 256 (debug): kernel 6's bound, the min over KL slots (list j -> slot j % KL)
  constexpr int kSlots = (MODE & 256) != 0 ? KL : (MODE & 32) != 0 ? kTauW - 1 : kTauW;
  const uint32_t slot_voff = (uint32_t)(q * kTauW + lst % kSlots) * 4u;
  const uint8_t* const tq = lds + kTauOff + (w * kQW + (lane & 15) + 16 * ((lane >> 4) & 1)) * (kTauW * 4);
  // A fragment of row block rb, k-step kk of a slot: row 16 rb + (lane & 15), chunk 4 kk + (lane >> 4)
  const uint8_t* const frag_base = lds + (lane & 15) * kRowB;
  const int sw = lane & 15;
  struct Frag {
    uint4 a[2];
  };
  auto read_frag = [&](int slot, int kk) -> Frag {
    const uint8_t* p = frag_base + slot * kSlot + (((4 * kk + (lane >> 4)) ^ sw) << 4);
    Frag f;
    f.a[0] = *(const uint4*)p;
    f.a[1] = *(const uint4*)(p + 16 * kRowB);
    return f;
  };

  // Schedule: stage h's piece goes out at k-step 0 of stage h - (RING - 1) into the slot freed at
  // stage h - RING's barrier; fragments are read one k-step ahead; the stage-end wait + barrier sit
  // at k-step KPS - 1.
  constexpr int PF = (D == 768 && (MODE & 4) == 0) ? 2 : 1;  // d 1024: 16 k-steps per tile, PF 2 would not realign
  constexpr int NF = PF + 1;
  constexpr int KB = KPS - PF;
  // Debug MODE 32768 (DEC): no stage barrier.  A wave waits only for the 8 pieces of its next stage (the
  // per-slot `ready` counter) and, before a DMA into a slot, for every wave to be done reading the
  // slot's previous stage (`done`); LAG free slots let a wave that is in the slow path fall up to LAG
  // stages behind the others without stalling them.  Pieces go out AHEAD = RING - 1 - LAG stages early.
  constexpr bool DEC = (MODE & 32768) != 0 && (MODE & 8) == 0;
  constexpr int LAG = DEC ? 3 : 0;
  // Debug kModeTileBarrier (TB): one wait + barrier per TILE (at its last stage) instead of one per stage.
  // Stage h's piece goes out at k-step 0 of stage h - AHEAD, AHEAD = RING - NST, into the slot of stage
  // h - RING, which the barrier of the tile before has freed; the tile-t barrier waits for every stage of
  // tile t + 1.  A wave in the slow path then has the rest of the tile's k-steps, not one stage's, before
  // the next rendezvous.  The slot table refreshed after tile t's barrier is read at tile t + TBD's start
  // (TBD: the first tile whose barrier wait covers that refresh without waiting for younger pieces).
  constexpr bool TB = (MODE & kModeTileBarrier) != 0 && !DEC && (MODE & 8) == 0;
  constexpr int AHEAD = TB ? RING - NST : RING - 1 - LAG;
  static_assert(!TB || RING >= 2 * NST + 2, "TB: at least two stages beyond the next tile in flight");
  constexpr int TBD = TB ? ((RING - NST + NST - 1) / NST > 2 ? (RING - NST + NST - 1) / NST : 2) : 2;
  constexpr int RA = AHEAD + 1;           // the counted-wait arithmetic below is in stages in flight
  static_assert(AHEAD >= 3, "at least three stages in flight");
  constexpr int YNG = (RA - 2) * GPW;  // ops younger than the next stage
  static_assert((NST * KPS) % NF == 0, "fragment rotation must realign every tile");

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // resident queries landed before the counted stream
  if constexpr ((MODE & 2) == 0) launder(bq);
  issue_tau();
#pragma unroll
  for (int p = 0; p < AHEAD; ++p) issue_piece(p, p);
  if constexpr (TB) {
    // tile 0 landed: younger are the pieces of stages NST .. AHEAD - 1 and their tile records
    constexpr int NMT = (AHEAD - 1) / NST;  // records of stages NST, 2 NST, ... <= AHEAD - 1
    if (META1 && w != 0)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"((AHEAD - NST) * GPW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"((AHEAD - NST) * GPW + NMT) : "memory");
  } else {
    // stage 0 landed: younger are stages 1 .. AHEAD - 1 and the metadata records issued with stages
    // 0 .. AHEAD - 1 (with piece 0's own record after it)
    constexpr int NM0 = (AHEAD - 1) / NST + 1;
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(YNG + NM0) : "memory");
  }
  if constexpr (DEC)
    if (lane == 0) lds_arrive(&ready[0]);  // stage 0's first use of slot 0 counts like every other
  asm volatile("s_barrier" ::: "memory");

  Frag fr[NF];
#pragma unroll
  for (int p = 0; p < PF; ++p) fr[p] = read_frag(0, p);
  // Accumulators alternate between tiles: the epilogue of tile it - 1 runs right after tile it's
  // first k-step of MFMAs (production), so its VALU / LDS work overlaps the matrix cores instead of
  // waiting for the MFMA pipeline to drain at every tile end (debug MODE 128: epilogue in place).
  v4i32 accA[4], accB[4];  // [rb * 2 + qb]
  auto epilogue = [&](const int it, v4i32(&acc4)[4]) {
    const int tile = tile_of(it);
    // Fast path: the max D of each of the lane's two queries, scaled by the tile's scale, against the
    // query's bound (qb 0 values in acc4[0], acc4[2]; qb 1 in acc4[1], acc4[3]).  Only when some lane of the wave
    // may hold a row to look at: the tile's scale and live word (LDS metadata slot), the pair swap (even
    // 16-lane row keeps query n, odd keeps 16 + n) and the exact fold.
    int m0 = max3i(acc4[0][0], acc4[0][1], acc4[0][2]);
    int m1 = max3i(acc4[1][0], acc4[1][1], acc4[1][2]);
    m0 = max3i(m0, acc4[0][3], acc4[2][0]);
    m1 = max3i(m1, acc4[1][3], acc4[3][0]);
    m0 = max3i(m0, acc4[2][1], acc4[2][2]);
    m1 = max3i(m1, acc4[3][1], acc4[3][2]);
    m0 = max(m0, acc4[2][3]);
    m1 = max(m1, acc4[3][3]);
    bool hit;
    if constexpr ((MODE & 64) != 0) {  // debug: the store-wide integer bound (no per-tile data)
      hit = (odd ? m1 : m0) >= ti_own || (odd ? m0 : m1) >= ti_oth;
    } else {
      const float st_t = *(const float*)(lds + kMetaOff + (it % kMR) * 1024 + lane * 16);
      hit = (float)(odd ? m1 : m0) * st_t >= tf_own || (float)(odd ? m0 : m1) * st_t >= tf_oth;
    }
    if constexpr ((MODE & 512) != 0) hit = hit && nq < 0;  // debug: the slow path compiled in, never taken
    if constexpr ((MODE & 1) == 0) {
      if (__builtin_amdgcn_ballot_w64(hit)) {
        // debug MODE 2048: the wave in the slow path takes issue priority over its SIMD partner (which
        // keeps issuing MFMAs), so it reaches the next stage barrier sooner
        if constexpr ((MODE & 2048) != 0) __builtin_amdgcn_s_setprio(3);
        if constexpr ((MODE & 32) != 0)  // debug: count slow-path entries per wave (unused threshold slot 15)
          if (lane == 0) atomicAdd(tau + (int64_t)(qg + w * kQW) * kTauW + 15, 1u);
        const uint2 md = *(const uint2*)(lds + kMetaOff + (it % kMR) * 1024 + lane * 16);
        const float st = __uint_as_float(md.x);
        uint32_t lw = qlive ? md.y : 0u;
        if constexpr (MASK) lw &= mask[tile];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const auto r = __builtin_amdgcn_permlane16_swap((uint32_t)acc4[2 * rb][i], (uint32_t)acc4[2 * rb + 1][i], false, false);
            acc4[2 * rb][i] = (int)r[0];
            acc4[2 * rb + 1][i] = (int)r[1];
          }
#ifdef RFX_K10_BLOCK_TIMES
        if constexpr ((MODE & 8192) != 0) {
          bool pub_;
          const uint32_t pm_ = (MODE & kModeFloatMask) != 0 ? fold_mask(acc4, st, lw >> (8 * half), thr, e2, pub_)
                                                             : fold_mask_int(acc4, st, lw >> (8 * half), thr, e2, pub_);
          int c = __popc(pm_);
#pragma unroll
          for (int off = 32; off; off >>= 1) c = max(c, __shfl_xor(c, off));
          if (lane == 0) {
            atomicAdd(&g_k10_trips[0][it < 63 ? it : 63], 1u);
            atomicAdd(&g_k10_trips[1][it < 63 ? it : 63], (unsigned)c);
          }
        }
#endif
        if constexpr (F2) {
          const uint32_t bits = lw >> (8 * half);
          const int rbase = tile * kTM + 8 * half;
          const float tf = thr ? unord(thr) - e2 : -__builtin_inff();
          bool ok;
          const int tq = pass_threshold(st, tf, ok);
          uint32_t all = 0, pm;
          if (__builtin_amdgcn_ballot_w64(!ok) == 0) {
            pm = pass_mask_int(acc4, tq, bits, all);
          } else {  // (|tf / s_t| > 2^22: the float test, exactly the round-4 mask)
            bool pubf;
            pm = fold_mask(acc4, st, bits, thr, e2, pubf);
            all = pubf ? 1u : 0u;
          }
          if (SWEEP && it < 2) {
            // the first tiles pass nearly every value (the list is empty, the bound not there yet): one
            // insert per row position, the value taken from its register (no select tree); lanes without
            // the position insert key 0 (a no-op)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float sv = (float)acc4[r >> 2][r & 3] * st;
              const uint32_t key = (pm >> r) & 1u ? ord(sv) : 0u;
              insert_s<KL>(LS, LR, key, (uint32_t)(rbase + (r & 7) + 16 * (r >> 3)), drop);
            }
          } else {
            while (pm) {
              const int r = __builtin_ctz(pm);
              pm &= pm - 1;
              int m3 = -((r >> 3) & 1), m2 = -((r >> 2) & 1), m1 = -((r >> 1) & 1), m0 = -(r & 1);
              asm volatile("" : "+v"(m3), "+v"(m2), "+v"(m1), "+v"(m0));
              int v[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = (acc4[(j + 8) >> 2][j & 3] & m3) | (acc4[j >> 2][j & 3] & ~m3);
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] = (v[j + 4] & m2) | (v[j] & ~m2);
#pragma unroll
              for (int j = 0; j < 2; ++j) v[j] = (v[j + 2] & m1) | (v[j] & ~m1);
              const int av = (v[1] & m0) | (v[0] & ~m0);
              insert_s<KL>(LS, LR, ord((float)av * st), (uint32_t)(rbase + (r & 7) + 16 * (r >> 3)), drop);
            }
          }
          if (all) {
            thr = LS[KL - 1] > thr ? LS[KL - 1] : thr;
            batomic_umax(tau_rsrc, slot_voff, LS[0]);
          }
        } else {
          fold_screen<KL, (MODE & 1024) == 0, (MODE & kModeFloatMask) != 0, (MODE & kModeSortMerge) != 0,
                      (MODE & kModePubOnChange) != 0>(
              acc4, st, lw >> (8 * half), Ls, Lr, thr, e2, drop,
                                                                              tile * kTM + 8 * half,
                                              tau_rsrc, slot_voff, pubd);
        }
        set_bounds();
        if constexpr ((MODE & 2048) != 0) __builtin_amdgcn_s_setprio(0);
      }
    } else if (hit && m0 == 12345 && m1 == 54321) {
      Ls[0] = 1;
    }
  };
  auto tile_body = [&](const int it, v4i32(&acc4)[4], v4i32(&accp)[4], const bool prev) {
    const int gbase = it * NST;
    if (it >= TBD && tau_refresh_tile<MODE>(it - TBD)) {
      thr = max(thr, (MODE & 256) != 0 ? tau_min<KL>(tq) : tau_kth<KL>(tq));
      set_bounds();
    }
    // metadata records younger than stage g+1's piece at stage s's wait: stages h in g+1 .. g+RING-1
    // with h % NST == 0
    auto nmeta = [&](int s) {
      int c = 0;
#pragma unroll
      for (int j = 1; j <= RA - 1; ++j) c += (s + j) % NST == 0;
      return c;
    };
    auto young = [&](int s) {
      const int dmax = (RA - 3 + NST - s) / NST;
      bool y = false;
#pragma unroll
      for (int d = 1; d <= dmax; ++d) y = y || (it >= d && tau_refresh_tile<MODE>(it - d));
      return y;
    };
#pragma unroll
    for (int s = 0; s < NST; ++s) {
      const int g = gbase + s;
      const int slot = g % RING;
#pragma unroll
      for (int kk = 0; kk < KPS; ++kk) {
        if constexpr ((MODE & 8) == 0)
          if (kk == 0) {
            const int h = g + AHEAD;
            if constexpr (DEC)  // the slot's previous stage h - RING read by all 8 waves
              if (h >= RING) lds_spin_ge(&done[h % RING], (uint32_t)(8 * (h / RING)));
            issue_piece(h, h % RING);
          }
        if (kk == KB && TB) {
          if (s == NST - 1) {
            // tile it + 1 landed: younger are the pieces of stages NST (it + 2) .. NST (it + 1) + RING - 1, their
            // tile records, and the refreshes issued after the last needed piece that tile it + 1 does not read
            // (tiles it + 2 - TBD .. it - 1); the refresh tile it + 1 reads (tile it + 1 - TBD) comes right
            // after that piece and is waited for
            constexpr int NMY = (RING - NST - 1) / NST;
            int nt_ = 0;
#pragma unroll
            for (int d = 1; d <= TBD - 2; ++d) nt_ += (it >= d && tau_refresh_tile<MODE>(it - d)) ? kTauGPW : 0;
            static_assert(kTauGPW == 2, "wait table below");
            if (META1 && w != 0) {  // (this wave issued no tile records)
              switch (nt_) {
#define RFX_K10_TWAIT(N)                                                                                      \
  case N:                                                                                                     \
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"((RING - 2 * NST) * GPW + N) : "memory");               \
    break;
                RFX_K10_TWAIT(0) RFX_K10_TWAIT(2)
                default:  // stricter, never looser
                  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"((RING - 2 * NST) * GPW) : "memory");
#undef RFX_K10_TWAIT
              }
            } else {
              switch (nt_) {
#define RFX_K10_TWAIT(N)                                                                                      \
  case N:                                                                                                     \
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"((RING - 2 * NST) * GPW + NMY + N) : "memory");         \
    break;
                RFX_K10_TWAIT(0) RFX_K10_TWAIT(2)
                default:  // stricter, never looser
                  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"((RING - 2 * NST) * GPW + NMY) : "memory");
#undef RFX_K10_TWAIT
              }
            }
            asm volatile("s_barrier" ::: "memory");
            if (tau_refresh_tile<MODE>(it)) issue_tau();
          }
        } else if (kk == KB) {
          if constexpr ((MODE & 8) == 0) {
            // younger than stage g+1's piece: stages g+2 .. g+RA-1 (YNG), the metadata records issued
            // with stages g+1 .. g+RA-1 that start a tile (nmeta(s): s = g mod NST), a refresh
            const int nm = nmeta(s) + (young(s) ? kTauGPW : 0);  // unrolled: a constant per stage
            static_assert(kTauGPW == 2 && RA <= 13, "wait table below covers nm <= 6");
            switch (nm) {
#define RFX_K10_WAIT(N)                                                                  \
  case N:                                                                                \
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(YNG + N) : "memory");            \
    break;
              RFX_K10_WAIT(0) RFX_K10_WAIT(1) RFX_K10_WAIT(2) RFX_K10_WAIT(3) RFX_K10_WAIT(4) RFX_K10_WAIT(5)
              default:  // (nm <= 6 for RING <= 13, NST >= 3): stricter, never looser
                asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(YNG + 6) : "memory");
#undef RFX_K10_WAIT
            }
          } else {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
          if constexpr (DEC) {
            // this wave's piece of stage g+1 landed and its reads of stage g completed (the wait above)
            if (lane == 0) {
              lds_arrive(&done[g % RING]);
              lds_arrive(&ready[(g + 1) % RING]);
            }
            if (s == NST - 1 && tau_refresh_tile<MODE>(it)) issue_tau();
            if (g + 1 < S) lds_spin_ge(&ready[(g + 1) % RING], (uint32_t)(8 * ((g + 1) / RING + 1)));
          } else {
            asm volatile("s_barrier" ::: "memory");
            if constexpr ((MODE & 8) == 0)
              if (s == NST - 1 && tau_refresh_tile<MODE>(it)) issue_tau();
          }
        }
        const int ks = s * KPS + kk;
        fr[(ks + PF) % NF] = kk + PF < KPS ? read_frag(slot, kk + PF) : read_frag((g + 1) % RING, kk + PF - KPS);
        const Frag& cur = fr[ks % NF];
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int qb = 0; qb < 2; ++qb)
            acc4[2 * rb + qb] = ks == 0 ? mfma_i8(cur.a[rb], bq[2 * ks + qb], v4i32{0, 0, 0, 0})
                                        : mfma_i8(cur.a[rb], bq[2 * ks + qb], acc4[2 * rb + qb]);
        if constexpr ((MODE & 128) == 0) {
          // where the epilogue of tile it - 1 runs inside tile it (its accumulators stay live until tile
          // it + 1's first k-step): production right after k-step 0 (before stage 0's barrier); debug
          // kModeEpiLate after the MFMAs of the barrier's k-step (a wave in the slow path then has a whole
          // stage of k-steps before the next barrier); kModeStagger: waves 4-7 (the SIMD partners of waves
          // 0-3) one stage later, so the two waves of a SIMD do not run their VALU epilogues together
          constexpr int EK = (MODE & kModeEpiLate) != 0 ? KB : 0;
          if (kk == EK && prev) {
            if constexpr ((MODE & kModeStagger) != 0 && NST >= 2) {
              if (s == 0 && w < 4) epilogue(it - 1, accp);
              if (s == 1 && w >= 4) epilogue(it - 1, accp);
            } else {
              if (s == 0) epilogue(it - 1, accp);
            }
          }
        }
      }
    }

  };
  if constexpr ((MODE & 128) != 0) {
    for (int it = 0; it < nt; ++it) {
      tile_body(it, accA, accB, false);
      epilogue(it, accA);
    }
  } else {
    int it = 0;
    for (; it + 1 < nt; it += 2) {
      tile_body(it, accA, accB, it > 0);
      tile_body(it + 1, accB, accA, true);
    }
    if (it < nt) {
      tile_body(it, accA, accB, it > 0);
      epilogue(it, accA);
    } else {
      epilogue(it - 1, accB);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (q < nq) {
    // entries below (the query's bound as it stands now) − e2 cannot be survivors: dropped here
    uint32_t sl[16];
#pragma unroll
    for (int j = 0; j < 16; ++j)
      sl[j] = j >= kSlots ? 0u : __hip_atomic_load(tau + (int64_t)q * kTauW + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t m = kth16<KL>(sl);
    if constexpr ((MODE & 256) != 0) {
      m = 0xffffffffu;
#pragma unroll
      for (int j = 0; j < KL; ++j)
        m = min(m, __hip_atomic_load(tau + (int64_t)q * kTauW + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    const uint32_t fin = max(thr, m);
    const float lo = fin ? unord(fin) - e2 : -__builtin_inff();
    const int64_t o = ((int64_t)q * n_lists + lst) * KL;
#pragma unroll
    for (int i = 0; i < KL; ++i) {
      const uint64_t key = F2 ? (((uint64_t)LS[i] << 32) | (uint32_t)~LR[i]) : (MODE & 1024) == 0 ? Lr[i] : Ls[i * 64];
      const float sc = unord((uint32_t)(key >> 32));
      const bool keep = (key >> 32) != 0 && sc >= lo;
      cand_s[o + i] = keep ? sc : -__builtin_inff();
      cand_r[o + i] = keep ? (int)(~(uint32_t)key) : kEmptyRow;
    }
    drops[(int64_t)q * n_lists + lst] = drop;
  }
  if (bal && blockIdx.y == 0 && tid == 0) {
    // speed bookkeeping for the next launches' split: the block's duration (wave 0's view) and tiles,
    // added to its XCD's sums (fire-and-forget atomics: no wait, nothing orders on them); the next
    // query quantiser turns the sums into weights (k_screen.hip)
    const uint64_t dt = wall_clock64() - t_start;
    __hip_atomic_fetch_add(xw + 8 + xc, (uint32_t)(dt < 0xffffffull ? dt : 0xffffffull), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(xw + 16 + xc, (uint32_t)nt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#ifdef RFX_K10_BLOCK_TIMES
  if constexpr ((MODE & 65536) != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0 && range < 1024 && blockIdx.y == 0) {
      g_k10_bt[range][1] = wall_clock64();
      g_k10_bt[range][3] = __builtin_amdgcn_s_memtime();
    }
  }
#endif
}

// Production schedule (round 5): one counted wait + barrier per TILE (kModeTileBarrier) over a 10-slot ring —
// against round 4's wait + barrier per stage over 8 slots: 2.004 against 2.054 ms at 10M rows, 0.3313 against
// 0.3393 ms at the 8-GPU shard (one box, interleaved, profiles/r05/k10_tb_ab_*.txt); round 4's schedule stays
// in the debug library as variant (8, 0).
// Production publishes a list's best only when it rose (kModePubOnChange: the same slot table, fewer
// atomics): 0.3344 against 0.3461 ms at the shard, 2.039 against 2.038 ms at 10M (profiles/r05/k10_pub_ab_*.txt).
constexpr int kProdRing = 10;
constexpr int kProdMode = kModeTileBarrier | kModePubOnChange;
// The 2-wave kernel (64 queries per workgroup, two workgroups per CU): the per-tile barrier over an 8-slot ring
// at d 768 (RING >= 2 NST + 2); at d 1024 (NST 4) the per-stage barrier over 8 slots (round 4's schedule), which
// keeps two workgroups within a CU's LDS
template <int D>
constexpr int w2_ring() { return 8; }
template <int D>
constexpr int w2_mode() { return D == 768 ? kProdMode : kModePubOnChange; }
#define RFX_K10_INSTANTIATE_W2(DV, NAME)                                                                      \
  int NAME(int kl, dim3 grid, hipStream_t st, const int8_t* X, const uint4* tm, const uint32_t* sts,           \
           const int8_t* Qc, const float* qe2, int nq, int ntiles, uint32_t* tau, float* cs, int* cr,          \
           uint32_t* dr, int64_t n_lists, const uint32_t* mask, uint32_t* xb, uint32_t* xw) {               \
    constexpr int R = w2_ring<DV>(), M = w2_mode<DV>();                                                     \
    if (kl == 4 && !mask)                                                                                   \
      hipLaunchKernelGGL((scan_screen_kernel<4, DV, false, R, M, 2>), grid, dim3(128), 0, st, X, tm, sts, Qc,  \
                         qe2, nq, ntiles, tau, cs, cr, dr, n_lists, mask, xb, xw);                           \
    else if (kl == 10 && !mask)                                                                             \
      hipLaunchKernelGGL((scan_screen_kernel<10, DV, false, R, M, 2>), grid, dim3(128), 0, st, X, tm, sts, Qc, \
                         qe2, nq, ntiles, tau, cs, cr, dr, n_lists, mask, xb, xw);                           \
    else if (kl == 4)                                                                                       \
      hipLaunchKernelGGL((scan_screen_kernel<4, DV, true, R, M, 2>), grid, dim3(128), 0, st, X, tm, sts, Qc,   \
                         qe2, nq, ntiles, tau, cs, cr, dr, n_lists, mask, xb, xw);                           \
    else if (kl == 10)                                                                                      \
      hipLaunchKernelGGL((scan_screen_kernel<10, DV, true, R, M, 2>), grid, dim3(128), 0, st, X, tm, sts, Qc,  \
                         qe2, nq, ntiles, tau, cs, cr, dr, n_lists, mask, xb, xw);                           \
    else                                                                                                    \
      return -1;                                                                                            \
    return 0;                                                                                               \
  }

// one translation unit per D instantiates the kernel for KL in {4, 10}, with and without a filter mask
#define RFX_K10_INSTANTIATE(DV, NAME)                                                                         \
  int NAME(int kl, dim3 grid, hipStream_t st, const int8_t* X, const uint4* tm, const uint32_t* sts,           \
           const int8_t* Qc, const float* qe2, int nq, int ntiles, uint32_t* tau, float* cs, int* cr,          \
           uint32_t* dr, int64_t n_lists, const uint32_t* mask, uint32_t* xb, uint32_t* xw) {               \
    if (kl == 4 && !mask)                                                                                   \
      hipLaunchKernelGGL((scan_screen_kernel<4, DV, false, kProdRing, kProdMode>), grid, dim3(512), 0, st, X, tm, sts, Qc, qe2, nq,   \
                         ntiles, tau, cs, cr, dr, n_lists, mask, xb, xw);                                    \
    else if (kl == 10 && !mask)                                                                             \
      hipLaunchKernelGGL((scan_screen_kernel<10, DV, false, kProdRing, kProdMode>), grid, dim3(512), 0, st, X, tm, sts, Qc, qe2, nq,  \
                         ntiles, tau, cs, cr, dr, n_lists, mask, xb, xw);                                    \
    else if (kl == 4)                                                                                       \
      hipLaunchKernelGGL((scan_screen_kernel<4, DV, true, kProdRing, kProdMode>), grid, dim3(512), 0, st, X, tm, sts, Qc, qe2, nq,    \
                         ntiles, tau, cs, cr, dr, n_lists, mask, xb, xw);                                    \
    else if (kl == 10)                                                                                      \
      hipLaunchKernelGGL((scan_screen_kernel<10, DV, true, kProdRing, kProdMode>), grid, dim3(512), 0, st, X, tm, sts, Qc, qe2, nq,   \
                         ntiles, tau, cs, cr, dr, n_lists, mask, xb, xw);                                    \
    else                                                                                                    \
      return -1;                                                                                            \
    return 0;                                                                                               \
  }

}  // namespace k10
}  // namespace rfx
