// k_scan_screen64.h — kernel 10, 64 queries per wave (round 6): the int8 screen of the
// exact two-pass scan for batches of 256 questions (BASELINE config 3: 10M x 768 bf16, nq 256, k 10) with
// half of the LDS traffic of the 32-queries-per-wave kernel (k_scan_screen.h).
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551).  The bound,
// the lists, the drops and the select are kernel 10's (k_scan_screen.h header comment: why the result is exact).
//
// What changes.  The 8-wave kernel holds 32 queries per wave (B fragments of all of d: 96 VGPRs at d 768), so
// every 32-row tile staged in LDS is read by all 8 waves: 24 KB of A fragments per wave per tile, 61 GB of LDS
// reads per launch at 10M rows (7.9x the HBM bytes; SQ counters, profiles/r05/pmc_sq/).  Here a workgroup is
// 4 waves x 64 queries (one wave per SIMD, up to 512 registers: the B fragments take 192 at d 768), so each A
// fragment read from LDS feeds 4 MFMAs instead of 2: 96 KB of LDS reads per tile instead of 192 KB, and half
// the ds_read_b128 issue per MFMA.  The price: no SIMD partner wave to fill the MFMA pipe while a wave is in
// its slow path or issues its LDS-DMA pieces (2 per stage).
//
// Layout.  Workgroup = 4 waves x 64 resident queries (256), 32-row tiles (2 row blocks of 16), per k-step 2 A
// fragments and 8 v_mfma_i32_16x16x64_i8 (2 row blocks x 4 query blocks) into eight i32 accumulators (two sets,
// alternating between tiles so a tile's epilogue overlaps the next tile's MFMAs).  Stage = 32 rows x 256 codes
// (8 KB, 8 LDS-DMA pieces of 1 KB, two per wave) into a RING-slot ring, one counted wait + barrier per tile
// (kernel 10's production schedule), the tile's 16-B record DMA'd with its first stage.  Epilogue: the fast
// path compares, per lane, the max D of each of its 4 query columns times the tile scale with the 4 queries'
// bounds; the slow path transposes the 4 x 4 (row group, query block) blocks of the accumulators across the
// wave's 16-lane groups (v_permlane32_swap + v_permlane16_swap) so that lane l owns query 64 w + l with all 32
// rows of the tile, and folds them into ONE list per lane (one list per query per workgroup: n_lists = blocks).
// Algorithmic bytes per tile: 32 * D (codes) + 16 (the tile record), as kernel 10.
#pragma once
#include "k_scan_screen.h"

namespace rfx {
namespace k10q {

using namespace mfc;
using k10::kTauW;
using k10::kTM;
using k10::kSK;
using k10::kRowB;
using k10::kSlot;
using k10::kMR;
using k10::kXbWords;

constexpr int kWaves = 4;
constexpr int kQW = 64;                  // queries per wave
constexpr int kQG = kWaves * kQW;        // 256 queries per workgroup
constexpr int kGPW = 8 / kWaves;         // LDS-DMA pieces per wave per stage
constexpr int kTauBytes = kQG * kTauW * 4;  // 16 KB
constexpr int kTauGPW = kTauBytes / 1024 / kWaves;  // 4
template <int RING>
constexpr int meta_off() { return RING * kSlot; }
template <int RING>
constexpr int tau_off() { return meta_off<RING>() + kMR * 1024; }
template <int RING>
constexpr int lds_bytes() { return tau_off<RING>() + kTauBytes; }
static_assert(lds_bytes<12>() <= 163840, "LDS budget");

// The pass mask of a lane's 32 values (value v = row v of the tile, a[v >> 2][v & 3] after the transpose)
// against the lane's bound: the integer threshold of k10::fold_mask_int (a superset of the float test), 32 bits.
__device__ __forceinline__ uint32_t fold_mask32(const v4i32 (&a)[8], float st, uint32_t bits, uint32_t thr_o, float e2,
                                                bool& pub) {
  int mx = k10::max3i(a[0][0], a[0][1], a[0][2]);
#pragma unroll
  for (int v = 3; v + 1 < 32; v += 2) mx = k10::max3i(mx, a[v >> 2][v & 3], a[(v + 1) >> 2][(v + 1) & 3]);
  mx = max(mx, a[7][3]);
  const float tf = thr_o ? unord(thr_o) - e2 : -__builtin_inff();
  constexpr int kBig = 1 << 30;
  int t;
  if (!(tf > -__builtin_inff())) {
    t = -kBig;
  } else if (!(st > 0.f)) {
    t = 0.f >= tf ? -kBig : kBig;
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
    for (int v = 31; v >= 0; --v) pm = __builtin_amdgcn_alignbit(pm, (uint32_t)(tm1 - a[v >> 2][v & 3]), 31);
    pm &= bits;
  }
  return pm;
}
// One passing value (the lowest bit of pm, cleared) into the lane's list: kernel 10's chain-free insert, the
// value taken by a 5-level bit-field-insert tree (the masks behind an empty asm keep it in registers).
template <int KL>
__device__ __forceinline__ void fold_trip32(const v4i32 (&a)[8], float st, int rbase, uint32_t& pm, uint64_t (&L)[KL],
                                            uint32_t& drop_o) {
  const int r = __builtin_ctz(pm);
  pm &= pm - 1;
  int m4 = -((r >> 4) & 1), m3 = -((r >> 3) & 1), m2 = -((r >> 2) & 1), m1 = -((r >> 1) & 1), m0 = -(r & 1);
  asm volatile("" : "+v"(m4), "+v"(m3), "+v"(m2), "+v"(m1), "+v"(m0));
  int v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = (a[(j + 16) >> 2][j & 3] & m4) | (a[j >> 2][j & 3] & ~m4);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (v[j + 8] & m3) | (v[j] & ~m3);
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = (v[j + 4] & m2) | (v[j] & ~m2);
#pragma unroll
  for (int j = 0; j < 2; ++j) v[j] = (v[j + 2] & m1) | (v[j] & ~m1);
  const int av = (v[1] & m0) | (v[0] & ~m0);
  const float s = (float)av * st;
  const uint64_t key = ((uint64_t)ord(s) << 32) | (uint32_t)(~(uint32_t)(rbase + r));
  bool c[KL];
#pragma unroll
  for (int i = 0; i < KL; ++i) c[i] = L[i] > key;
  const uint64_t k = c[KL - 1] ? key : L[KL - 1];
#pragma unroll
  for (int i = KL - 1; i > 0; --i) L[i] = c[i - 1] ? (c[i] ? L[i] : key) : L[i - 1];
  L[0] = c[0] ? L[0] : key;
  drop_o = max(drop_o, (uint32_t)(k >> 32));
}

// X, tmeta, stats, Qc, qe2, tau, xb, xw: as kernel 10.  Outputs per (query, list = workgroup): KL candidates
// (A, row) best first (empty tail -inf / kEmptyRow) and the list's drop.  MODE (debug library only, timing;
// wrong results): 1 = the slow path compiled in, never taken; 8 = no corpus stream after the prologue.
template <int KL, int D, bool MASK, int RING, int MODE = 0>
__global__ __launch_bounds__(256, 1) void scan_screen_q64_kernel(const int8_t* __restrict__ X, const uint4* __restrict__ tmeta,
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
  static_assert(RING >= 2 * NST + 2, "at least two stages beyond the next tile in flight");
  __shared__ __attribute__((aligned(1024))) uint8_t lds[lds_bytes<RING>()];
  constexpr int kTauOff = tau_off<RING>();
  constexpr int kMetaOff = meta_off<RING>();

  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int range = blockIdx.x;
  const int qg = blockIdx.y * kQG;
  const int q = qg + w * kQW + lane;  // the lane's query after the transpose (lists, bounds, outputs)
  const int nblk = gridDim.x;
  // the XCD-balanced tile split of kernel 10 (k_scan_screen.h)
  const bool bal = xb != nullptr && xw != nullptr && (nblk & 7) == 0 && ntiles >= 64 * nblk;
  const int xc = range & 7;
  int tb0 = range, tstride = nblk, nt = range < ntiles ? (ntiles - range + nblk - 1) / nblk : 0;
  if (bal) {
    uint64_t pre = 0, tot = 0;
    uint32_t wx = 1;
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      const uint32_t wv = xb[x];
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
  const int lst = range;
  const float e2 = qe2[q];
  {
    uint4* tz = (uint4*)(lds + kTauOff);
#pragma unroll
    for (int i = 0; i < kTauBytes / 16 / 256; ++i) tz[tid + 256 * i] = uint4{0u, 0u, 0u, 0u};
  }
  uint64_t L[KL];
#pragma unroll
  for (int i = 0; i < KL; ++i) L[i] = 0ull;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // resident query codes: query block qb, lane holds column 16 qb + (lane & 15), k = 64 ks + 16 (lane >> 4) + j
  uint4 bq[4 * NKS];
#pragma unroll
  for (int qb = 0; qb < 4; ++qb) {
    const int8_t* qa = Qc + (int64_t)(qg + w * kQW + 16 * qb + (lane & 15)) * D + 16 * (lane >> 4);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) bq[4 * ks + qb] = *(const uint4*)(qa + 64 * ks);
  }

  // LDS-DMA pieces of wave w: pieces w and w + 4 of each stage (slot bytes [1024 p, +1024) = rows 4p .. 4p + 3)
  uint32_t laneoff[kGPW];
#pragma unroll
  for (int u = 0; u < kGPW; ++u) {
    const int pr = 4 * (w + kWaves * u) + (lane >> 4);
    laneoff[u] = (uint32_t)(pr * D + (((lane & 15) ^ (pr & 15)) * 16));
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  const v4i32 meta_rsrc = make_rsrc(tmeta);
  auto issue_piece = [&](int gi, int slot) {
    const bool first = gi % NST == 0;
    gi = gi < S ? gi : S - 1;  // tail: harmless duplicate loads keep the counted waits exact
    const int ti = gi / NST;
    const int si = gi - ti * NST;
    const v4i32 rs = make_rsrc(X + (int64_t)tile_of(ti) * kTM * D + si * kSK);
#pragma unroll
    for (int u = 0; u < kGPW; ++u) {
      const uint32_t dst =
          __builtin_amdgcn_readfirstlane(lds_base + (uint32_t)(slot * kSlot) + (uint32_t)((w + kWaves * u) * 1024));
      bdma_nt(rs, laneoff[u], dst);
    }
    if (first) {
      const uint32_t mdst = __builtin_amdgcn_readfirstlane(lds_base + kMetaOff + (uint32_t)((ti % kMR) * 1024));
      bdma(meta_rsrc, (uint32_t)tile_of(ti) * 16u, mdst);
    }
  };
  const v4i32 tau_rsrc = make_rsrc(tau);
  auto issue_tau = [&]() {
#pragma unroll
    for (int u = 0; u < kTauGPW; ++u) {
      const int i = w + kWaves * u;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + kTauOff + i * 1024);
      bdma_sc1(tau_rsrc, (uint32_t)(qg * kTauW * 4 + tid * 16 + u * kWaves * 1024), dst);
    }
  };

  uint32_t thr = 0u, drop = 0u, pubd = 0u;
  const bool qlive = q < nq;
  // the bound (thr - e2) of the lane's own query, and of the 4 queries of its accumulator columns (query
  // 16 qb + (lane & 15) of the wave: owned by lane 16 qb + (lane & 15)); +inf for padded queries
  float tf_own = qlive ? -__builtin_inff() : __builtin_inff();
  float tfq[4];
#pragma unroll
  for (int qb = 0; qb < 4; ++qb) tfq[qb] = qg + w * kQW + 16 * qb + (lane & 15) < nq ? -__builtin_inff() : __builtin_inff();
  auto set_bounds = [&]() {
    tf_own = !qlive ? __builtin_inff() : thr ? unord(thr) - e2 : -__builtin_inff();
#pragma unroll
    for (int qb = 0; qb < 4; ++qb) tfq[qb] = __shfl(tf_own, 16 * qb + (lane & 15));
  };
  if (xb != nullptr) {  // the quantiser's seed bound (kernel 10)
    thr = xb[kXbWords + q];
    set_bounds();
  }
  const uint32_t slot_voff = (uint32_t)(q * kTauW + lst % kTauW) * 4u;
  const uint8_t* const tq = lds + kTauOff + (w * kQW + lane) * (kTauW * 4);
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

  // schedule (kernel 10's per-tile barrier): stage h's pieces go out at k-step 0 of stage h - AHEAD into the
  // slot of stage h - RING (freed by the barrier of the tile before); the tile-t barrier waits for every stage
  // of tile t + 1; the slot table refreshed after tile t's barrier is read at tile t + TBD, the first tile
  // whose barrier wait covers that refresh without waiting for younger pieces (3 at d 768, 2 at d 1024)
  constexpr int PF = (D == 768) ? 2 : 1;
  constexpr int NF = PF + 1;
  constexpr int KB = KPS - PF;
  constexpr int AHEAD = RING - NST;
  constexpr int TBD = (RING - 1) / NST > 2 ? (RING - 1) / NST : 2;
  static_assert((RING - NST - 1) / NST + 2 <= 64, "wait counts");
  static_assert((NST * KPS) % NF == 0, "fragment rotation must realign every tile");

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // resident queries landed before the counted stream
  launder(bq);
  issue_tau();
#pragma unroll
  for (int p = 0; p < AHEAD; ++p) issue_piece(p, p);
  {
    constexpr int NMT = (AHEAD - 1) / NST;  // records of stages NST, 2 NST, ... <= AHEAD - 1
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"((AHEAD - NST) * kGPW + NMT) : "memory");
  }
  asm volatile("s_barrier" ::: "memory");

  Frag fr[NF];
#pragma unroll
  for (int p = 0; p < PF; ++p) fr[p] = read_frag(0, p);
  v4i32 accA[8], accB[8];  // [rb * 4 + qb]
  auto epilogue = [&](const int it, v4i32(&acc)[8]) {
    const int tile = tile_of(it);
    int m[4];
#pragma unroll
    for (int qb = 0; qb < 4; ++qb) {
      int x = k10::max3i(acc[qb][0], acc[qb][1], acc[qb][2]);
      x = k10::max3i(x, acc[qb][3], acc[4 + qb][0]);
      x = k10::max3i(x, acc[4 + qb][1], acc[4 + qb][2]);
      m[qb] = max(x, acc[4 + qb][3]);
    }
    const float st_t = *(const float*)(lds + kMetaOff + (it % kMR) * 1024 + lane * 16);
    bool hit = false;
#pragma unroll
    for (int qb = 0; qb < 4; ++qb) hit = hit || (float)m[qb] * st_t >= tfq[qb];
    if constexpr ((MODE & 1) != 0) hit = hit && nq < 0;
    if (__builtin_amdgcn_ballot_w64(hit)) {
      const uint2 md = *(const uint2*)(lds + kMetaOff + (it % kMR) * 1024 + lane * 16);
      const float st = __uint_as_float(md.x);
      uint32_t lw = qlive ? md.y : 0u;
      if constexpr (MASK) lw &= mask[tile];
      // 4 x 4 transpose of (16-lane row group g, query block qb) per (rb, i): afterwards register
      // acc[rb * 4 + r][i] of lane (g, n) holds D(row 16 rb + 4 r + i, query 16 g + n)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {  // bit 1 of the group <-> bit 1 of the register
            const auto r = __builtin_amdgcn_permlane32_swap((uint32_t)acc[rb * 4 + h][i], (uint32_t)acc[rb * 4 + h + 2][i],
                                                            false, false);
            acc[rb * 4 + h][i] = (int)r[0];
            acc[rb * 4 + h + 2][i] = (int)r[1];
          }
#pragma unroll
          for (int h = 0; h < 4; h += 2) {  // bit 0 of the group <-> bit 0 of the register
            const auto r = __builtin_amdgcn_permlane16_swap((uint32_t)acc[rb * 4 + h][i], (uint32_t)acc[rb * 4 + h + 1][i],
                                                            false, false);
            acc[rb * 4 + h][i] = (int)r[0];
            acc[rb * 4 + h + 1][i] = (int)r[1];
          }
        }
      bool pub;
      uint32_t pm = fold_mask32(acc, st, lw, thr, e2, pub);
      while (pm) fold_trip32<KL>(acc, st, tile * kTM, pm, L, drop);
      k10::fold_end<KL, true>(L, thr, pub, tau_rsrc, slot_voff, pubd);
      set_bounds();
    }
  };
  auto tile_body = [&](const int it, v4i32(&acc)[8], v4i32(&accp)[8], const bool prev) {
    const int gbase = it * NST;
    if (it >= TBD && k10::tau_refresh_tile<0>(it - TBD)) {
      thr = max(thr, k10::tau_kth<KL>(tq));
      set_bounds();
    }
#pragma unroll
    for (int s = 0; s < NST; ++s) {
      const int g = gbase + s;
      const int slot = g % RING;
#pragma unroll
      for (int kk = 0; kk < KPS; ++kk) {
        if constexpr ((MODE & 8) == 0)
          if (kk == 0) {
            const int h = g + AHEAD;
            issue_piece(h, h % RING);
          }
        if (kk == KB && s == NST - 1 && (MODE & 8) != 0) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          asm volatile("s_barrier" ::: "memory");
        } else if (kk == KB && s == NST - 1) {
          // tile it + 1 landed: younger are the pieces of stages NST (it + 2) .. NST it + RING - 1, their records,
          // and the refreshes issued after the last needed piece (tiles it + 2 - TBD .. it - 1)
          constexpr int NMY = (RING - NST - 1) / NST;
          int nt_ = 0;
#pragma unroll
          for (int d = 1; d <= TBD - 2; ++d) nt_ += (it >= d && k10::tau_refresh_tile<0>(it - d)) ? kTauGPW : 0;
          if (nt_ == kTauGPW)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"((RING - 2 * NST) * kGPW + NMY + kTauGPW) : "memory");
          else  // (none, or more than one refresh: stricter, never looser)
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"((RING - 2 * NST) * kGPW + NMY) : "memory");
          asm volatile("s_barrier" ::: "memory");
          if (k10::tau_refresh_tile<0>(it)) issue_tau();
        }
        const int ks = s * KPS + kk;
        fr[(ks + PF) % NF] = kk + PF < KPS ? read_frag(slot, kk + PF) : read_frag((g + 1) % RING, kk + PF - KPS);
        const Frag& cur = fr[ks % NF];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int qb = 0; qb < 4; ++qb)
            acc[rb * 4 + qb] = ks == 0 ? k10::mfma_i8(cur.a[rb], bq[4 * ks + qb], v4i32{0, 0, 0, 0})
                                       : k10::mfma_i8(cur.a[rb], bq[4 * ks + qb], acc[rb * 4 + qb]);
        if (kk == 0 && s == 0 && prev) epilogue(it - 1, accp);
      }
    }
  };
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
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (q < nq) {
    // entries below (the query's bound as it stands now) - e2 cannot be survivors: dropped here
    uint32_t sl[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) sl[j] = __hip_atomic_load(tau + (int64_t)q * kTauW + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t fin = max(thr, k10::kth16<KL>(sl));
    const float lo = fin ? unord(fin) - e2 : -__builtin_inff();
    const int64_t o = ((int64_t)q * n_lists + lst) * KL;
#pragma unroll
    for (int i = 0; i < KL; ++i) {
      const uint64_t key = L[i];
      const float sc = unord((uint32_t)(key >> 32));
      const bool keep = (key >> 32) != 0 && sc >= lo;
      cand_s[o + i] = keep ? sc : -__builtin_inff();
      cand_r[o + i] = keep ? (int)(~(uint32_t)key) : kEmptyRow;
    }
    drops[(int64_t)q * n_lists + lst] = drop;
  }
  if (bal && blockIdx.y == 0 && tid == 0) {  // the XCD split's bookkeeping (kernel 10)
    const uint64_t dt = wall_clock64() - t_start;
    __hip_atomic_fetch_add(xw + 8 + xc, (uint32_t)(dt < 0xffffffull ? dt : 0xffffffull), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(xw + 16 + xc, (uint32_t)nt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

constexpr int kRing768 = 10, kRing1024 = 10;
#define RFX_K10Q_INSTANTIATE(DV, RINGV, NAME)                                                                 \
  int NAME(int kl, dim3 grid, hipStream_t st, const int8_t* X, const uint4* tm, const uint32_t* sts,           \
           const int8_t* Qc, const float* qe2, int nq, int ntiles, uint32_t* tau, float* cs, int* cr,          \
           uint32_t* dr, int64_t n_lists, const uint32_t* mask, uint32_t* xb, uint32_t* xw) {               \
    if (kl == 4 && !mask)                                                                                   \
      hipLaunchKernelGGL((scan_screen_q64_kernel<4, DV, false, RINGV>), grid, dim3(256), 0, st, X, tm, sts, Qc, \
                         qe2, nq, ntiles, tau, cs, cr, dr, n_lists, mask, xb, xw);                           \
    else if (kl == 10 && !mask)                                                                             \
      hipLaunchKernelGGL((scan_screen_q64_kernel<10, DV, false, RINGV>), grid, dim3(256), 0, st, X, tm, sts,  \
                         Qc, qe2, nq, ntiles, tau, cs, cr, dr, n_lists, mask, xb, xw);                       \
    else if (kl == 4)                                                                                       \
      hipLaunchKernelGGL((scan_screen_q64_kernel<4, DV, true, RINGV>), grid, dim3(256), 0, st, X, tm, sts, Qc, \
                         qe2, nq, ntiles, tau, cs, cr, dr, n_lists, mask, xb, xw);                           \
    else if (kl == 10)                                                                                      \
      hipLaunchKernelGGL((scan_screen_q64_kernel<10, DV, true, RINGV>), grid, dim3(256), 0, st, X, tm, sts,   \
                         Qc, qe2, nq, ntiles, tau, cs, cr, dr, n_lists, mask, xb, xw);                       \
    else                                                                                                    \
      return -1;                                                                                            \
    return 0;                                                                                               \
  }

}  // namespace k10q
}  // namespace rfx
