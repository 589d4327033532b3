// k_scan_mfma6.h — the headline scan (BASELINE config 3: 10M×768 bf16, nq 256, k 10): all-query-
// stationary, two waves per SIMD, v_mfma_f32_16x16x32, corpus stream by LDS-DMA into an LDS image
// whose fragment reads need no per-read address arithmetic.
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551).
// Fused scan + per-query top-k; the score matrix never reaches HBM.
//
// What changed against k_scan_mfma5.h (its ablations: tools/k5_variants.py, profiles/r02_*):
//   * MFMA shape 16x16x32 (2 row blocks × 2 query blocks per 32-deep k-step): same MFMA cycles and
//     LDS bytes per FLOP as 32x32x16, and the chip holds a higher clock on it (MI355X_MICROARCH.md
//     'DVFS give-back' item 7); measured -2.4 % on kernel 5.  The epilogue's query-pair swap is one
//     v_permlane16_swap per register pair.
//   * Non-temporal corpus DMA (the corpus is read once per batch).
//   * The production instantiations are MODE 0 and kModeMask (row filter); the other MODE bits
//     (below the template) are debug-build ablations (k6_dbg.hip, librfx_dbg.so) and compile
//     out of the product library's instantiations.
// Why not more: the launch runs at the board's power cap (rocm-smi: 1400 W package power, sclk
// 1.8-1.95 GHz, profiles/r02_power_*), so its time is the batch's energy over the cap; measured
// alternatives that traded cycles for energy (tools/k5_variants.py, steady-state 8-s bursts):
// an LDS image read with immediate offsets only (32-B skewed 1 KB pieces: no address VALU, no
// spills, 13 % faster without the stream) took 2 % MORE time with the stream running (more stall
// cycles at a higher clock), with 2-row or 8-row × 128 B pieces alike.
// Everything else as kernel 5: workgroup = 8 waves × 32 resident queries (192 VGPRs of B
// fragments); 32-row tiles, block b takes tiles b, b + B, ...; a stage = 32 rows × 256 dims
// (16 KB of rows) in a 4-slot ring, 3 stages in flight, one counted vmcnt + s_barrier per stage; per-lane
// sorted top-KL lists in LDS behind a pruning bound shared across workgroups through a per-query
// slot table (k_mfma_common.h fold / tau_min).
// Requires the index invariant of rfx_api.hip: rows [nrows, capacity) are NaN and capacity is a
// multiple of 128, so the ragged last tile needs no clamping or masking.
// Algorithmic bytes per tile: 32 * D * esize.
#pragma once
#include "k_mfma_common.h"

namespace rfx {
namespace k6 {

using namespace mfc;

constexpr int kWaves = 8;
constexpr int kTM = 32;                   // rows per tile
constexpr int kQW = 32;                   // queries per wave
constexpr int kQG = kWaves * kQW;         // 256 queries per workgroup
constexpr int kSK = 256;                  // dims per stage
constexpr int kRowB = kSK * 2;            // 512 B per row per stage
constexpr int kSlot = kTM * kRowB;        // 16 KB: 32 rows × 256 dims
// Ring depth, measured by side builds (-DRFX_K6_RING=N, tools/gpu_k6ring.sh, alternating in one
// call): config 3 6 slots 3.646 ms, 5 slots 3.614 ms, 4 slots 3.543-3.551 ms per launch.
#ifndef RFX_K6_RING
#define RFX_K6_RING 4
#endif
constexpr int kRing = RFX_K6_RING;        // 4 slots, 3 stages (48 KB) in flight
constexpr int kGPW = 2;                   // LDS-DMA pieces per wave per stage (16 KB / 1 KB / 8 waves)
constexpr int kTauW = 16;                 // u32 per query in the threshold table (KL <= 10 used)
constexpr int kTauBytes = kQG * kTauW * 4;  // 16 KB: 16 DMA pieces, 2 per wave
constexpr int kTauGPW = kTauBytes / 1024 / kWaves;
// LDS: RING slots | threshold image | lane lists [wave][KL][64] u64
template <int RING>
constexpr int tau_off() { return RING * kSlot; }
template <int RING>
constexpr int list_off() { return tau_off<RING>() + kTauBytes; }
template <int KL, int RING>
constexpr int lds_bytes() { return list_off<RING>() + kWaves * KL * 64 * 8; }
static_assert(lds_bytes<10, 6>() <= 163840 && lds_bytes<4, 7>() <= 163840, "LDS budget");
static_assert(kSlot / 1024 == kWaves * kGPW && kTauGPW == 2, "DMA pieces per wave");

// Threshold-table refreshes go out after the last stage of tiles 0, 1, 3, 7, 11, ... (the lists
// start empty, so the first tiles take the slow insert path until the slot table's bound arrives;
// then every 4 tiles: a staler bound sends more lanes into the insert path — kernel 5 ablations).
__device__ __forceinline__ bool tau_refresh_tile(int it) { return it < 2 || (it & 3) == 3; }

// Metadata filter: row bit of the lane's value r after the epilogue's pair swap (fold ROWMAP 1,
// bits pre-shifted by 8 * half): (r & 7) + 16 * (r >> 3).
template <class V>
__device__ __forceinline__ void mask_rowmap1(V& a, uint32_t bits) {
#pragma unroll
  for (int r = 0; r < 16; ++r)
    if (!((bits >> ((r & 7) + 16 * (r >> 3))) & 1u)) a[r >> 2][r & 3] = __builtin_nanf("");
}

// Debug-build ablations of the first tile's fold (MODE 64 / 256 below).  fold_nopub: the list insert
// of mfc::fold (ROWMAP 1) without publishing the list's best to the slot table.  fold_first: the
// lane's list is empty at tile 0, so each of the 16 values goes straight to its final position
// rank = #{better values} (score desc, row asc; rows grow with r in ROWMAP 1), no shifting.
template <int KL>
__device__ __forceinline__ void fold_nopub(const Acc4View& acc, uint64_t* Ls, uint32_t& thr_o, int rbase) {
  const float thr = thr_o ? unord(thr_o) : -__builtin_inff();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float s = acc[r];
    if (s >= thr) {
      const int row = rbase + (r & 7) + 16 * (r >> 3);
      const uint64_t key = ((uint64_t)ord(s) << 32) | (uint32_t)(~(uint32_t)row);
      if (key > Ls[(KL - 1) * 64]) {
        int i = KL - 1;
        for (; i > 0; --i) {
          const uint64_t prev = Ls[(i - 1) * 64];
          if (prev >= key) break;
          Ls[i * 64] = prev;
        }
        Ls[i * 64] = key;
      }
    }
  }
  const uint32_t own = (uint32_t)(Ls[(KL - 1) * 64] >> 32);
  thr_o = own > thr_o ? own : thr_o;
}
template <int KL, bool PUB>
__device__ __forceinline__ void fold_first(const Acc4View& acc, uint64_t* Ls, uint32_t& thr_o, int rbase, v4i32 tau_rsrc,
                                           uint32_t slot_voff) {
  uint32_t best = 0u, kth = 0u;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float si = acc[i];
    int rank = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j != i) rank += (acc[j] > si) || (j < i && acc[j] == si);
    if (si == si && rank < KL) {  // NaN never enters
      const int row = rbase + (i & 7) + 16 * (i >> 3);
      Ls[rank * 64] = ((uint64_t)ord(si) << 32) | (uint32_t)(~(uint32_t)row);
      if (rank == 0) best = ord(si);
      if (rank == KL - 1) kth = ord(si);
    }
  }
  thr_o = kth > thr_o ? kth : thr_o;
  if (PUB && best) batomic_umax(tau_rsrc, slot_voff, best);
}

// MODE: 0 production; kModeMask = row-masked variant (metadata filter); debug-build ablations:
// 1 = no top-k epilogue (MFMAs kept live), 8 = no corpus stream after the prologue, 16 = corpus
// DMA WITHOUT the non-temporal hint, 32 = every other k-step reuses the previous A fragments (half
// the LDS reads; wrong scores, timing/energy only), 64 = no slot-table publication at tile 0,
// 256 = tile 0 folded by rank (fold_first), 512 = MFMAs of a k-step in snake order.
constexpr int kModeMask = 2097152;

// The body of one workgroup: row range `range` of `nblk`, query group `qgb`, in the LDS image `lds`
// (lds_bytes<KL, RING>() bytes, 1024-aligned); scan_mfma6_kernel runs it as block (range, qgb) of its grid.
template <int DT, int KL, int D, int MODE = 0, int RING = kRing>
__device__ __forceinline__ void scan_mfma6_body(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Qp, int nq,
                                                int ntiles, uint32_t* __restrict__ tau, float* __restrict__ cand_s,
                                                int* __restrict__ cand_r, int64_t n_lists,
                                                const uint32_t* __restrict__ mask, int range, int qgb, int nblk,
                                                uint8_t* __restrict__ lds) {
  constexpr int NKS = D / 32;   // 32-deep k-steps per tile
  constexpr int NST = D / kSK;  // stages per tile
  constexpr int KPS = kSK / 32;  // k-steps per stage (8)
  static_assert(D % kSK == 0, "D must be a multiple of 256");
  static_assert(KL <= 10, "threshold table holds 10 slots");
  constexpr int kTauOff = tau_off<RING>();
  constexpr int kListOff = list_off<RING>();

  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int half = lane >> 5;
  const int qg = qgb * kQG;
  // this lane's query after the epilogue's pair swap: lanes of odd 16-lane row hold query block 1
  const int q = qg + w * kQW + 16 * ((lane >> 4) & 1) + (lane & 15);
  const int nt = range < ntiles ? (ntiles - range + nblk - 1) / nblk : 0;
  const int S = nt * NST;
  if (S == 0) return;  // (cannot happen with the host plan; whole workgroup exits together)
  const int lst = range * 2 + half;  // this lane's list id (per query)

  // ---- LDS init: threshold image and lane lists start at 0 (= "no bound" / empty) ----
  {
    uint4* tz = (uint4*)(lds + kTauOff);
#pragma unroll
    for (int i = 0; i < kTauBytes / 16 / 512; ++i) tz[tid + 512 * i] = uint4{0u, 0u, 0u, 0u};
  }
  uint64_t* const Ls = (uint64_t*)(lds + kListOff) + (w * KL) * 64 + lane;
#pragma unroll
  for (int i = 0; i < KL; ++i) Ls[i * 64] = 0ull;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();  // no LDS-DMA in flight yet: a plain barrier

  // ---- resident query fragments (B[k][col] of 16x16x32): query block qb, lane holds col
  // 16 qb + (lane & 15), k = 32 ks + 8 (lane >> 4) + j
  uint4 bq[2 * NKS];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const uint16_t* qa = Qp + (int64_t)(qg + w * kQW + 16 * qb + (lane & 15)) * D + 8 * (lane >> 4);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) bq[2 * ks + qb] = *(const uint4*)(qa + 32 * ks);
  }

  // ---- LDS-DMA pieces: piece i = w + 8 u (u = 0, 1) of a stage fills slot bytes [1024 i, +1024) =
  // rows 2i, 2i+1 (512 B each); lane -> (row 2i + half, position lane & 31) <- source chunk
  // position ^ (row & 15): the 16 rows a 16-lane group of a fragment read touches sit in 16
  // distinct bank quads (the permutation rides on the DMA source address)
  uint32_t laneoff[kGPW];  // byte offset of this lane's 16 B inside a [32 rows][D] tile (stage 0)
#pragma unroll
  for (int u = 0; u < kGPW; ++u) {
    const int r = 2 * (w + kWaves * u) + half;
    laneoff[u] = (uint32_t)(r * D + (((lane & 31) ^ (r & 15)) * 8)) * 2u;
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  const int64_t tile_stride = (int64_t)nblk * kTM * D;  // elements between a block's tiles
  // piece u of stage gi -> LDS slot `slot`.  gi is clamped to the last stage so the tail of the
  // stream issues harmless duplicate loads into free slots: every stage issues exactly kGPW
  // LDS-DMA ops per wave and the counted waits stay exact.
  auto issue_piece = [&](int gi, int slot, int u) {
    gi = gi < S ? gi : S - 1;
    const int ti = gi / NST;
    const int si = gi - ti * NST;
    const uint16_t* tbase = X + (int64_t)range * kTM * D + ti * tile_stride + si * kSK;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + (uint32_t)(slot * kSlot) + (uint32_t)((w + kWaves * u) * 1024));
    // the corpus is read once per batch: non-temporal (measured at the power cap, 8-s bursts:
    // -1.2 % against the default policy; the chip's time per batch is set by energy there)
    if constexpr ((MODE & 16) != 0)
      bdma(make_rsrc(tbase), laneoff[u], dst);
    else
      bdma_nt(make_rsrc(tbase), laneoff[u], dst);
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

  uint32_t thr = 0u;  // pruning bound (orderable score; 0 = none)
  const uint32_t slot_voff = (uint32_t)(q * kTauW + lst % KL) * 4u;
  const uint8_t* const tq = lds + kTauOff + (w * kQW + (lane & 15) + 16 * ((lane >> 4) & 1)) * (kTauW * 4);
  int n_slow = 0;  // (fold's diagnostic counter; unused here)
  // A fragment of row block rb, k-step kk of a slot (16x16x32): row 16 rb + (lane & 15), chunk
  // 4 kk + (lane >> 4), stored at position chunk ^ (row & 15); the two row blocks are 8 KB apart
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

  // Schedule.  Stage h's pieces go out during stage h - (RING - 1), at k-steps 0 and 4, into the
  // slot freed at stage h - RING's barrier (production RING 4: during stage h - 3, slot of h - 4).  Fragments are read one k-step ahead of their MFMAs; the stage-end
  // wait + barrier sit at k-step KPS - 1, once every wave has issued (and, by lgkmcnt(0), received)
  // its last read of the stage.
  constexpr int PF = 1;
  constexpr int NF = PF + 1;
  constexpr int KB = KPS - PF;
  constexpr int AHEAD = RING - 1;
  constexpr int YNG = (RING - 2) * kGPW;  // ops younger than the next stage (4 with the 4-slot ring)
  static_assert((NST * KPS) % NF == 0, "fragment rotation must realign every tile");

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // resident queries landed before the counted stream
  // NOT laundered (k_mfma_common.h): hipcc's own vmcnt waits on the fragments' loads stay in the loop
  // and drain the DMA ring at the end of each tile's first stage — measured FASTER at the power cap
  // (round 3, one box, interleaved bursts: 3.57 ms against 3.93 ms laundered, debug MODE 1024)
  if constexpr ((MODE & 1024) != 0) launder(bq);
  issue_tau();
#pragma unroll
  for (int p = 0; p < AHEAD; ++p)
#pragma unroll
    for (int u = 0; u < kGPW; ++u) issue_piece(p, p, u);
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(YNG) : "memory");  // stage 0 landed: stages 1..4 younger
  asm volatile("s_barrier" ::: "memory");

  Frag fr[NF];
  fr[0] = read_frag(0, 0);
  v4f32x4 acc4[4];  // [rb * 2 + qb]
  for (int it = 0; it < nt; ++it) {
    const int tile = range + it * nblk;
    const int gbase = it * NST;
    if constexpr ((MODE & 1) == 0)  // refreshed threshold image (issued 2 tiles ago; any value is a valid bound)
      if (it >= 2 && tau_refresh_tile(it - 2)) thr = max(thr, tau_min<KL>(tq));
    // A threshold refresh (kTauGPW ops) issued after the barrier of stage g_r = last stage of a
    // refresh tile it_r is younger than stage g+1's pieces iff g-RING+2 <= g_r <= g-1, i.e. iff
    // it - young_depth(s) <= it_r <= it - 1 (6 slots: it-2.. at stage 0, it-1 at stages 1, 2).
    // Two young refreshes count as one: the wait is then stricter, never looser.
    auto young = [&](int s) {
      const int dmax = (RING - 3 + NST - s) / NST;
      bool y = false;
#pragma unroll
      for (int d = 1; d <= dmax; ++d) y = y || (it >= d && tau_refresh_tile(it - d));
      return y;
    };
#pragma unroll
    for (int s = 0; s < NST; ++s) {
      const int g = gbase + s;
      const int slot = g % RING;
#pragma unroll
      for (int kk = 0; kk < KPS; ++kk) {
        if constexpr ((MODE & 8) == 0)
          if (kk % (KPS / kGPW) == 0) issue_piece(g + RING - 1, (g + RING - 1) % RING, kk / (KPS / kGPW));
        if (kk == KB) {
          // stage g+1 landed for this wave: ops younger than its pieces = stages g+2..g+RING-1
          // (YNG) [+ a threshold refresh (2)]; lgkmcnt(0) + barrier: every wave has received its last
          // fragment of slot g, which may be refilled from here on.
          if constexpr ((MODE & 8) == 0) {
            if (young(s))
              asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(YNG + kTauGPW) : "memory");
            else
              asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(YNG) : "memory");
          } else {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
          asm volatile("s_barrier" ::: "memory");
          if constexpr ((MODE & 8) == 0)
            if (s == NST - 1 && tau_refresh_tile(it)) issue_tau();
        }
        const int ks = s * KPS + kk;
        // prefetch k-step kk + 1 (crossing into stage g+1 after the barrier)
        if constexpr ((MODE & 32) != 0) {
          if ((ks & 1) == 0)
            fr[(ks + PF) % NF] = fr[ks % NF];
          else
            fr[(ks + PF) % NF] = kk + PF < KPS ? read_frag(slot, kk + PF) : read_frag((g + 1) % RING, kk + PF - KPS);
        } else {
          fr[(ks + PF) % NF] = kk + PF < KPS ? read_frag(slot, kk + PF) : read_frag((g + 1) % RING, kk + PF - KPS);
        }
        const Frag& cur = fr[ks % NF];
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // the prefetch reads go out first
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int qq = 0; qq < 2; ++qq) {
            // MODE 512 (debug): snake order, consecutive MFMAs share an operand (A, B, A)
            const int qb = (MODE & 512) != 0 ? (rb ? 1 - qq : qq) : qq;
            acc4[2 * rb + qb] = ks == 0 ? mfma16<DT>(cur.a[rb], bq[2 * ks + qb], v4f32x4{})
                                        : mfma16<DT>(cur.a[rb], bq[2 * ks + qb], acc4[2 * rb + qb]);
          }
      }
    }

    // ---- epilogue: pair swap (lane of even 16-lane row g keeps query n, odd keeps 16 + n; one
    // v_permlane16_swap per register pair), then fold the lane's 16 rows into its list
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc4[2 * rb][i]),
                                                        __float_as_uint(acc4[2 * rb + 1][i]), false, false);
        acc4[2 * rb][i] = __uint_as_float(r[0]);
        acc4[2 * rb + 1][i] = __uint_as_float(r[1]);
      }
    if constexpr ((MODE & 1) == 0) {
      if constexpr ((MODE & kModeMask) != 0) mask_rowmap1(acc4, mask[tile] >> (8 * half));
      if constexpr ((MODE & (64 | 256)) != 0) {
        if (it == 0) {
          if constexpr ((MODE & 256) != 0)
            fold_first<KL, (MODE & 64) == 0>(Acc4View{acc4}, Ls, thr, tile * kTM + 8 * half, tau_rsrc, slot_voff);
          else
            fold_nopub<KL>(Acc4View{acc4}, Ls, thr, tile * kTM + 8 * half);
        } else {
          fold<KL, 1>(Acc4View{acc4}, Ls, thr, tile * kTM + 8 * half, tau_rsrc, slot_voff, n_slow);
        }
      } else {
        fold<KL, 1>(Acc4View{acc4}, Ls, thr, tile * kTM + 8 * half, tau_rsrc, slot_voff, n_slow);
      }
    } else {
      if (acc4[0][0] == 12345.f && acc4[1][1] == 54321.f && acc4[2][2] == 1.f && acc4[3][3] == 2.f) Ls[0] = 1;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (q < nq) {
    // Drop entries below the query's bound as it stands now, read fresh from the slot table (all
    // workgroups end together, so it is close to final): valid bound => exact, and the merge then
    // sees ~k live candidates per query instead of 512 lists.
    uint32_t m = 0xffffffffu;
#pragma unroll
    for (int j = 0; j < KL; ++j)
      m = min(m, __hip_atomic_load(tau + (int64_t)q * kTauW + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const uint32_t fin = max(thr, m);
    const int64_t o = ((int64_t)q * n_lists + lst) * KL;
#pragma unroll
    for (int i = 0; i < KL; ++i) {
      const uint64_t key = Ls[i * 64];
      const bool keep = key && (uint32_t)(key >> 32) >= fin;
      cand_s[o + i] = keep ? unord((uint32_t)(key >> 32)) : -__builtin_inff();
      cand_r[o + i] = keep ? (int)(~(uint32_t)key) : kEmptyRow;
    }
  }
}

template <int DT, int KL, int D, int MODE = 0, int RING = kRing>
__global__ __launch_bounds__(512, 1) void scan_mfma6_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Qp,
                                                            int nq, int ntiles, uint32_t* __restrict__ tau,
                                                            float* __restrict__ cand_s, int* __restrict__ cand_r,
                                                            int64_t n_lists, const uint32_t* __restrict__ mask,
                                                            const uint32_t* __restrict__ gate) {
  // gate (the two-pass scan's fallback, k_screen.hip): run only when the screen asked for it
  if (gate && *gate == 0u) return;
  __shared__ __attribute__((aligned(1024))) uint8_t lds[lds_bytes<KL, RING>()];
  scan_mfma6_body<DT, KL, D, MODE, RING>(X, Qp, nq, ntiles, tau, cand_s, cand_r, n_lists, mask, (int)blockIdx.x,
                                         (int)blockIdx.y, (int)gridDim.x, lds);
}

// one translation unit per (dtype, D) instantiates the kernel for the lane-list sizes KL in {4, 10}
#define RFX_K6_INSTANTIATE(DTV, DV, NAME)                                                                  \
  int NAME(int kl, dim3 grid, hipStream_t st, const uint16_t* X, const uint16_t* Qp, int nq, int ntiles,     \
           uint32_t* tau, float* cs, int* cr, int64_t n_lists, const uint32_t* mask, const uint32_t* gate) {  \
    if (kl == 4 && !mask)                                                                                \
      hipLaunchKernelGGL((scan_mfma6_kernel<DTV, 4, DV>), grid, dim3(512), 0, st, X, Qp, nq, ntiles, tau, cs, \
                         cr, n_lists, mask, gate);                                                              \
    else if (kl == 10 && !mask)                                                                          \
      hipLaunchKernelGGL((scan_mfma6_kernel<DTV, 10, DV>), grid, dim3(512), 0, st, X, Qp, nq, ntiles, tau,  \
                         cs, cr, n_lists, mask, gate);                                                          \
    else if (kl == 4)                                                                                    \
      hipLaunchKernelGGL((scan_mfma6_kernel<DTV, 4, DV, kModeMask>), grid, dim3(512), 0, st, X, Qp, nq,     \
                         ntiles, tau, cs, cr, n_lists, mask, gate);                                             \
    else if (kl == 10)                                                                                   \
      hipLaunchKernelGGL((scan_mfma6_kernel<DTV, 10, DV, kModeMask>), grid, dim3(512), 0, st, X, Qp, nq,    \
                         ntiles, tau, cs, cr, n_lists, mask, gate);                                             \
    else                                                                                                 \
      return -1;                                                                                         \
    return 0;                                                                                            \
  }

}  // namespace k6
}  // namespace rfx
