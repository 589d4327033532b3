// k_scan_mfma5.h — all-query-stationary batched scan, two waves per SIMD.
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551),
// BASELINE.json config 3 (10M×768 bf16, nq=256, k=10).  Fused scan + per-query top-k; the score
// matrix never reaches HBM.
//
// Why (measured on MI355X with k_scan_mfma4.h's ablations, profiles/r01_*): with ONE wave per SIMD
// (64 resident queries, 512 registers) the corpus stream (2.4 ms alone) and the MFMA work (2.6 ms
// alone) did not overlap: 4.0 ms together.  Every LDS-DMA issue (~100-150 cycles under load), every
// stage barrier and every top-k epilogue stalled the only MFMA issuer of its SIMD.  Here a
// workgroup is 8 waves, two per SIMD, each with 32 resident queries (192 VGPRs of B-fragments, no
// AGPR copies): while one wave issues DMA, waits at a barrier or folds its tile into its top-k
// list, its SIMD partner keeps the matrix core busy.  The price is one ds_read_b128 per MFMA
// instead of one per two (LDS at ~half its read bandwidth).
//   * workgroup = 8 waves × 32 queries = 256 queries; every corpus byte crosses the fabric once.
//   * tile = 32 corpus rows; a stage = 32 rows × 256 dims (16 KB) arrives by LDS-DMA
//     (global_load_lds_dwordx4, 2 wave-instructions per wave, spread over the stage's k-steps)
//     into a 6-slot ring, 5 stages (80 KB) in flight; one counted `s_waitcnt vmcnt` + `s_barrier`
//     per stage.
//   * LDS row image: 512 B per row; 16-B chunk c of row r at position c ^ (r & 15): conflict-free
//     32-row ds_read_b128 fragment reads (the permutation rides on the DMA source address).
//   * per k-step and wave: 1 ds_read_b128 (32 rows × 16 k) → 1 v_mfma_f32_32x32x16.
//   * top-k and the cross-workgroup pruning bound: as k_scan_mfma4.h (lane lists in LDS, per-query
//     10-slot best-of-list table refreshed by DMA, see tau_refresh_tile) — one list per lane.
// Requires the index invariant of rfx_api.hip: rows [nrows, capacity) are NaN and capacity is a
// multiple of 128, so the ragged last tile needs no clamping or masking.
// Algorithmic bytes per tile: 32 * D * esize.
#pragma once
#include "k_mfma_common.h"

namespace rfx {
namespace k5 {

using mfc::batomic_umax;
using mfc::bdma;
using mfc::bdma_nt;
using mfc::bdma_sc1;
using mfc::fold;
using mfc::make_rsrc;
using mfc::v4i32;
using mfc::glds;
using mfc::glds_sc1;
using mfc::mfma;
using mfc::mfma16;
using mfc::v4f32x4;
using mfc::tau_min;
using mfc::unord;
using mfc::v4f32x16;

using mfc::Acc4View;

constexpr int kWaves = 8;
constexpr int kTM = 32;                   // rows per tile
constexpr int kQW = 32;                   // queries per wave
constexpr int kQG = kWaves * kQW;         // 256 queries per workgroup
constexpr int kSK = 256;                  // dims per stage
constexpr int kRowB = kSK * 2;            // 512 B per row per stage
constexpr int kSlot = kTM * kRowB;        // 16 KB
constexpr int kRing = 6;                  // 5 stages (80 KB) in flight
constexpr int kGPW = kSlot / 1024 / kWaves;  // LDS-DMA wave-instructions per wave per stage (2)
constexpr int kTauW = 16;                 // u32 per query in the threshold table (KL <= 10 used)
// Threshold-table refreshes go out after the last stage of tiles 3, 7, 11, ... (16 KB of DMA each).
// Measured: refreshing only every 16th tile after tile 31 made the kernel 20 % slower (a staler
// bound sends more lanes into the insert path), so the table is refreshed every 4 tiles throughout.
// (MODE 524288, diagnostic: every 2nd tile.  The vmcnt windows below allow refresh tiles >= 2 apart.)
template <int MODE>
__device__ __forceinline__ bool tau_refresh_tile(int it) {
  // production: right after tiles 0 and 1 (the lists start empty, so the first tiles take the
  // slow insert path until the slot table's bound arrives: 2x fewer slow entries, -13 us per
  // launch at 8 tiles per block, tools/early_refresh.py), then every 4 tiles.
  // MODE 4194304: every 4 tiles only; 8388608: also after tile 2; 524288: every 2 tiles.
  if constexpr ((MODE & 8388608) != 0) return it < 4 || (it & 3) == 3;
  if constexpr ((MODE & 4194304) != 0) return (it & 3) == 3;
  if constexpr ((MODE & 524288) != 0) return (it & 1) == 1;
  return it < 2 || (it & 3) == 3;
}
constexpr int kTauOff = kRing * kSlot;    // 96 KB
constexpr int kTauBytes = kQG * kTauW * 4;  // 16 KB: 16 DMA wave-instructions, 2 per wave
constexpr int kTauGPW = kTauBytes / 1024 / kWaves;
constexpr int kListOff = kTauOff + kTauBytes;
template <int KL>
constexpr int lds_bytes() { return kListOff + kWaves * KL * 64 * 8; }  // + lane lists [wave][KL][64] u64
static_assert(lds_bytes<10>() <= 163840, "LDS budget");
static_assert(kGPW == 2 && kTauGPW == 2, "DMA pieces per wave");

// MODE (profiling ablations, production = 0), bit flags: 1 = no top-k epilogue, 2 = no MFMA,
// 8 = no corpus stream after the prologue, 16 = count the lanes' top-k slow-path entries into
// cand_r[0] instead of writing candidates, 64 = a stage's DMA pieces bunched after the barrier,
// 128 = fragment prefetch distance 1 instead of 2, 256 = every corpus piece re-reads tile 0,
// 512 = shared threshold table ignored, 1024 = no pruning bound at all, 2048 = threshold table
// refreshed by a plain (L1) buffer LDS-DMA, 4096 = by global_load_lds sc1, 8192 = write each lane
// list's final pruning bound instead of candidates, 16384 = stage-end wait drains vmcnt to 0,
// 32768 = stage-end wait one stage stricter, 65536 = write every list entry (no final bound),
// 131072 = v_mfma_f32_16x16x32 shape (S16), 262144 = every other A fragment reused (half the LDS
// reads; wrong scores, timing only), 524288 = threshold refresh every 2nd tile, 1048576 = corpus
// DMA with the non-temporal hint.
// MODE bit for the row-masked (metadata-filter) production variant; all other bits are ablations
constexpr int kModeMask = 2097152;

template <int DT, int KL, int D, int MODE = 0>
__global__ __launch_bounds__(512, 1) void scan_mfma5_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Qp,
                                                            int nq, int ntiles, uint32_t* __restrict__ tau,
                                                            float* __restrict__ cand_s, int* __restrict__ cand_r,
                                                            int64_t n_lists, const uint32_t* __restrict__ mask) {
  // S16: v_mfma_f32_16x16x32 (2 row blocks × 2 query blocks per 32-deep k-step) instead of one
  // v_mfma_f32_32x32x16 per 16-deep k-step: same LDS bytes and MFMA cycles per FLOP; the chip holds
  // a higher clock on it with random operands (MI355X_MICROARCH.md 'DVFS give-back' item 7).
  constexpr bool S16 = (MODE & 131072) != 0;
  constexpr int KD = S16 ? 32 : 16;  // depth of one k-step
  constexpr int NKS = D / KD;        // k-steps per tile
  constexpr int NST = D / kSK;       // stages per tile
  constexpr int KPS = kSK / KD;      // k-steps per stage (16 | 8)
  static_assert(D % kSK == 0, "D must be a multiple of 256");
  static_assert(KL <= 10, "threshold table holds 10 slots");
  __shared__ __attribute__((aligned(1024))) uint8_t lds[lds_bytes<KL>()];

  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int half = lane >> 5, l32 = lane & 31;
  const int range = blockIdx.x;
  const int qg = blockIdx.y * kQG;
  // this lane's query: 32x32 layout: column l32; S16 (after the epilogue's pair swap): lanes of
  // odd 16-lane row hold query block 1
  const int q = S16 ? qg + w * kQW + 16 * ((lane >> 4) & 1) + (lane & 15) : qg + w * kQW + l32;
  // tile mapping: block b of B takes tiles b, b + B, ... (the grid streams one window of the store)
  const int nblk = gridDim.x;
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

  // ---- resident query fragments ----
  // 32x32x16: B[k][col], lane holds col l32, k = 16 ks + 8 half + j
  // 16x16x32: B[k][col] per query block qb, lane holds col 16 qb + (lane & 15), k = 32 ks + 8 (lane >> 4) + j
  constexpr int NB = S16 ? 2 * NKS : NKS;
  uint4 bq[NB];
  if constexpr (S16) {
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const uint16_t* qa = Qp + (int64_t)(qg + w * kQW + 16 * qb + (lane & 15)) * D + 8 * (lane >> 4);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) bq[2 * ks + qb] = *(const uint4*)(qa + 32 * ks);
    }
  } else {
    const uint16_t* qa = Qp + (int64_t)q * D + 8 * half;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) bq[ks] = *(const uint4*)(qa + 16 * ks);
  }

  // ---- LDS-DMA pattern: wave-instruction i (0..15) fills slot bytes [1024 i, +1024) = rows 2i,
  // 2i+1; lane -> (row 2i + lane/32, position lane%32) <- source chunk position ^ (row & 15);
  // wave w issues i = w + 8u, u = 0..1.
  uint32_t laneoff[kGPW];  // byte offset of this lane's 16 B inside a [32 rows][D] tile (stage 0)
#pragma unroll
  for (int u = 0; u < kGPW; ++u) {
    const int r = 2 * (w + kWaves * u) + half;
    laneoff[u] = (uint32_t)(r * D + ((l32 ^ (r & 15)) * 8)) * 2u;
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  // piece u of stage gi -> LDS slot `slot`.  gi is clamped to the last stage so the tail of the
  // stream issues harmless duplicate loads into free slots: every stage issues exactly kGPW
  // LDS-DMA ops per wave and the counted waits stay exact.
  auto issue_piece = [&](int gi, int slot, int u) {
    gi = gi < S ? gi : S - 1;
    if constexpr ((MODE & 256) != 0) gi = 0;
    const int ti = gi / NST;
    const int si = gi - ti * NST;
    const uint16_t* tbase = X + (int64_t)(range + ti * nblk) * kTM * D + si * kSK;
    const uint32_t dst = lds_base + (uint32_t)(slot * kSlot) + (uint32_t)((w + kWaves * u) * 1024);
    if constexpr ((MODE & 1048576) != 0)
      bdma_nt(make_rsrc(tbase), laneoff[u], __builtin_amdgcn_readfirstlane(dst));
    else
      bdma(make_rsrc(tbase), laneoff[u], __builtin_amdgcn_readfirstlane(dst));
  };
  // threshold table of the 256 queries -> LDS image (16 KB; wave w moves pieces w, w + 8)
  const v4i32 tau_rsrc = make_rsrc(tau);
  auto issue_tau = [&]() {
#pragma unroll
    for (int u = 0; u < kTauGPW; ++u) {
      const int i = w + kWaves * u;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + kTauOff + i * 1024);
      const uint32_t off = (uint32_t)(qg * kTauW * 4 + tid * 16 + u * kWaves * 1024);
      if constexpr ((MODE & 2048) != 0)
        bdma(tau_rsrc, off, dst);
      else if constexpr ((MODE & 4096) != 0)
        glds_sc1((const uint8_t*)tau + off, dst);
      else
        bdma_sc1(tau_rsrc, off, dst);
    }
  };

  uint32_t thr = 0u;  // pruning bound (orderable score; 0 = none)
  const uint32_t slot_voff = (uint32_t)(q * kTauW + lst % KL) * 4u;
  const uint8_t* const tq = lds + kTauOff + (w * kQW + l32) * (kTauW * 4);
  int n_slow = 0;  // slow-path entries of this lane (diagnostic MODE 16 only; dead code otherwise)
  // A fragments.  32x32x16: rows l32, k chunk 2 kk + half.  16x16x32: rows 16 rb + (lane & 15),
  // k chunk 4 kk + (lane >> 4), rb = 0, 1 (8 KB apart).
  const uint8_t* frag_base = lds + (S16 ? (lane & 15) : l32) * kRowB;
  const int sw = S16 ? (lane & 15) : (l32 & 15);
  struct Frag {
    uint4 a[S16 ? 2 : 1];
  };
  auto read_frag = [&](int slot, int kk) -> Frag {
    Frag f;
    if constexpr (S16) {
      const uint8_t* p = frag_base + slot * kSlot + (((4 * kk + (lane >> 4)) ^ sw) << 4);
      f.a[0] = *(const uint4*)p;
      f.a[1] = *(const uint4*)(p + 16 * kRowB);
    } else {
      f.a[0] = *(const uint4*)(frag_base + slot * kSlot + (((2 * kk + half) ^ sw) << 4));
    }
    return f;
  };

  // Schedule.  Stage h's pieces go out during stage h - 5, at k-steps 0 and 8 (spread), into the
  // slot freed at stage h - 6's barrier.  Fragments are read PF k-steps ahead of their MFMA; the
  // stage-end wait + barrier sit at k-step KPS - PF, once every wave has issued (and, by
  // lgkmcnt(0), received) its last read of the stage.
  constexpr bool kSpread = (MODE & 64) == 0;
  constexpr int PF = ((MODE & 128) != 0) != S16 ? 1 : 2;  // S16 (two fragments per k-step): 1 by default
  constexpr int NF = PF + 1;      // fragment registers in rotation
  constexpr int KB = KPS - PF;    // k-step of the stage-end wait + barrier
  constexpr int AHEAD = kSpread ? kRing - 1 : kRing;  // stages issued by the prologue
  constexpr int YNG = (kRing - 2) * kGPW;             // ops younger than the next stage (8)
  static_assert((NST * KPS) % NF == 0, "fragment rotation must realign every tile");

  // the resident query loads must land before the LDS-DMA stream starts counting
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  issue_tau();
#pragma unroll
  for (int p = 0; p < AHEAD; ++p)
#pragma unroll
    for (int u = 0; u < kGPW; ++u) issue_piece(p, p, u);
  // stage 0 landed: stages 1..AHEAD-1 younger
  if constexpr (kSpread)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(YNG) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(YNG + kGPW) : "memory");
  asm volatile("s_barrier" ::: "memory");

  Frag fr[NF];
#pragma unroll
  for (int i = 0; i < PF; ++i) fr[i] = read_frag(0, i);
  v4f32x16 acc;
  v4f32x4 acc4[4];  // S16: [rb * 2 + qb]
  for (int it = 0; it < nt; ++it) {
    const int tile = range + it * nblk;
    const int gbase = it * NST;
    if constexpr ((MODE & 1) == 0) {
      // refreshed threshold image (issued 2 tiles ago; any image value is a valid bound), read
      // before the tile's first MFMA while the accumulator is dead.
      if constexpr ((MODE & 512) == 0)
        if (it >= 2 && tau_refresh_tile<MODE>(it - 2)) thr = max(thr, tau_min<KL>(tq));
    }
    // A threshold refresh (kTauGPW ops) issued after the barrier of stage g_r = last stage of a
    // refresh tile it_r is younger than stage g+1's pieces iff g-4 <= g_r <= g-1: at every stage
    // of tile it_r + 1 and at stage 0 of tile it_r + 2.  Where two refreshes overlap (tiles 0, 1)
    // the count below admits one: the wait is then stricter than needed, never looser.
    const bool tau_young12 = it >= 1 && tau_refresh_tile<MODE>(it - 1);
    const bool tau_young0 = tau_young12 || (it >= 2 && tau_refresh_tile<MODE>(it - 2));
#pragma unroll
    for (int s = 0; s < NST; ++s) {
      const int g = gbase + s;
      const int slot = g % kRing;
#pragma unroll
      for (int kk = 0; kk < KPS; ++kk) {
        if constexpr (kSpread && (MODE & 8) == 0) {
          constexpr int SP = KPS / kGPW;  // k-steps between a stage's DMA pieces
          if (kk % SP == 0) issue_piece(g + kRing - 1, (g + kRing - 1) % kRing, kk / SP);
        }
        if (kk == KB) {
          // stage g+1 landed for this wave: ops younger than its pieces = stages g+2..g+5 (8)
          // [+ a threshold refresh (2)]; lgkmcnt(0) + barrier: every wave has received its last
          // fragment of slot g, which may be refilled from here on.
          if constexpr ((MODE & 16384) != 0) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // diagnostic: drain
          } else if constexpr ((MODE & 32768) != 0) {
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(YNG - kGPW) : "memory");  // one stage stricter
          } else if constexpr ((MODE & 8) == 0) {
            if (s == 0 ? tau_young0 : tau_young12)
              asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(YNG + kTauGPW) : "memory");
            else
              asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(YNG) : "memory");
          } else {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
          asm volatile("s_barrier" ::: "memory");
          if constexpr ((MODE & 8) == 0) {
            if (s == NST - 1 && tau_refresh_tile<MODE>(it)) issue_tau();
            if constexpr (!kSpread) {
#pragma unroll
              for (int u = 0; u < kGPW; ++u) issue_piece(g + kRing, slot, u);
            }
          }
        }
        const int ks = s * KPS + kk;
        // prefetch k-step kk + PF (crossing into stage g+1 after the barrier)
        if constexpr ((MODE & 262144) != 0) {  // diagnostic: every other fragment reused, half the LDS reads
          if ((ks & 1) == 0)
            fr[(ks + PF) % NF] = fr[(ks + PF - 1) % NF];
          else
            fr[(ks + PF) % NF] = kk + PF < KPS ? read_frag(slot, kk + PF) : read_frag((g + 1) % kRing, kk + PF - KPS);
        } else {
          fr[(ks + PF) % NF] = kk + PF < KPS ? read_frag(slot, kk + PF) : read_frag((g + 1) % kRing, kk + PF - KPS);
        }
        const Frag& cur = fr[ks % NF];
        if constexpr ((MODE & 2) == 0) {
          if constexpr (S16) {
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // the prefetch reads go out first
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
#pragma unroll
              for (int qb = 0; qb < 2; ++qb)
                acc4[2 * rb + qb] = ks == 0 ? mfma16<DT>(cur.a[rb], bq[2 * ks + qb], v4f32x4{})
                                            : mfma16<DT>(cur.a[rb], bq[2 * ks + qb], acc4[2 * rb + qb]);
          } else {
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // the prefetch read goes out first
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            acc = ks == 0 ? mfma<DT>(cur.a[0], bq[ks], v4f32x16{}) : mfma<DT>(cur.a[0], bq[ks], acc);
          }
        } else {
          if (ks == 0) acc = v4f32x16{};
          acc[kk & 15] += __uint_as_float(cur.a[0].x & 0x3f000000u);  // keep the reads live
        }
      }
    }

    // ---- epilogue: fold this tile's 32 rows into the lane list ----
    if constexpr (S16 && (MODE & 2) == 0) {
      // pair swap, in place, one v_permlane16_swap per register pair: lane (n, g) holds rows
      // 16 rb + 4 g + i of queries n (qb 0) and 16 + n (qb 1).  The swap trades the odd 16-lane rows
      // of the qb-0 register with the even rows of the qb-1 register, so afterwards a lane of even
      // g holds query n and one of odd g query 16 + n, acc4[2 rb + gg][i] being row
      // 16 rb + 8 (g >> 1) + 4 gg + i: flat value rb*8 + gg*4 + i (fold's ROWMAP 1).
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc4[2 * rb][i]),
                                                          __float_as_uint(acc4[2 * rb + 1][i]), false, false);
          acc4[2 * rb][i] = __uint_as_float(r[0]);
          acc4[2 * rb + 1][i] = __uint_as_float(r[1]);
        }
    }
    if constexpr ((MODE & 1) == 0) {
      const int rbase = S16 ? tile * kTM + 8 * half : tile * kTM + 4 * half;
      uint32_t t0 = 0u;  // MODE 1024 (diagnostic): no pruning bound at all
      uint32_t& bound = (MODE & 1024) != 0 ? t0 : thr;
      if constexpr (S16) {
        fold<KL, 1>(Acc4View{acc4}, Ls, bound, rbase, tau_rsrc, slot_voff, n_slow);
      } else {
        // metadata filter: one mask word per 32-row tile (uniform load); excluded rows -> NaN
        if constexpr ((MODE & kModeMask) != 0) mask_acc16(acc, mask[tile] >> (4 * half));
        fold<KL, 0>(acc, Ls, bound, rbase, tau_rsrc, slot_voff, n_slow);
      }
    } else {
      if (acc[0] == 12345.f) Ls[0] = 1;  // keep the MFMAs live
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr ((MODE & 16) != 0) {  // diagnostic: total slow-path entries -> cand_r[0]
    atomicAdd(cand_r, n_slow);
    return;
  }
  if constexpr ((MODE & 8192) != 0) {  // diagnostic: final pruning bound of every lane list
    cand_s[(int64_t)q * n_lists + lst] = thr ? unord(thr) : -__builtin_inff();
    cand_r[(int64_t)q * n_lists + lst] = (int)(tau_min<KL>(tq) == thr);
    return;
  }
  if (q < nq) {
    // Drop entries below the query's bound as it stands now, read fresh from the slot table (all
    // workgroups end together, so it is close to final): valid bound => exact, and the merge then
    // sees ~k live candidates per query instead of 512 lists.
    uint32_t fin = thr;
    if constexpr ((MODE & 65536) == 0) {
      uint32_t m = 0xffffffffu;
#pragma unroll
      for (int j = 0; j < KL; ++j)
        m = min(m, __hip_atomic_load(tau + (int64_t)q * kTauW + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      fin = max(fin, m);
    }
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

// one translation unit per (dtype, D) instantiates the kernel for the lane-list sizes KL in {4, 10}
#define RFX_K5_INSTANTIATE(DTV, DV, NAME)                                                                  \
  int NAME(int kl, dim3 grid, hipStream_t st, const uint16_t* X, const uint16_t* Qp, int nq, int ntiles,     \
           uint32_t* tau, float* cs, int* cr, int64_t n_lists, const uint32_t* mask) {                      \
    if (kl == 4 && !mask)                                                                                \
      hipLaunchKernelGGL((scan_mfma5_kernel<DTV, 4, DV>), grid, dim3(512), 0, st, X, Qp, nq, ntiles, tau, cs, \
                         cr, n_lists, mask);                                                              \
    else if (kl == 10 && !mask)                                                                          \
      hipLaunchKernelGGL((scan_mfma5_kernel<DTV, 10, DV>), grid, dim3(512), 0, st, X, Qp, nq, ntiles, tau,  \
                         cs, cr, n_lists, mask);                                                          \
    else if (kl == 4)                                                                                    \
      hipLaunchKernelGGL((scan_mfma5_kernel<DTV, 4, DV, kModeMask>), grid, dim3(512), 0, st, X, Qp, nq,     \
                         ntiles, tau, cs, cr, n_lists, mask);                                             \
    else if (kl == 10)                                                                                   \
      hipLaunchKernelGGL((scan_mfma5_kernel<DTV, 10, DV, kModeMask>), grid, dim3(512), 0, st, X, Qp, nq,    \
                         ntiles, tau, cs, cr, n_lists, mask);                                             \
    else                                                                                                 \
      return -1;                                                                                         \
    return 0;                                                                                            \
  }

}  // namespace k5
}  // namespace rfx
