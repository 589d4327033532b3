// k_scan_mfma4.h — all-query-stationary batched scan: one workgroup holds 256 queries.
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551),
// BASELINE.json config 3 (10M×768 bf16, nq=256, k=10).  Fused scan + per-query top-k; the score
// matrix never reaches HBM.
//
// Why (measured, profiles/r01_v3_*): the 128-query kernel (k_scan_mfma3.h) needs two workgroups
// per row range at nq=256.  The second read of each tile was meant to hit L2, but rocprofv3
// FETCH_SIZE showed 24.3 GB of fabric reads per launch against 15.36 GB of corpus (1.58×).  Here one
// workgroup covers all 256 queries, so every corpus byte crosses the fabric once, and each LDS
// fragment read feeds two MFMAs instead of one:
//   * workgroup = 4 waves (one per SIMD, 512 registers each) × 64 queries.  Each wave keeps its
//     64 queries' B-fragments for the whole of K resident: 2 × D/16 × 16 B per lane
//     (384 registers at d = 768, split by the compiler between VGPRs and AGPRs).
//   * tile = 32 corpus rows; a stage = 32 rows × 192 dims (12 KB) arrives by LDS-DMA
//     (global_load_lds_dwordx4, 3 wave-instructions per wave) into a 9-slot ring, 8 stages
//     (96 KB) in flight; one counted `s_waitcnt vmcnt` + `s_barrier` per stage.
//   * LDS row image: 384 B per row; 16-B chunk c of row r sits at position c ^ ((r >> 1) & 7)
//     (stays inside c's aligned 8-chunk block), so the 32-row ds_read_b128 fragment reads are
//     bank-conflict free in all four lane groups; the permutation rides on the LDS-DMA source
//     address.
//   * per k-step and wave: 1 ds_read_b128 (rows × 16 k) → 2 × v_mfma_f32_32x32x16 (query blocks
//     0 and 1), accumulators 2 × 16 registers.
//   * top-k: lane l holds queries (l&31) and 32+(l&31) of its wave for 16 rows per tile; two
//     sorted lane lists of KL 64-bit keys (orderable score << 32 | ~row) kept in LDS (a register
//     holds each list's pruning bound).
//   * pruning threshold shared across workgroups (measured: with each list publishing its own
//     KL-th best, 1.7 % of lane-folds still took the insert path and the epilogue cost 20 % of
//     the kernel): per query a table of KL slots; list j (of 2 per workgroup) publishes its BEST
//     key's score to slot j % KL by device atomicMax.  The KL slots hold scores of KL distinct
//     rows, so min(slots) ≤ the query's KL-th best, and max(own KL-th best, min(slots)) is a valid
//     pruning bound whatever stale value a workgroup sees: the result stays exact.  The table
//     ([nq][12] u32) is refreshed into LDS by LDS-DMA every 4 tiles; each lane takes the min of
//     its queries' slots every 4 tiles.
// Requires the index invariant of rfx_api.hip: rows [nrows, capacity) are NaN and capacity is a
// multiple of 128, so the ragged last tile needs no clamping or masking.
// Algorithmic bytes per tile: 32 * D * esize.
#pragma once
#include "k_mfma_common.h"

namespace rfx {
namespace k4 {

using namespace mfc;

constexpr int kTM = 32;                  // rows per tile
constexpr int kQW = 64;                  // queries per wave
constexpr int kQG = 256;                 // queries per workgroup
constexpr int kSK = 192;                 // dims per stage
constexpr int kRowB = kSK * 2;           // 384 B per row per stage
constexpr int kSlot = kTM * kRowB;       // 12 KB
constexpr int kRing = 9;                 // 8 stages (96 KB) in flight
constexpr int kGPW = kSlot / 1024 / 4;   // LDS-DMA wave-instructions per wave per stage (3)
constexpr int kTauW = 12;                // u32 per query in the threshold table (KL <= 10 slots used)
constexpr int kTauEvery = 4;             // tiles between threshold refreshes
constexpr int kTauOff = kRing * kSlot;   // 108 KB
constexpr int kTauBytes = kQG * kTauW * 4;  // 12 KB: 12 DMA wave-instructions, 3 per wave
constexpr int kListOff = kTauOff + kTauBytes;
template <int KL>
constexpr int lds_bytes() { return kListOff + 4 * 2 * KL * 64 * 8; }  // + lane lists [wave][2][KL][64] u64
static_assert(lds_bytes<10>() <= 163840, "LDS budget");
static_assert(kGPW * 4 * 1024 == kSlot && kTauBytes == 3 * 4 * 1024, "DMA pieces per wave");

// Tile mapping: block b of B takes tiles b, b + B, b + 2B, ... so at any moment the whole grid
// streams one contiguous window of the store (even spread over HBM channels).
// MODE (profiling ablations, production = 0), bit flags: 1 = no top-k epilogue, 2 = no MFMA,
// 4 = contiguous row range per block (tiles b·T .. b·T + T - 1, T = tiles_per_block),
// 8 = no corpus stream after the prologue (MFMA + LDS reads on the first 9 stages, recycled),
// 16 = count the lanes' top-k slow-path entries into cand_r[0] instead of writing candidates,
// 32 = threshold refresh through L1 (plain load instead of sc1), 64 = all of a stage's DMA pieces
// right after the barrier (no spreading), 128 = fragment prefetch distance 1 instead of 2,
// 256 = every corpus piece re-reads tile 0 (same LDS traffic, no HBM stream: L2 hits).
template <int DT, int KL, int D, int MODE = 0>
__global__ __launch_bounds__(256, 1) void scan_mfma4_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Qp,
                                                            int nq, int tiles_per_block, int ntiles,
                                                            uint32_t* __restrict__ tau, float* __restrict__ cand_s,
                                                            int* __restrict__ cand_r, int64_t n_lists) {
  constexpr int NKS = D / 16;    // 16-deep MFMA k-steps
  constexpr int NST = D / kSK;   // stages per tile
  constexpr int KPS = kSK / 16;  // k-steps per stage (12)
  static_assert(D % kSK == 0, "D must be a multiple of 192");
  static_assert(KL <= 10, "threshold table holds 10 slots");
  __shared__ __attribute__((aligned(1024))) uint8_t lds[lds_bytes<KL>()];

  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int half = lane >> 5, l32 = lane & 31;
  const int range = blockIdx.x;
  const int qg = blockIdx.y * kQG;
  const int q0 = qg + w * kQW + l32;  // this lane's queries: q0 and q0 + 32
  constexpr bool kContig = (MODE & 4) != 0;
  const int nblk = gridDim.x;
  const int t0 = kContig ? range * tiles_per_block : range;                // first tile
  const int tstep = kContig ? 1 : nblk;                                    // tile stride
  const int nt = kContig ? max(0, min(ntiles, t0 + tiles_per_block) - t0)  // tiles of this block
                         : (range < ntiles ? (ntiles - range + nblk - 1) / nblk : 0);
  const int S = nt * NST;
  if (S == 0) return;  // (cannot happen with the host plan; whole workgroup exits together)
  const int lst = range * 2 + half;  // this lane's list id (per query)

  // ---- LDS init: threshold image and lane lists start at 0 (= "no bound" / empty) ----
  {
    uint4* tz = (uint4*)(lds + kTauOff);
#pragma unroll
    for (int i = 0; i < kTauBytes / 16 / 256; ++i) tz[tid + 256 * i] = uint4{0u, 0u, 0u, 0u};
  }
  uint64_t* const Ls0 = (uint64_t*)(lds + kListOff) + (w * 2 * KL) * 64 + lane;
  uint64_t* const Ls1 = Ls0 + KL * 64;
#pragma unroll
  for (int i = 0; i < KL; ++i) Ls0[i * 64] = Ls1[i * 64] = 0ull;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();  // no LDS-DMA in flight yet: a plain barrier

  // ---- resident query fragments: B[k][col] of 32x32x16, lane holds k = 16 ks + 8 half + j ----
  uint4 bq0[NKS], bq1[NKS];
  {
    const uint16_t* qa = Qp + (int64_t)q0 * D + 8 * half;
    const uint16_t* qb = qa + (int64_t)32 * D;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      bq0[ks] = *(const uint4*)(qa + 16 * ks);
      bq1[ks] = *(const uint4*)(qb + 16 * ks);
    }
  }

  // ---- LDS-DMA pattern: wave-instruction i (0..11) fills slot bytes [1024 i, +1024): lane L
  // writes linear chunk n = 64 i + L = (row n / 24, position n % 24) <- source chunk
  // position ^ ((row >> 1) & 7); wave w issues i = w + 4u, u = 0..2.
  int laneoff[kGPW];  // element offset of this lane's 16 B inside a [32 rows][D] tile (stage 0)
#pragma unroll
  for (int u = 0; u < kGPW; ++u) {
    const int n = 64 * (w + 4 * u) + lane;
    const int r = n / 24, p = n - 24 * (n / 24);
    laneoff[u] = r * D + ((p ^ ((r >> 1) & 7)) * 8);
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  // Stage gi -> LDS slot `slot`.  gi is clamped to the last stage so the tail of the stream issues
  // harmless duplicate loads into already-consumed slots: every stage issues exactly kGPW LDS-DMA
  // ops per wave, the counted waits stay exact, and the tile body has no branches.
  auto issue = [&](int gi, int slot) {
    gi = gi < S ? gi : S - 1;
    if constexpr ((MODE & 256) != 0) gi = 0;
    const int ti = gi / NST;
    const int si = gi - ti * NST;
    const uint16_t* tbase = X + (int64_t)(t0 + ti * tstep) * kTM * D + si * kSK;
    const uint32_t dst = lds_base + (uint32_t)(slot * kSlot) + (uint32_t)(w * 1024);
#pragma unroll
    for (int u = 0; u < kGPW; ++u) glds(tbase + laneoff[u], __builtin_amdgcn_readfirstlane(dst + u * 4096));
  };
  // one of the kGPW pieces of stage gi (same clamping)
  auto issue_piece = [&](int gi, int slot, int u) {
    gi = gi < S ? gi : S - 1;
    if constexpr ((MODE & 256) != 0) gi = 0;
    const int ti = gi / NST;
    const int si = gi - ti * NST;
    const uint16_t* tbase = X + (int64_t)(t0 + ti * tstep) * kTM * D + si * kSK;
    const uint32_t dst = lds_base + (uint32_t)(slot * kSlot) + (uint32_t)(w * 1024);
    glds(tbase + laneoff[u], __builtin_amdgcn_readfirstlane(dst + u * 4096));
  };
  // threshold table of the 256 queries -> LDS image (12 KB; wave w moves pieces w, w+4, w+8)
  const uint32_t* tau_g = tau + (int64_t)qg * kTauW;
  auto issue_tau = [&]() {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int i = w + 4 * u;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + kTauOff + i * 1024);
      if constexpr ((MODE & 32) != 0)
        glds(tau_g + i * 256 + lane * 4, dst);
      else
        glds_sc1(tau_g + i * 256 + lane * 4, dst);
    }
  };

  uint32_t thr0 = 0u, thr1 = 0u;  // pruning bounds (orderable scores; 0 = none)
  const v4i32 tau_rsrc = make_rsrc(tau);
  const uint32_t slot_voff = (uint32_t)(q0 * kTauW + lst % KL) * 4u;  // this lane's slot of query q0
  const uint8_t* const tq = lds + kTauOff + (w * kQW + l32) * (kTauW * 4);
  int n_slow = 0;  // slow-path entries of this lane (diagnostic MODE 16 only; dead code otherwise)
  const uint8_t* frag_base = lds + l32 * kRowB;
  const int sw = (l32 >> 1) & 7;
  auto read_frag = [&](int slot, int kk) -> uint4 {
    return *(const uint4*)(frag_base + slot * kSlot + (((2 * kk + half) ^ sw) << 4));
  };

  // Schedule.  Stage h's 3 pieces per wave go out during stage h - 8, one every 4 k-steps
  // (kSpread; bunched right after a barrier each piece costs the issuing wave ~150 cycles while
  // its MFMAs starve), into the slot freed at stage h - 9's barrier.  Fragments are read PF
  // k-steps ahead of their MFMAs; the stage-end wait + barrier sit at k-step KPS - PF, once every
  // wave has issued (and, by lgkmcnt(0), received) its last read of the stage.
  constexpr bool kSpread = (MODE & 64) == 0;
  constexpr int PF = (MODE & 128) ? 1 : 2;
  constexpr int NF = PF + 1;      // fragment registers in rotation
  constexpr int KB = KPS - PF;    // k-step of the stage-end wait + barrier
  constexpr int AHEAD = kSpread ? kRing - 1 : kRing;  // stages issued by the prologue
  static_assert((NST * KPS) % NF == 0, "fragment rotation must realign every tile");

  // the resident query loads must land before the LDS-DMA stream starts counting
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  issue_tau();
#pragma unroll
  for (int p = 0; p < AHEAD; ++p) issue(p, p);
  // stage 0 landed: stages 1..AHEAD-1 younger
  if constexpr (kSpread)
    asm volatile("s_waitcnt vmcnt(21)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  asm volatile("s_barrier" ::: "memory");

  uint4 fr[NF];
#pragma unroll
  for (int i = 0; i < PF; ++i) fr[i] = read_frag(0, i);
  v4f32x16 acc0, acc1;
  for (int it = 0; it < nt; ++it) {
    const int tile = t0 + it * tstep;
    const int gbase = it * NST;
    if constexpr ((MODE & 1) == 0) {
      // refreshed threshold image (issued 2 tiles ago; any image value is a valid bound).  Here,
      // before the tile's first MFMA, the accumulators are dead: no register pressure.
      if ((it & (kTauEvery - 1)) == 1) {
        thr0 = max(thr0, tau_min<KL>(tq));
        thr1 = max(thr1, tau_min<KL>(tq + 32 * kTauW * 4));
      }
    }
#pragma unroll
    for (int s = 0; s < NST; ++s) {
      const int g = gbase + s;
      const int slot = g % kRing;
#pragma unroll
      for (int kk = 0; kk < KPS; ++kk) {
        if constexpr (kSpread && (MODE & 8) == 0) {
          if (kk % 4 == 0 && kk / 4 < kGPW) issue_piece(g + kRing - 1, (g + kRing - 1) % kRing, kk / 4);
        }
        if (kk == KB) {
          // Stage g+1 must have landed for this wave.  Ops younger than its pieces: stages
          // g+2..g+8 (21) plus a threshold refresh (3) issued after the barrier of a stage g_r
          // with g-7 <= g_r <= g-1; refreshes go out every kTauEvery-th tile (g_r ≡ 15 mod 16).
          // lgkmcnt(0) + barrier: every wave has received its last fragment of slot g, so
          // slot g may be refilled from here on.
          if constexpr ((MODE & 8) == 0) {
            if (g >= kTauEvery * NST && (g & (kTauEvery * NST - 1)) <= 6)
              asm volatile("s_waitcnt vmcnt(24) lgkmcnt(0)" ::: "memory");
            else
              asm volatile("s_waitcnt vmcnt(21) lgkmcnt(0)" ::: "memory");
          } else {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
          asm volatile("s_barrier" ::: "memory");
          if constexpr ((MODE & 8) == 0) {
            if (s == NST - 1 && (it & (kTauEvery - 1)) == kTauEvery - 1) issue_tau();
            if constexpr (!kSpread) issue(g + kRing, slot);
          }
        }
        const int ks = s * KPS + kk;
        // prefetch k-step kk + PF (crossing into stage g+1 after the barrier)
        fr[(ks + PF) % NF] = kk + PF < KPS ? read_frag(slot, kk + PF) : read_frag((g + 1) % kRing, kk + PF - KPS);
        const uint4& cur = fr[ks % NF];
        if constexpr ((MODE & 2) == 0) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // the prefetch read goes out first
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          if (ks == 0) {
            acc0 = mfma<DT>(cur, bq0[ks], v4f32x16{});
            acc1 = mfma<DT>(cur, bq1[ks], v4f32x16{});
          } else {
            acc0 = mfma<DT>(cur, bq0[ks], acc0);
            acc1 = mfma<DT>(cur, bq1[ks], acc1);
          }
        } else {
          if (ks == 0) acc0 = acc1 = v4f32x16{};
          acc0[kk & 15] += __uint_as_float(cur.x & 0x3f000000u);  // keep the reads live
        }
      }
    }

    // ---- epilogue: fold this tile's 32 rows into the two lane lists ----
    if constexpr ((MODE & 1) == 0) {
      const int rbase = tile * kTM + 4 * half;
      fold<KL>(acc0, Ls0, thr0, rbase, tau_rsrc, slot_voff, n_slow);
      fold<KL>(acc1, Ls1, thr1, rbase, tau_rsrc, slot_voff + 32 * kTauW * 4, n_slow);
    } else {
      if (acc0[0] == 12345.f && acc1[1] == 54321.f) Ls0[0] = 1;  // keep the MFMAs live
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr ((MODE & 16) != 0) {  // diagnostic: total slow-path entries -> cand_r[0]
    atomicAdd(cand_r, n_slow);
    return;
  }

  if (q0 < nq) {
    const int64_t o = ((int64_t)q0 * n_lists + lst) * KL;
#pragma unroll
    for (int i = 0; i < KL; ++i) {
      const uint64_t key = Ls0[i * 64];
      cand_s[o + i] = key ? unord((uint32_t)(key >> 32)) : -__builtin_inff();
      cand_r[o + i] = key ? (int)(~(uint32_t)key) : kEmptyRow;
    }
  }
  if (q0 + 32 < nq) {
    const int64_t o = ((int64_t)(q0 + 32) * n_lists + lst) * KL;
#pragma unroll
    for (int i = 0; i < KL; ++i) {
      const uint64_t key = Ls1[i * 64];
      cand_s[o + i] = key ? unord((uint32_t)(key >> 32)) : -__builtin_inff();
      cand_r[o + i] = key ? (int)(~(uint32_t)key) : kEmptyRow;
    }
  }
}

// one translation unit per (dtype, D) instantiates the kernel for the lane-list sizes KL in {4, 10}
#define RFX_K4_INSTANTIATE(DTV, DV, NAME)                                                                   \
  int NAME(int kl, dim3 grid, hipStream_t st, const uint16_t* X, const uint16_t* Qp, int nq,                  \
           int tiles_per_block, int ntiles, uint32_t* tau, float* cs, int* cr, int64_t n_lists) {           \
    if (kl == 4)                                                                                          \
      hipLaunchKernelGGL((scan_mfma4_kernel<DTV, 4, DV>), grid, dim3(256), 0, st, X, Qp, nq, tiles_per_block, \
                         ntiles, tau, cs, cr, n_lists);                                                    \
    else if (kl == 10)                                                                                    \
      hipLaunchKernelGGL((scan_mfma4_kernel<DTV, 10, DV>), grid, dim3(256), 0, st, X, Qp, nq,              \
                         tiles_per_block, ntiles, tau, cs, cr, n_lists);                                   \
    else                                                                                                  \
      return -1;                                                                                          \
    return 0;                                                                                             \
  }

}  // namespace k4
}  // namespace rfx
