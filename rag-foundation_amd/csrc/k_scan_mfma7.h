// k_scan_mfma7.h — the d = 1024 batched scan (BASELINE config 4: 100M×1024 f16 over 8 GPUs, a
// 12.5M-row shard per GPU, nq 256, k 10): kernel 6's design with 16 resident queries per wave, so
// that two waves per SIMD still fit when a query's B-fragments take 1024 dims.
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551).
// Fused scan + per-query top-k; the score matrix never reaches HBM.
//
// Why a new kernel: at d = 1024 the B-fragments of 256 queries are 512 KB, the
// whole register file of a CU, so a CU holds at most 128 queries and nq = 256 needs two query
// groups sweeping the same rows.  Kernel 3 (one wave per SIMD, 32 queries per wave) paired the two
// groups only by launch order and read 1.81x the algorithmic bytes (profiles/pmc_traffic.json).
//   * Workgroup = 8 waves (two per SIMD) × 16 queries = 128 queries, B-fragments of the whole of d
//     resident in 128 VGPRs; v_mfma_f32_16x16x32 with A = 16 corpus rows, B = the wave's queries.
//   * Tile = 64 rows (4 row blocks): per 32-deep k-step a wave reads 4 A-fragments (ds_read_b128,
//     conflict-free) and issues 4 MFMAs.  Per CU that is 128 LDS-array cycles against 128 MFMA
//     cycles per SIMD: the LDS read rate equals the MFMA rate (kernel 6 reads half as much).
//   * XCD-paired query groups: block b runs on XCD b % 8 (round-robin dispatch); the G query
//     groups of a row range are consecutive slots on ONE XCD, start together and stream the same
//     tiles in the same order, so the second group's reads hit that XCD's L2.  Placement only
//     affects speed, never results.
//   * Stage = 64 rows × 128 dims (16 KB) by LDS-DMA (default cache policy, so the partner group's
//     read of the same lines hits L2; the non-temporal hint of kernel 6 made it miss) into a 6-slot ring (5 stages = 80 KB in
//     flight); LDS image 256 B per row per stage, 16-B chunk c of row r at c ^ (r & 15).
//   * Top-k epilogue, cross-workgroup slot table, output format: as kernel 6 (k_mfma_common.h
//     fold, ROWMAP 2: lane l holds query l & 15, rows 4 (l >> 4) + (r & 3) + 16 (r >> 2) of the
//     tile; four lists per query per workgroup).
// Requires the index invariant of rfx_api.hip: rows [nrows, capacity) are NaN and capacity is a
// multiple of 128, so the ragged last tile needs no clamping or masking.
// Algorithmic bytes per tile: 64 * D * esize.
#pragma once
#include "k_mfma_common.h"

namespace rfx {
namespace k7 {

using namespace mfc;

constexpr int kWaves = 8;
constexpr int kTM = 64;                   // rows per tile
constexpr int kRB = kTM / 16;             // 16-row MFMA blocks per tile
constexpr int kQW = 16;                   // queries per wave
constexpr int kQG = kWaves * kQW;         // 128 queries per workgroup
constexpr int kSK = 128;                  // dims per stage
constexpr int kRowB = kSK * 2;            // 256 B per row per stage
constexpr int kSlot = kTM * kRowB;        // 16 KB: 64 rows × 128 dims
constexpr int kRing = 6;                  // 6 slots, 5 stages (80 KB) in flight
constexpr int kGPW = 2;                   // LDS-DMA pieces per wave per stage (16 KB / 1 KB / 8 waves)
constexpr int kTauW = 16;                 // u32 per query in the threshold table (KL <= 10 used)
constexpr int kTauBytes = kQG * kTauW * 4;  // 8 KB: 8 DMA pieces, 1 per wave
constexpr int kTauGPW = kTauBytes / 1024 / kWaves;
constexpr int kListsPerBlock = 4;         // lane lists per query per workgroup (the 4 lanes of a query)
constexpr int kTauOff = kRing * kSlot;
constexpr int kListOff = kTauOff + kTauBytes;
template <int KL>
constexpr int lds_bytes() { return kListOff + kWaves * KL * 64 * 8; }
static_assert(lds_bytes<10>() <= 163840, "LDS budget");
static_assert(kSlot / 1024 == kWaves * kGPW && kTauGPW == 1, "DMA pieces per wave");

__device__ __forceinline__ bool tau_refresh_tile(int it) { return it < 2 || (it & 3) == 3; }

// Metadata filter: the tile's 64 row bits (two mask words) shifted by 4 (lane >> 4); value r of the
// lane is tile row 4 (lane >> 4) + (r & 3) + 16 (r >> 2).
template <class V>
__device__ __forceinline__ void mask_rowmap2(V& a, uint64_t bits) {
#pragma unroll
  for (int r = 0; r < 16; ++r)
    if (!((bits >> ((r & 3) + 16 * (r >> 2))) & 1ull)) a[r >> 2][r & 3] = __builtin_nanf("");
}

// MODE: 0 production; kModeMask = row-masked variant (metadata filter).
constexpr int kModeMask = 2097152;

// Block -> (row range, query group).  pair_g > 0: the pair_g query groups of a range sit on one XCD
// (requires gridDim.x = 8 * (ranges / 8) * pair_g... i.e. ranges % 8 == 0); 0: plain row-major.
__device__ __forceinline__ void block_map(int b, int ranges, int groups, bool paired, int& range, int& grp) {
  if (paired) {
    const int xcd = b & 7, s = b >> 3;
    range = (s / groups) * 8 + xcd;
    grp = s % groups;
  } else {
    range = b % ranges;
    grp = b / ranges;
  }
}

template <int DT, int KL, int D, int MODE = 0>
__global__ __launch_bounds__(512, 1) void scan_mfma7_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Qp,
                                                            int nq, int ntiles, int ranges, int groups, int paired,
                                                            uint32_t* __restrict__ tau, float* __restrict__ cand_s,
                                                            int* __restrict__ cand_r, int64_t n_lists,
                                                            const uint32_t* __restrict__ mask, int mask_words) {
  constexpr int NKS = D / 32;   // 32-deep k-steps per tile
  constexpr int NST = D / kSK;  // stages per tile
  constexpr int KPS = kSK / 32;  // k-steps per stage (4)
  static_assert(D % kSK == 0, "D must be a multiple of 128");
  static_assert(KL <= 10, "threshold table holds 10 slots");
  __shared__ __attribute__((aligned(1024))) uint8_t lds[lds_bytes<KL>()];

  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int quad = lane >> 4;  // row group of the 16x16 accumulator (4 rows per row block)
  int range, grp;
  block_map(blockIdx.x, ranges, groups, paired != 0, range, grp);
  const int qg = grp * kQG;
  const int q = qg + w * kQW + (lane & 15);
  const int nt = range < ntiles ? (ntiles - range + ranges - 1) / ranges : 0;
  const int S = nt * NST;
  if (S == 0) return;  // (cannot happen with the host plan; whole workgroup exits together)
  const int lst = range * kListsPerBlock + quad;  // this lane's list id (per query)

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

  // ---- resident query fragments (B[k][col] of 16x16x32): lane holds col (lane & 15) = query
  // qg + 16 w + (lane & 15), k = 32 ks + 8 quad + j
  uint4 bq[NKS];
  {
    const uint16_t* qa = Qp + (int64_t)q * D + 8 * quad;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) bq[ks] = *(const uint4*)(qa + 32 * ks);
  }

  // ---- LDS-DMA pieces: piece i = w + 8 u of a stage fills slot bytes [1024 i, +1024) = rows
  // 4i..4i+3 (256 B each); lane -> (row 4i + quad, position lane & 15) <- source chunk
  // position ^ (row & 15)
  uint32_t laneoff[kGPW];  // byte offset of this lane's 16 B inside a [64 rows][D] tile (stage 0)
#pragma unroll
  for (int u = 0; u < kGPW; ++u) {
    const int r = 4 * (w + kWaves * u) + quad;
    laneoff[u] = (uint32_t)(r * D + (((lane & 15) ^ (r & 15)) * 8)) * 2u;
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  const int64_t tile_stride = (int64_t)ranges * kTM * D;  // elements between a block's tiles
  auto issue_piece = [&](int gi, int slot, int u) {
    gi = gi < S ? gi : S - 1;  // tail: duplicate loads into free slots keep the counted waits exact
    const int ti = gi / NST;
    const int si = gi - ti * NST;
    const uint16_t* tbase = X + (int64_t)range * kTM * D + ti * tile_stride + si * kSK;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + (uint32_t)(slot * kSlot) + (uint32_t)((w + kWaves * u) * 1024));
    // default cache policy, NOT non-temporal: the paired group re-reads these lines from L2.
    // Measured at the config-4 shard (profiles/r02g_cfg4_*): nt 8.42 ms, FETCH 1.75x algorithmic;
    // default 7.54 ms, FETCH 1.002x.
    bdma(make_rsrc(tbase), laneoff[u], dst);
  };
  const v4i32 tau_rsrc = make_rsrc(tau);
  auto issue_tau = [&]() {
    const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + kTauOff + w * 1024);
    bdma_sc1(tau_rsrc, (uint32_t)(qg * kTauW * 4 + tid * 16), dst);
  };

  uint32_t thr = 0u;  // pruning bound (orderable score; 0 = none)
  const uint32_t slot_voff = (uint32_t)(q * kTauW + lst % KL) * 4u;
  const uint8_t* const tq = lds + kTauOff + (w * kQW + (lane & 15)) * (kTauW * 4);
  int n_slow = 0;
  // A fragment of row block rb, k-step kk of a slot: row 16 rb + (lane & 15), chunk 4 kk + quad,
  // stored at position chunk ^ (row & 15) = chunk ^ (lane & 15); row blocks 4 KB apart
  const uint8_t* const frag_base = lds + (lane & 15) * kRowB;
  const int sw = lane & 15;
  struct Frag {
    uint4 a[kRB];
  };
  auto read_frag = [&](int slot, int kk) -> Frag {
    const uint8_t* p = frag_base + slot * kSlot + (((4 * kk + quad) ^ sw) << 4);
    Frag f;
#pragma unroll
    for (int rb = 0; rb < kRB; ++rb) f.a[rb] = *(const uint4*)(p + rb * 16 * kRowB);
    return f;
  };

  // Schedule (kernel 6's): stage h's pieces go out during stage h - 5, at k-steps 0 and 2, into the
  // slot freed at stage h - 6's barrier; fragments are read one k-step ahead of their MFMAs; the
  // stage-end wait + barrier sit at k-step KPS - 1.
  constexpr int PF = 1;
  constexpr int NF = PF + 1;
  constexpr int KB = KPS - PF;
  constexpr int AHEAD = kRing - 1;
  constexpr int YNG = (kRing - 2) * kGPW;  // ops younger than the next stage (8)
  static_assert((NST * KPS) % NF == 0, "fragment rotation must realign every tile");

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // resident queries landed before the counted stream
  issue_tau();
#pragma unroll
  for (int p = 0; p < AHEAD; ++p)
#pragma unroll
    for (int u = 0; u < kGPW; ++u) issue_piece(p, p, u);
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(YNG) : "memory");  // stage 0 landed: stages 1..4 younger
  asm volatile("s_barrier" ::: "memory");

  Frag fr[NF];
  fr[0] = read_frag(0, 0);
  v4f32x4 acc4[kRB];
  for (int it = 0; it < nt; ++it) {
    const int tile = range + it * ranges;
    const int gbase = it * NST;
    if (it >= 2 && tau_refresh_tile(it - 2)) thr = max(thr, tau_min<KL>(tq));
    // a threshold refresh issued after the barrier of the last stage of tile it_r is younger than
    // stage g+1's pieces iff it - young_depth(s) <= it_r <= it - 1 (see k_scan_mfma6.h)
    auto young = [&](int s) {
      const int dmax = (kRing - 3 + NST - s) / NST;
      bool y = false;
#pragma unroll
      for (int d = 1; d <= dmax; ++d) y = y || (it >= d && tau_refresh_tile(it - d));
      return y;
    };
#pragma unroll
    for (int s = 0; s < NST; ++s) {
      const int g = gbase + s;
      const int slot = g % kRing;
#pragma unroll
      for (int kk = 0; kk < KPS; ++kk) {
        if (kk % (KPS / kGPW) == 0) issue_piece(g + kRing - 1, (g + kRing - 1) % kRing, kk / (KPS / kGPW));
        if (kk == KB) {
          if (young(s))
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(YNG + kTauGPW) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(YNG) : "memory");
          asm volatile("s_barrier" ::: "memory");
          if (s == NST - 1 && tau_refresh_tile(it)) issue_tau();
        }
        const int ks = s * KPS + kk;
        fr[(ks + PF) % NF] = kk + PF < KPS ? read_frag(slot, kk + PF) : read_frag((g + 1) % kRing, kk + PF - KPS);
        const Frag& cur = fr[ks % NF];
        __builtin_amdgcn_sched_group_barrier(0x100, kRB, 0);  // the prefetch reads go out first
        __builtin_amdgcn_sched_group_barrier(0x008, kRB, 0);
#pragma unroll
        for (int rb = 0; rb < kRB; ++rb)
          acc4[rb] = ks == 0 ? mfma16<DT>(cur.a[rb], bq[ks], v4f32x4{}) : mfma16<DT>(cur.a[rb], bq[ks], acc4[rb]);
      }
    }

    // ---- epilogue: the lane's 16 rows of query lane & 15 into its list
    if constexpr ((MODE & kModeMask) != 0) {
      const uint32_t lo = mask[2 * tile];
      const uint32_t hi = 2 * tile + 1 < mask_words ? mask[2 * tile + 1] : 0u;
      mask_rowmap2(acc4, (((uint64_t)hi << 32) | lo) >> (4 * quad));
    }
    fold<KL, 2>(Acc4View{acc4}, Ls, thr, tile * kTM + 4 * quad, tau_rsrc, slot_voff, n_slow);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (q < nq) {
    // drop entries below the query's bound as it stands now (valid bound => exact)
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

#define RFX_K7_ARGS                                                                                      \
  X, Qp, nq, ntiles, ranges, groups, paired, tau, cs, cr, n_lists, mask, mask_words
// one translation unit per (dtype, D) instantiates the kernel for the lane-list sizes KL in {4, 10}
#define RFX_K7_INSTANTIATE(DTV, DV, NAME)                                                                 \
  int NAME(int kl, dim3 grid, hipStream_t st, const uint16_t* X, const uint16_t* Qp, int nq, int ntiles,     \
           int ranges, int groups, int paired, uint32_t* tau, float* cs, int* cr, int64_t n_lists,        \
           const uint32_t* mask, int mask_words) {                                                        \
    if (kl == 4 && mask)                                                                                \
      hipLaunchKernelGGL((scan_mfma7_kernel<DTV, 4, DV, kModeMask>), grid, dim3(512), 0, st, RFX_K7_ARGS);  \
    else if (kl == 10 && mask)                                                                          \
      hipLaunchKernelGGL((scan_mfma7_kernel<DTV, 10, DV, kModeMask>), grid, dim3(512), 0, st, RFX_K7_ARGS); \
    else if (kl == 4)                                                                                   \
      hipLaunchKernelGGL((scan_mfma7_kernel<DTV, 4, DV>), grid, dim3(512), 0, st, RFX_K7_ARGS);             \
    else if (kl == 10)                                                                                  \
      hipLaunchKernelGGL((scan_mfma7_kernel<DTV, 10, DV>), grid, dim3(512), 0, st, RFX_K7_ARGS);            \
    else                                                                                                \
      return -1;                                                                                        \
    return 0;                                                                                           \
  }

}  // namespace k7
}  // namespace rfx
