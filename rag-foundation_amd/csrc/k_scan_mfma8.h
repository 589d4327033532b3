// k_scan_mfma8.h — the d = 1024 batched scan with k-split wave pairs (BASELINE config 4: 100M×1024
// f16 over 8 GPUs, a 12.5M-row shard per GPU, nq 256, k 10).
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551).
// Fused scan + per-query top-k; the score matrix never reaches HBM.
//
// Why: kernel 7 keeps 16 queries per wave so that two waves per SIMD fit at
// d = 1024, but then every A-fragment read from LDS feeds one MFMA: the LDS array (reads plus the
// LDS-DMA writes) is busier than the matrix cores (7.5 ms per 12.5M-row launch, 0.87 PF/s against
// kernel 6's 1.08).  Here the two waves of a pair hold the SAME 32 queries, each for half of the
// k-steps (wave kh takes k-steps 2 kh, 2 kh + 1 of every 128-dim stage): 32 queries × 512 dims of
// B-fragments = 128 VGPRs, two waves per SIMD, and every A-fragment read feeds two MFMAs, as in
// kernel 6.  At the end of a 64-row tile the pair swaps partial sums through LDS (wave kh keeps
// rows 32 kh .. 32 kh + 31), adds them, and runs kernel 6's epilogue on 32 rows × 32 queries.
//   * Workgroup = 4 pairs × 32 queries = 128 queries; XCD-paired query groups, 64-row tiles,
//     16-KB stages (64 rows × 128 dims, LDS image c ^ (r & 15)), default-cached corpus DMA: as
//     kernel 7 (k_scan_mfma7.h), with a 4-slot ring (3 stages = 48 KB in flight; 5 slots measured
//     2 % slower, 3 slots 4 % slower) beside the 32-KB partial-sum exchange.
//   * Scores are a sum of two f32 partial dot products (each over 512 dims), within the parity
//     tolerance of the f64 oracle like every other accumulation order.
// Requires the index invariant of rfx_api.hip: rows [nrows, capacity) are NaN and capacity is a
// multiple of 128, so the ragged last tile needs no clamping or masking.
// Algorithmic bytes per tile: 64 * D * esize.
#pragma once
#include <type_traits>

#include "k_mfma_common.h"

namespace rfx {
namespace k8 {

using namespace mfc;

constexpr int kWaves = 8;
constexpr int kPairs = 4;
constexpr int kTM = 64;                   // rows per tile
constexpr int kRB = kTM / 16;             // 16-row MFMA blocks per tile
constexpr int kQW = 32;                   // queries per wave (= per pair)
constexpr int kQG = kPairs * kQW;         // 128 queries per workgroup
constexpr int kSK = 128;                  // dims per stage
constexpr int kRowB = kSK * 2;            // 256 B per row per stage
constexpr int kSlot = kTM * kRowB;        // 16 KB: 64 rows × 128 dims
// Ring depth, measured by side builds (-DRFX_K8_RING=N, tools/gpu_k8ring.sh, config-4 shard):
// 5 slots 7.17-7.20 ms, 4 slots 7.00-7.03 ms, 3 slots 7.45 ms per launch.
#ifndef RFX_K8_RING
#define RFX_K8_RING 4
#endif
constexpr int kRing = RFX_K8_RING;        // 4 slots, 3 stages (48 KB) in flight
constexpr int kGPW = 2;                   // LDS-DMA pieces per wave per stage (16 KB / 1 KB / 8 waves)
constexpr int kTauW = 16;                 // u32 per query in the threshold table (KL <= 10 used)
constexpr int kTauBytes = kQG * kTauW * 4;  // 8 KB: 8 DMA pieces, 1 per wave
constexpr int kTauGPW = kTauBytes / 1024 / kWaves;
constexpr int kListsPerBlock = 4;         // lists per query per workgroup: (kh, half-wave)
constexpr int kXBytes = kWaves * 16 * 64 * 4;  // partial-sum exchange: 16 floats per lane per wave
constexpr int kTauOff = kRing * kSlot;
constexpr int kXOff = kTauOff + kTauBytes;
constexpr int kListOff = kXOff + kXBytes;
template <int KL>
constexpr int lds_bytes() { return kListOff + kWaves * KL * 64 * 8; }
static_assert(lds_bytes<10>() <= 163840, "LDS budget");
static_assert(kSlot / 1024 == kWaves * kGPW && kTauGPW == 1, "DMA pieces per wave");

__device__ __forceinline__ bool tau_refresh_tile(int it) { return it < 2 || (it & 3) == 3; }

// Metadata filter on the pair-swapped 32-row layout (kernel 6's): value r of the lane is row
// (r & 7) + 16 (r >> 3) of its 32-row half, bits pre-shifted by 8 * half.
template <class V>
__device__ __forceinline__ void mask_rowmap1(V& a, uint32_t bits) {
#pragma unroll
  for (int r = 0; r < 16; ++r)
    if (!((bits >> ((r & 7) + 16 * (r >> 3))) & 1u)) a[r >> 2][r & 3] = __builtin_nanf("");
}

constexpr int kModeMask = 2097152;

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
__global__ __launch_bounds__(512, 1) void scan_mfma8_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Qp,
                                                            int nq, int ntiles, int ranges, int groups, int paired,
                                                            uint32_t* __restrict__ tau, float* __restrict__ cand_s,
                                                            int* __restrict__ cand_r, int64_t n_lists,
                                                            const uint32_t* __restrict__ mask, int mask_words,
                                                            const uint32_t* __restrict__ gate) {
  if (gate && *gate == 0u) return;  // the two-pass scan's gated fallback (k_screen.hip)
  constexpr int NST = D / kSK;   // stages per tile (8)
  constexpr int KPS = kSK / 32;  // k-steps per stage (4); a wave runs 2 of them
  constexpr int KW = KPS / 2;    // k-steps per stage per wave
  static_assert(D % kSK == 0 && KW == kGPW, "D must be a multiple of 128");
  static_assert(KL <= 10, "threshold table holds 10 slots");
  __shared__ __attribute__((aligned(1024))) uint8_t lds[lds_bytes<KL>()];

  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int quad = lane >> 4, half = lane >> 5;
  const int pr = w & 3, kh = w >> 2;  // pair (32 queries) and k-half of this wave
  int range, grp;
  block_map(blockIdx.x, ranges, groups, paired != 0, range, grp);
  const int qg = grp * kQG;
  // the lane's query after the epilogue's pair swap (kernel 6): odd 16-lane rows hold query block 1
  const int q = qg + pr * kQW + 16 * (quad & 1) + (lane & 15);
  const int nt = range < ntiles ? (ntiles - range + ranges - 1) / ranges : 0;
  const int S = nt * NST;
  if (S == 0) return;  // (cannot happen with the host plan; whole workgroup exits together)
  const int lst = range * kListsPerBlock + kh * 2 + half;  // this lane's list id (per query)

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

  // ---- resident query fragments: query block qb, lane holds col 16 qb + (lane & 15); the wave's
  // k-steps are ks = 4 s + 2 kh + j (j < 2), k = 32 ks + 8 quad + e
  uint4 bq[NST * KW * 2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const uint16_t* qa = Qp + (int64_t)(qg + pr * kQW + 16 * qb + (lane & 15)) * D + 8 * quad + 32 * KW * kh;
#pragma unroll
    for (int s = 0; s < NST; ++s)
#pragma unroll
      for (int j = 0; j < KW; ++j) bq[(s * KW + j) * 2 + qb] = *(const uint4*)(qa + 32 * (KPS * s + j));
  }

  uint32_t laneoff[kGPW];
#pragma unroll
  for (int u = 0; u < kGPW; ++u) {
    const int r = 4 * (w + kWaves * u) + quad;
    laneoff[u] = (uint32_t)(r * D + (((lane & 15) ^ (r & 15)) * 8)) * 2u;
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  const int64_t tile_stride = (int64_t)ranges * kTM * D;
  auto issue_piece = [&](int gi, int slot, int u) {
    gi = gi < S ? gi : S - 1;  // tail: duplicate loads into free slots keep the counted waits exact
    const int ti = gi / NST;
    const int si = gi - ti * NST;
    const uint16_t* tbase = X + (int64_t)range * kTM * D + ti * tile_stride + si * kSK;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + (uint32_t)(slot * kSlot) + (uint32_t)((w + kWaves * u) * 1024));
    bdma(make_rsrc(tbase), laneoff[u], dst);  // default policy: the partner group re-reads from L2
  };
  const v4i32 tau_rsrc = make_rsrc(tau);
  auto issue_tau = [&]() {
    const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + kTauOff + w * 1024);
    bdma_sc1(tau_rsrc, (uint32_t)(qg * kTauW * 4 + tid * 16), dst);
  };

  uint32_t thr = 0u;
  const uint32_t slot_voff = (uint32_t)(q * kTauW + lst % KL) * 4u;
  const uint8_t* const tq = lds + kTauOff + (pr * kQW + (lane & 15) + 16 * (quad & 1)) * (kTauW * 4);
  int n_slow = 0;
  const uint8_t* const frag_base = lds + (lane & 15) * kRowB;
  const int sw = lane & 15;
  struct Frag {
    uint4 a[kRB];
  };
  // A-fragments of k-step kk of a slot: row 16 rb + (lane & 15), chunk 4 kk + quad
  auto read_frag = [&](int slot, int kk) -> Frag {
    const uint8_t* p = frag_base + slot * kSlot + (((4 * kk + quad) ^ sw) << 4);
    Frag f;
#pragma unroll
    for (int rb = 0; rb < kRB; ++rb) f.a[rb] = *(const uint4*)(p + rb * 16 * kRowB);
    return f;
  };

  // Schedule: stage h's pieces go out during stage h - (kRing - 1) (one per k-step of the wave) into
  // the slot freed at stage h - kRing's barrier; fragments are read one k-step ahead of their MFMAs; the stage-end
  // wait + barrier sit at the wave's last k-step of the stage.
  constexpr int AHEAD = kRing - 1;
  constexpr int YNG = (kRing - 2) * kGPW;  // ops younger than the next stage (4)
  float* const xw = (float*)(lds + kXOff);  // exchange: [wave][16][64] f32

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  launder(bq);  // hipcc stops tracking the fragments' loads (k_mfma_common.h)
  issue_tau();
#pragma unroll
  for (int p = 0; p < AHEAD; ++p)
#pragma unroll
    for (int u = 0; u < kGPW; ++u) issue_piece(p, p, u);
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(YNG) : "memory");
  asm volatile("s_barrier" ::: "memory");

  Frag fr[2];
  fr[0] = read_frag(0, 2 * kh);
  v4f32x4 acc[kRB * 2];  // [rb * 2 + qb]
  for (int it = 0; it < nt; ++it) {
    const int tile = range + it * ranges;
    const int gbase = it * NST;
    if (it >= 2 && tau_refresh_tile(it - 2)) thr = max(thr, tau_min<KL>(tq));
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
      for (int j = 0; j < KW; ++j) {
        issue_piece(g + kRing - 1, (g + kRing - 1) % kRing, j);
        if (j == KW - 1) {
          if (young(s))
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(YNG + kTauGPW) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(YNG) : "memory");
          asm volatile("s_barrier" ::: "memory");
          if (s == NST - 1 && tau_refresh_tile(it)) issue_tau();
        }
        const int ks = s * KW + j;  // the wave's k-step index within the tile
        fr[(ks + 1) & 1] = j + 1 < KW ? read_frag(slot, 2 * kh + j + 1) : read_frag((g + 1) % kRing, 2 * kh);
        const Frag& cur = fr[ks & 1];
        __builtin_amdgcn_sched_group_barrier(0x100, kRB, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * kRB, 0);
#pragma unroll
        for (int rb = 0; rb < kRB; ++rb)
#pragma unroll
          for (int qb = 0; qb < 2; ++qb)
            acc[rb * 2 + qb] = ks == 0 ? mfma16<DT>(cur.a[rb], bq[2 * ks + qb], v4f32x4{})
                                       : mfma16<DT>(cur.a[rb], bq[2 * ks + qb], acc[rb * 2 + qb]);
      }
    }

    // ---- partial-sum exchange: wave kh keeps row blocks 2 kh, 2 kh + 1 (acc[4 kh .. 4 kh + 3] in
    // kernel 6's [rb * 2 + qb] order) and hands the other two to its partner (wave w ^ 4).  The
    // previous tile's reads of this buffer finished before this tile's first stage barrier, so the
    // writes need no barrier before them.  kh is wave-uniform: one statically indexed body per half.
    auto epilogue = [&](auto khc) {
      constexpr int KH = decltype(khc)::value;
      v4f32x4* mine = (v4f32x4*)xw + w * (4 * 64) + lane;  // [wave][v][lane], 16 B per lane
#pragma unroll
      for (int v = 0; v < 4; ++v) mine[v * 64] = acc[4 * (1 - KH) + v];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      asm volatile("s_barrier" ::: "memory");
      v4f32x4(&own)[4] = *reinterpret_cast<v4f32x4(*)[4]>(&acc[4 * KH]);
      const v4f32x4* other = (const v4f32x4*)xw + (w ^ 4) * (4 * 64) + lane;
#pragma unroll
      for (int v = 0; v < 4; ++v) own[v] += other[v * 64];
      // kernel 6's epilogue: pair swap, then the lane's 16 rows of one query into its list
#pragma unroll
      for (int rr = 0; rr < 2; ++rr)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(own[2 * rr][i]),
                                                          __float_as_uint(own[2 * rr + 1][i]), false, false);
          own[2 * rr][i] = __uint_as_float(r[0]);
          own[2 * rr + 1][i] = __uint_as_float(r[1]);
        }
      if constexpr ((MODE & kModeMask) != 0) {
        const int mw = 2 * tile + KH;  // the last tile's second word may lie past the mask's end
        mask_rowmap1(own, (mw < mask_words ? mask[mw] : 0u) >> (8 * half));
      }
      fold<KL, 1>(Acc4View{own}, Ls, thr, tile * kTM + 32 * KH + 8 * half, tau_rsrc, slot_voff, n_slow);
    };
    if (kh == 0)
      epilogue(std::integral_constant<int, 0>{});
    else
      epilogue(std::integral_constant<int, 1>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (q < nq) {
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

#define RFX_K8_ARGS X, Qp, nq, ntiles, ranges, groups, paired, tau, cs, cr, n_lists, mask, mask_words, gate
#define RFX_K8_INSTANTIATE(DTV, DV, NAME)                                                                 \
  int NAME(int kl, dim3 grid, hipStream_t st, const uint16_t* X, const uint16_t* Qp, int nq, int ntiles,     \
           int ranges, int groups, int paired, uint32_t* tau, float* cs, int* cr, int64_t n_lists,        \
           const uint32_t* mask, int mask_words, const uint32_t* gate) {                                  \
    if (kl == 4 && mask)                                                                                \
      hipLaunchKernelGGL((scan_mfma8_kernel<DTV, 4, DV, kModeMask>), grid, dim3(512), 0, st, RFX_K8_ARGS);  \
    else if (kl == 10 && mask)                                                                          \
      hipLaunchKernelGGL((scan_mfma8_kernel<DTV, 10, DV, kModeMask>), grid, dim3(512), 0, st, RFX_K8_ARGS); \
    else if (kl == 4)                                                                                   \
      hipLaunchKernelGGL((scan_mfma8_kernel<DTV, 4, DV>), grid, dim3(512), 0, st, RFX_K8_ARGS);             \
    else if (kl == 10)                                                                                  \
      hipLaunchKernelGGL((scan_mfma8_kernel<DTV, 10, DV>), grid, dim3(512), 0, st, RFX_K8_ARGS);            \
    else                                                                                                \
      return -1;                                                                                        \
    return 0;                                                                                           \
  }

}  // namespace k8
}  // namespace rfx
