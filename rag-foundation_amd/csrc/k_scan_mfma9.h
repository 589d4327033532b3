// k_scan_mfma9.h — the batched scan for f32 stores (v_mfma_f32_16x16x4_f32): one pass over the
// store for up to 128 queries per workgroup, where the VALU scan streams the store once per
// 8-query slice.
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551),
// micro-batched (rfx/batcher.py: concurrent chat requests, chat.py:40,496-521) on an f32 store
// (RFX_DTYPE=f32; BASELINE configs 1-2 are f32).  Fused scan + per-query top-k.
//
// Shape:
//   * f32 MFMA runs at 1/8 of the bf16 rate (32 cycles per 16x16x4), so at 128 queries the scan is
//     matrix-core bound, not HBM bound: one wave per SIMD (up to 512 registers) keeps 32 queries'
//     B-fragments for the whole of d resident (D / 2 VGPRs: 384 at d = 768) and issues 32
//     independent MFMAs per 16-dim k-step, enough to keep the matrix core busy without a second
//     wave.  Workgroup = 4 waves = 128 queries; query groups of a row range share an XCD (kernel 7).
//   * A k-step covers 16 dims: lane l reads dims 4 (l >> 4) .. + 3 of row l & 15 with one
//     ds_read_b128 and feeds them to four MFMAs (k = 4 each); the query fragments use the same
//     order of the reduction dimension.
//   * Stage = 64 rows × 64 dims (16 KB, 256 B per row) by LDS-DMA into a 4-slot ring; LDS image
//     16-B chunk c of row r at c ^ (r & 15) (kernel 7's image with f32 elements).
//   * Top-k: lane l holds, per query block, 16 rows of query l & 15 (ROWMAP 2); two lane lists per
//     lane (one per query block); cross-workgroup slot table and output as kernels 6-8.
// Requires the index invariant of rfx_api.hip: rows [nrows, capacity) are NaN and capacity is a
// multiple of 128, so the ragged last tile needs no clamping or masking.
// Algorithmic bytes per tile: 64 * D * 4.
#pragma once
#include "k_mfma_common.h"

namespace rfx {
namespace k9 {

using namespace mfc;

constexpr int kWaves = 4;
constexpr int kTM = 64;                   // rows per tile
constexpr int kRB = kTM / 16;             // 16-row MFMA blocks per tile
constexpr int kQW = 32;                   // queries per wave (2 query blocks)
constexpr int kQG = kWaves * kQW;         // 128 queries per workgroup
constexpr int kSK = 64;                   // dims per stage
constexpr int kRowB = kSK * 4;            // 256 B per row per stage
constexpr int kSlot = kTM * kRowB;        // 16 KB: 64 rows × 64 dims
constexpr int kRing = 4;                  // 4 slots, 3 stages (48 KB) in flight
constexpr int kGPW = kSlot / 1024 / kWaves;  // LDS-DMA pieces per wave per stage (4)
constexpr int kTauW = 16;
constexpr int kTauBytes = kQG * kTauW * 4;  // 8 KB
constexpr int kTauGPW = kTauBytes / 1024 / kWaves;  // 2
constexpr int kListsPerBlock = 4;         // lane lists per query per workgroup (the 4 lanes of a query)
constexpr int kTauOff = kRing * kSlot;
constexpr int kListOff = kTauOff + kTauBytes;
template <int KL>
constexpr int lds_bytes() { return kListOff + kWaves * 2 * KL * 64 * 8; }
static_assert(lds_bytes<10>() <= 163840, "LDS budget");
static_assert(kGPW == 4 && kTauGPW == 2, "DMA pieces per wave");

__device__ __forceinline__ bool tau_refresh_tile(int it) { return it < 2 || (it & 3) == 3; }

template <class V>
__device__ __forceinline__ void mask_rowmap2(V& a, uint64_t bits) {
#pragma unroll
  for (int r = 0; r < 16; ++r)
    if (!((bits >> ((r & 3) + 16 * (r >> 2))) & 1ull)) a[r >> 2][r & 3] = __builtin_nanf("");
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

__device__ __forceinline__ v4f32x4 mfma4(float a, float b, const v4f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int KL, int D, int MODE = 0>
__global__ __launch_bounds__(256, 1) void scan_mfma9_kernel(const float* __restrict__ X, const float* __restrict__ Qp,
                                                            int nq, int ntiles, int ranges, int groups, int paired,
                                                            uint32_t* __restrict__ tau, float* __restrict__ cand_s,
                                                            int* __restrict__ cand_r, int64_t n_lists,
                                                            const uint32_t* __restrict__ mask, int mask_words,
                                                            const uint32_t* __restrict__ gate) {
  // gate (the two-pass scan's fallback for f32 stores, k_screen.hip): run only when the screen asked for it
  if (gate && *gate == 0u) return;
  constexpr int NKS = D / 16;   // 16-dim k-steps per tile
  constexpr int NST = D / kSK;  // stages per tile
  constexpr int KPS = kSK / 16;  // k-steps per stage (4)
  static_assert(D % kSK == 0, "D must be a multiple of 64");
  static_assert(KPS % kGPW == 0 || kGPW % KPS == 0, "piece issue schedule");
  static_assert(KL <= 10, "threshold table holds 10 slots");
  __shared__ __attribute__((aligned(1024))) uint8_t lds[lds_bytes<KL>()];

  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int quad = lane >> 4;
  int range, grp;
  block_map(blockIdx.x, ranges, groups, paired != 0, range, grp);
  const int qg = grp * kQG;
  const int q0 = qg + w * kQW + (lane & 15);  // query of block 0; block 1 is q0 + 16
  const int nt = range < ntiles ? (ntiles - range + ranges - 1) / ranges : 0;
  const int S = nt * NST;
  if (S == 0) return;  // (cannot happen with the host plan; whole workgroup exits together)
  const int lst = range * kListsPerBlock + quad;

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
  __syncthreads();

  // ---- resident query fragments: block qb, lane holds query 16 qb + (lane & 15), dims
  // 16 ks + 4 quad .. + 3 (the same reduction order as the A reads)
  uint4 bq[NKS * 2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const float* qa = Qp + (int64_t)(q0 + 16 * qb) * D + 4 * quad;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) bq[2 * ks + qb] = *(const uint4*)(qa + 16 * ks);
  }

  // ---- LDS-DMA pieces: piece i = w + 4 u fills slot bytes [1024 i, +1024) = rows 4i..4i+3
  uint32_t laneoff[kGPW];
#pragma unroll
  for (int u = 0; u < kGPW; ++u) {
    const int r = 4 * (w + kWaves * u) + quad;
    laneoff[u] = (uint32_t)(r * D + (((lane & 15) ^ (r & 15)) * 4)) * 4u;
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  const int64_t tile_stride = (int64_t)ranges * kTM * D;
  auto issue_piece = [&](int gi, int slot, int u) {
    gi = gi < S ? gi : S - 1;
    const int ti = gi / NST;
    const int si = gi - ti * NST;
    const float* tbase = X + (int64_t)range * kTM * D + ti * tile_stride + si * kSK;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + (uint32_t)(slot * kSlot) + (uint32_t)((w + kWaves * u) * 1024));
    bdma(make_rsrc(tbase), laneoff[u], dst);
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

  uint32_t thr0 = 0u, thr1 = 0u;
  const uint32_t slot_voff0 = (uint32_t)(q0 * kTauW + lst % KL) * 4u;
  const uint32_t slot_voff1 = (uint32_t)((q0 + 16) * kTauW + lst % KL) * 4u;
  const uint8_t* const tq0 = lds + kTauOff + (w * kQW + (lane & 15)) * (kTauW * 4);
  const uint8_t* const tq1 = tq0 + 16 * kTauW * 4;
  int n_slow = 0;
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

  // Schedule: stage h's 4 pieces go out during stage h - 3 (one per k-step) into the slot freed at
  // stage h - 4's barrier; fragments one k-step ahead; the stage-end wait + barrier at the last
  // k-step of the stage.
  constexpr int AHEAD = kRing - 1;
  constexpr int YNG = (kRing - 2) * kGPW;  // ops younger than the next stage (8)

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
  fr[0] = read_frag(0, 0);
  v4f32x4 acc[2][kRB];  // [qb][rb]
  for (int it = 0; it < nt; ++it) {
    const int tile = range + it * ranges;
    const int gbase = it * NST;
    if (it >= 2 && tau_refresh_tile(it - 2)) {
      thr0 = max(thr0, tau_min<KL>(tq0));
      thr1 = max(thr1, tau_min<KL>(tq1));
    }
    auto young = [&](int s) {
      const int dmax = (kRing - 3 + NST - s) / NST;
      bool y = false;
#pragma unroll
      for (int d = 1; d <= dmax; ++d) y = y || (it >= d && tau_refresh_tile(it - d));
      return y;
    };
#pragma unroll
    for (int s = 0; s < NST; ++s) {  // unrolled: the resident fragments are statically indexed
      const int g = gbase + s;
      const int slot = g % kRing;
#pragma unroll
      for (int kk = 0; kk < KPS; ++kk) {
        issue_piece(g + kRing - 1, (g + kRing - 1) % kRing, kk);
        if (kk == KPS - 1) {
          if (young(s))
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(YNG + kTauGPW) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(YNG) : "memory");
          asm volatile("s_barrier" ::: "memory");
          if (s == NST - 1 && tau_refresh_tile(it)) issue_tau();
        }
        fr[(kk + 1) & 1] = kk + 1 < KPS ? read_frag(slot, kk + 1) : read_frag((g + 1) % kRing, 0);
        const Frag& cur = fr[kk & 1];
        const int ks = s * KPS + kk;
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int rb = 0; rb < kRB; ++rb)
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) {
              const float a = __uint_as_float((&cur.a[rb].x)[e]);
              const float b = __uint_as_float((&bq[2 * ks + qb].x)[e]);
              acc[qb][rb] = (ks == 0 && e == 0) ? mfma4(a, b, v4f32x4{}) : mfma4(a, b, acc[qb][rb]);
            }
      }
    }

    // ---- epilogue: per query block, the lane's 16 rows of query q0 + 16 qb into its list
    const int rbase = tile * kTM + 4 * quad;
    if constexpr ((MODE & kModeMask) != 0) {
      const uint32_t lo = mask[2 * tile];
      const uint32_t hi = 2 * tile + 1 < mask_words ? mask[2 * tile + 1] : 0u;
      const uint64_t bits = (((uint64_t)hi << 32) | lo) >> (4 * quad);
      mask_rowmap2(acc[0], bits);
      mask_rowmap2(acc[1], bits);
    }
    fold<KL, 2>(Acc4View{acc[0]}, Ls0, thr0, rbase, tau_rsrc, slot_voff0, n_slow);
    fold<KL, 2>(Acc4View{acc[1]}, Ls1, thr1, rbase, tau_rsrc, slot_voff1, n_slow);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int q = q0 + 16 * qb;
    if (q < nq) {
      uint32_t m = 0xffffffffu;
#pragma unroll
      for (int j = 0; j < KL; ++j)
        m = min(m, __hip_atomic_load(tau + (int64_t)q * kTauW + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      const uint32_t fin = max(qb ? thr1 : thr0, m);
      const uint64_t* L = qb ? Ls1 : Ls0;
      const int64_t o = ((int64_t)q * n_lists + lst) * KL;
#pragma unroll
      for (int i = 0; i < KL; ++i) {
        const uint64_t key = L[i * 64];
        const bool keep = key && (uint32_t)(key >> 32) >= fin;
        cand_s[o + i] = keep ? unord((uint32_t)(key >> 32)) : -__builtin_inff();
        cand_r[o + i] = keep ? (int)(~(uint32_t)key) : kEmptyRow;
      }
    }
  }
}

#define RFX_K9_ARGS X, Qp, nq, ntiles, ranges, groups, paired, tau, cs, cr, n_lists, mask, mask_words, gate
#define RFX_K9_INSTANTIATE(DV, NAME)                                                                      \
  int NAME(int kl, dim3 grid, hipStream_t st, const float* X, const float* Qp, int nq, int ntiles,          \
           int ranges, int groups, int paired, uint32_t* tau, float* cs, int* cr, int64_t n_lists,        \
           const uint32_t* mask, int mask_words, const uint32_t* gate) {                                   \
    if (kl == 4 && mask)                                                                                \
      hipLaunchKernelGGL((scan_mfma9_kernel<4, DV, kModeMask>), grid, dim3(256), 0, st, RFX_K9_ARGS);       \
    else if (kl == 10 && mask)                                                                          \
      hipLaunchKernelGGL((scan_mfma9_kernel<10, DV, kModeMask>), grid, dim3(256), 0, st, RFX_K9_ARGS);      \
    else if (kl == 4)                                                                                   \
      hipLaunchKernelGGL((scan_mfma9_kernel<4, DV>), grid, dim3(256), 0, st, RFX_K9_ARGS);                  \
    else if (kl == 10)                                                                                  \
      hipLaunchKernelGGL((scan_mfma9_kernel<10, DV>), grid, dim3(256), 0, st, RFX_K9_ARGS);                 \
    else                                                                                                \
      return -1;                                                                                        \
    return 0;                                                                                           \
  }

}  // namespace k9
}  // namespace rfx
