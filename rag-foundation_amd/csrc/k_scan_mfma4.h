// k_scan_mfma4.h — all-query-stationary batched scan: one workgroup holds 256 queries.
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551),
// BASELINE.json config 3 (10M×768 bf16, nq=256, k=10).  Fused scan + per-query top-k; the score
// matrix never reaches HBM.
//
// Why (measured, profiles/r01_v3_*): the 128-query kernel (k_scan_mfma3.h) needs two workgroups
// per row range at nq=256.  The second read of each tile was meant to hit L2, but rocprofv3
// FETCH_SIZE showed 24.3 GB of fabric reads per launch against 15.36 GB of corpus (1.58×), at
// 4.9 TB/s: the stream itself was the ceiling.  Here one workgroup covers all 256 queries, so every
// corpus byte crosses the fabric once, and each LDS fragment read feeds two MFMAs instead of one:
//   * workgroup = 4 waves (one per SIMD, 512 registers each) × 64 queries.  Each wave keeps its
//     64 queries' B-fragments for the whole of K resident: 2 × D/16 × 16 B per lane
//     (384 registers at d = 768, split by the compiler between VGPRs and AGPRs).
//   * tile = 32 corpus rows; a stage = 32 rows × 256 dims (16 KB) arrives by LDS-DMA
//     (global_load_lds_dwordx4, 4 wave-instructions per wave) into a 7-slot ring, 6 stages
//     (96 KB) in flight; one counted `s_waitcnt vmcnt(20)` + `s_barrier` per stage.
//   * LDS row image: 512 B per row; 16-B chunk c of row r sits at position c ^ (r & 15), so the
//     32-row ds_read_b128 fragment reads are bank-conflict free in all four lane groups (the
//     permutation rides on the LDS-DMA source address).
//   * per k-step and wave: 1 ds_read_b128 (rows × 16 k) → 2 × v_mfma_f32_32x32x16 (query blocks
//     0 and 1), accumulators 2 × 16 registers.
//   * top-k: lane l holds queries (l&31) and 32+(l&31) of its wave for 16 rows per tile; two
//     sorted lane lists of KL 64-bit keys (orderable score << 32 | ~row) kept in LDS (a register
//     holds each list's k-th best) and the cross-workgroup threshold τ (device atomicMax; any value read is a lower bound of the final k-th best, so the
//     result stays exact whatever τ a workgroup sees).
// Requires the index invariant of rfx_api.hip: rows [nrows, capacity) are NaN and capacity is a
// multiple of 128, so the ragged last tile needs no clamping or masking.
// Algorithmic bytes per tile: 32 * D * esize.
#pragma once
#include "rfx_device.h"
#include "rfx_kernels.h"

namespace rfx {
namespace k4 {

typedef __attribute__((ext_vector_type(8))) __bf16 v4bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 v4f16x8;
typedef __attribute__((ext_vector_type(16))) float v4f32x16;

template <int DT>
__device__ __forceinline__ v4f32x16 mfma(const uint4& a, const uint4& b, const v4f32x16& c) {
  if constexpr (DT == RFX_BF16)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v4bf16x8, a), __builtin_bit_cast(v4bf16x8, b),
                                                   c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v4f16x8, a), __builtin_bit_cast(v4f16x8, b), c,
                                                  0, 0, 0);
}

__device__ __forceinline__ uint32_t ord(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unord(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

constexpr int kTM = 32;                 // rows per tile
constexpr int kQW = 64;                 // queries per wave
constexpr int kQG = 256;                // queries per workgroup
constexpr int kSK = 256;                // dims per stage
constexpr int kSlot = kTM * kSK * 2;    // 16 KB
constexpr int kRing = 7;                // 6 stages (96 KB) in flight
constexpr int kGPW = kSlot / 1024 / 4;  // LDS-DMA wave-instructions per wave per stage (4)
constexpr int kTauOff = kRing * kSlot;  // 112 KB
constexpr int kListOff = kTauOff + 1024;  // thresholds of the 256 queries: one DMA wave-instruction
template <int KL>
constexpr int lds_bytes() { return kListOff + 4 * 2 * KL * 64 * 8; }  // + lane lists [wave][2][KL][64] u64

// LDS-DMA (global_load_lds_dwordx4) from inline asm; M0 = wave-uniform LDS destination.  The
// compiler cannot see a VMEM op writing LDS, so it does not drain the queue before LDS reads;
// the kernel orders them itself (counted vmcnt + s_barrier before a slot is read).
__device__ __forceinline__ void glds(const void* src, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_addr)
               : "memory", "m0");
}

template <int KL>
__device__ __forceinline__ void key_insert(uint64_t (&L)[KL], uint64_t key) {
#pragma unroll
  for (int i = 0; i < KL; ++i) {
    const bool b = key > L[i];
    const uint64_t t = L[i];
    L[i] = b ? key : t;
    key = b ? t : key;
  }
}

// Fold one 32×32 accumulator (16 rows of one query per lane) into the lane's list.  The list lives
// in LDS (entry i of this lane at Ls[i * 64], best first); the lane keeps only its k-th best in a
// register (`own`, orderable score).  Lists are read and written back only when some row of the
// tile reaches the threshold, which after the first tiles is rare.
template <int KL>
__device__ __forceinline__ void fold(const v4f32x16& acc, uint64_t* Ls, uint32_t& own, uint32_t shared_o,
                                     int rbase, uint32_t* __restrict__ tau_q, uint32_t& published) {
  float mx = max3f(acc[0], acc[1], acc[2]);
#pragma unroll
  for (int r = 3; r < 15; r += 2) mx = max3f(mx, acc[r], acc[r + 1]);
  mx = fmaxf(mx, acc[15]);  // NaN-ignoring max
  const uint32_t thr_o = own > shared_o ? own : shared_o;
  const float thr = thr_o ? unord(thr_o) : -__builtin_inff();
  if (mx >= thr) {
    uint64_t L[KL];
#pragma unroll
    for (int i = 0; i < KL; ++i) L[i] = Ls[i * 64];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float s = acc[r];
      if (s >= thr) {  // NaN (tombstoned rows, rows past the end) never passes
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        const uint64_t key = ((uint64_t)ord(s) << 32) | (uint32_t)(~(uint32_t)row);
        if (key > L[KL - 1]) key_insert<KL>(L, key);
      }
    }
#pragma unroll
    for (int i = 0; i < KL; ++i) Ls[i * 64] = L[i];
    own = (uint32_t)(L[KL - 1] >> 32);
    if (own > published && own > shared_o) {
      __hip_atomic_fetch_max(tau_q, own, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      published = own;
    }
  }
}

// Tile mapping: block b of B takes tiles b, b + B, b + 2B, ... so at any moment the whole grid
// streams one contiguous window of the store (even spread over HBM channels).
// MODE (profiling ablations, production = 0), bit flags: 1 = no top-k epilogue, 2 = no MFMA,
// 4 = contiguous row range per block (tiles b·T .. b·T + T - 1, T = tiles_per_block),
// 8 = no corpus stream after the prologue (MFMA + LDS reads on the first 7 stages, recycled).
template <int DT, int KL, int D, int MODE = 0>
__global__ __launch_bounds__(256, 1) void scan_mfma4_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Qp,
                                                            int nq, int tiles_per_block, int ntiles,
                                                            uint32_t* __restrict__ tau, float* __restrict__ cand_s,
                                                            int* __restrict__ cand_r, int64_t n_lists) {
  constexpr int NKS = D / 16;    // 16-deep MFMA k-steps
  constexpr int NST = D / kSK;   // stages per tile
  constexpr int KPS = kSK / 16;  // k-steps per stage (16)
  static_assert(D % kSK == 0, "D must be a multiple of 256");
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

  // ---- LDS-DMA pattern: wave-instruction i (0..15) fills slot bytes [1024 i, +1024) = rows 2i, 2i+1;
  // lane -> (row 2i + lane/32, position lane%32) <- chunk position ^ (row & 15); wave w issues
  // i = w + 4u, u = 0..3.
  int laneoff[kGPW];  // element offset of this lane's 16 B inside a [32 rows][D] tile (stage 0)
#pragma unroll
  for (int u = 0; u < kGPW; ++u) {
    const int r = 2 * (w + 4 * u) + half;
    laneoff[u] = r * D + ((l32 ^ (r & 15)) * 8);
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  // Stage gi -> LDS slot `slot`.  gi is clamped to the last stage so the tail of the stream issues
  // harmless duplicate loads into already-consumed slots: every stage issues exactly kGPW LDS-DMA
  // ops per wave, the counted waits stay exact, and the tile body has no branches.
  auto issue = [&](int gi, int slot) {
    gi = gi < S ? gi : S - 1;
    const int ti = gi / NST;
    const int si = gi - ti * NST;
    const uint16_t* tbase = X + (int64_t)(t0 + ti * tstep) * kTM * D + si * kSK;
    const uint32_t dst = lds_base + (uint32_t)(slot * kSlot) + (uint32_t)(w * 1024);
#pragma unroll
    for (int u = 0; u < kGPW; ++u) glds(tbase + laneoff[u], __builtin_amdgcn_readfirstlane(dst + u * 4096));
  };
  // shared thresholds of the 256 queries -> LDS (every wave, 64 lanes × 16 B = 1 KB; identical data)
  auto issue_tau = [&]() { glds(tau + qg + lane * 4, __builtin_amdgcn_readfirstlane(lds_base + kTauOff)); };

  uint64_t* const Ls0 = (uint64_t*)(lds + kListOff) + (w * 2 * KL) * 64 + lane;
  uint64_t* const Ls1 = Ls0 + KL * 64;
#pragma unroll
  for (int i = 0; i < KL; ++i) Ls0[i * 64] = Ls1[i * 64] = 0ull;
  uint32_t own0 = 0u, own1 = 0u, pub0 = 0u, pub1 = 0u;
  const uint8_t* frag_base = lds + l32 * 512;
  const int sw = l32 & 15;
  auto read_frag = [&](int slot, int kk) -> uint4 {
    return *(const uint4*)(frag_base + slot * kSlot + (((2 * kk + half) ^ sw) << 4));
  };

  issue_tau();
  // the resident query loads must land before the LDS-DMA stream starts counting
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int p = 0; p < kRing; ++p) issue(p, p);
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");  // stage 0 landed (stages 1..6 in flight)
  asm volatile("s_barrier" ::: "memory");

  uint4 fa = read_frag(0, 0), fb;
  v4f32x16 acc0, acc1;
  for (int it = 0; it < nt; ++it) {
    const int tile = t0 + it * tstep;
    const int gbase = it * NST;
#pragma unroll
    for (int s = 0; s < NST; ++s) {
      const int g = gbase + s;
      const int slot = g % kRing;
#pragma unroll
      for (int kk = 0; kk < KPS; ++kk) {
        if (kk == KPS - 1) {
          // stage g+1 landed for this wave (younger: stages g+2..g+6 = 20 ops); every wave has read
          // its last fragment of slot g (lgkmcnt(0) + barrier) -> stage g+7 may overwrite it
          asm volatile("s_waitcnt vmcnt(20) lgkmcnt(0)" ::: "memory");
          asm volatile("s_barrier" ::: "memory");
          if constexpr ((MODE & 8) == 0) {
            if (s == NST - 1) issue_tau();  // refreshed thresholds for the next tile's epilogue
            issue(g + kRing, slot);
          }
        }
        // prefetch the next k-step's fragment (crossing into stage g+1 at the last k-step)
        uint4& nxt = (kk & 1) ? fa : fb;
        nxt = kk < KPS - 1 ? read_frag(slot, kk + 1) : read_frag((g + 1) % kRing, 0);
        const uint4& cur = (kk & 1) ? fb : fa;
        const int ks = s * KPS + kk;
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
      const uint32_t* tl = (const uint32_t*)(lds + kTauOff) + w * kQW + l32;
      fold<KL>(acc0, Ls0, own0, tl[0], rbase, tau + q0, pub0);
      fold<KL>(acc1, Ls1, own1, tl[32], rbase, tau + q0 + 32, pub1);
    } else {
      if (acc0[0] == 12345.f && acc1[1] == 54321.f) Ls0[0] = 1;  // keep the MFMAs live
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const int64_t lst = (int64_t)range * 2 + half;
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
