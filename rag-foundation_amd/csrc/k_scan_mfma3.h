// k_scan_mfma3.hip — query-stationary batched scan (d = 768 / 1024, bf16 / f16).
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551),
// BASELINE.json config 3 (10M×768 bf16, nq=256, k=10).  Fused scan + per-query top-k; the score
// matrix never reaches HBM.
//
// Why this shape (measured on MI355X): re-streaming the query block
// through LDS every K-stage doubled the LDS-DMA traffic and capped the corpus stream at
// ~3.3 TB/s.  Here every wave keeps its 32 queries' MFMA B-fragments for the WHOLE of K in
// VGPRs (D/4 registers: 192 at d=768), so only corpus rows move:
//   * workgroup = 4 waves (one per SIMD, up to 512 VGPRs each) = 128 queries ("query group");
//     nq = 256 is served by two groups that sweep the same row range at the same time (blocks x
//     and x + R share an XCD under round-robin dispatch, so the second read is an L2/MALL hit;
//     placement only affects speed, never results).
//   * tile = 128 corpus rows; per 64-wide K-stage a 16 KB slice arrives by LDS-DMA
//     (global_load_lds_dwordx4, 4 wave-instructions per wave) into an 8-slot ring (7 stages =
//     112 KB in flight); one counted `s_waitcnt vmcnt(24)` + raw `s_barrier` per stage.
//   * LDS row image: 128 B = 8 slots of 16 B, chunk c of row r in slot c ^ ((r>>1)&7):
//     conflict-free 32-row ds_read_b128 fragment reads (the permutation rides on the LDS-DMA
//     source address).  Each wave computes 128 rows × 32 queries = 4 sub-tiles of
//     v_mfma_f32_32x32x16_{bf16,f16} (64 accumulator VGPRs); K is fully unrolled per tile so
//     the resident B-fragments are statically indexed.
//   * top-k: lane l holds query (l&31) for 64 rows per tile; sorted lane list of KL 64-bit keys
//     (orderable score << 32 | ~row) + the cross-workgroup threshold of k_scan_mfma2.hip
//     (device atomicMax; any value read is a lower bound of the final k-th best: exact).
// Requires the index invariant of rfx_api.hip: rows [nrows, capacity) are NaN and capacity is a
// multiple of 128, so the ragged last tile needs no clamping or masking.
// Algorithmic bytes per tile: 128 * D * 2.
#pragma once
#include "rfx_device.h"
#include "rfx_kernels.h"

namespace rfx {
namespace k3 {

typedef __attribute__((ext_vector_type(8))) __bf16 v3bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 v3f16x8;
typedef __attribute__((ext_vector_type(16))) float v3f32x16;

template <int DT>
__device__ __forceinline__ v3f32x16 mfma3(const uint4& a, const uint4& b, const v3f32x16& c) {
  if constexpr (DT == RFX_BF16)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v3bf16x8, a), __builtin_bit_cast(v3bf16x8, b),
                                                   c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v3f16x8, a), __builtin_bit_cast(v3f16x8, b), c,
                                                  0, 0, 0);
}

__device__ __forceinline__ uint32_t ord3(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unord3(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
// NaN-ignoring 3-way max as plain fmaxf (hipcc emits v_max3_f32 and pads the MFMA->VALU hazard an
// inline-asm reader of an accumulator would not get).
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

constexpr int k3M = 128;        // rows per tile
constexpr int k3QW = 32;        // queries per wave
constexpr int k3QG = 128;       // queries per workgroup (4 waves)
constexpr int k3BK = 64;        // K per stage
constexpr int k3Slot = k3M * k3BK * 2;   // 16 KB
constexpr int k3Ring = 8;                  // 7 stages (112 KB) in flight
constexpr int k3GPW = k3Slot / 1024 / 4;   // LDS-DMA wave-instructions per wave per stage (4)
constexpr int k3TauOff = k3Ring * k3Slot;  // 128 KB
constexpr int k3Lds = k3TauOff + 1024;      // thresholds: 256 slots (128 used), one DMA wave-instruction

// LDS-DMA (global_load_lds_dwordx4) issued from inline asm; M0 = wave-uniform LDS destination.
__device__ __forceinline__ void glds_asm(const void* src, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_addr)
               : "memory", "m0");
}

template <int KL>
__device__ __forceinline__ void key_insert3(uint64_t (&L)[KL], uint64_t key) {
#pragma unroll
  for (int i = 0; i < KL; ++i) {
    const bool b = key > L[i];
    const uint64_t t = L[i];
    L[i] = b ? key : t;
    key = b ? t : key;
  }
}

template <int DT, int KL, int D>
__global__ __launch_bounds__(256, 1) void scan_mfma3_kernel(const uint16_t* __restrict__ X, int nrows,
                                                            const uint16_t* __restrict__ Qp, int nq,
                                                            int tiles_per_block, int ntiles, uint32_t* __restrict__ tau,
                                                            float* __restrict__ cand_s, int* __restrict__ cand_r,
                                                            int64_t n_lists, const uint32_t* __restrict__ mask) {
  constexpr int NKS = D / 16;      // 16-deep MFMA k-steps
  constexpr int NST = D / k3BK;    // stages per tile
  __shared__ __attribute__((aligned(1024))) uint8_t lds[k3Lds];

  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int half = lane >> 5, l32 = lane & 31;
  const int range = blockIdx.x;
  const int qg = blockIdx.y * k3QG;
  const int q = qg + w * k3QW + l32;  // this lane's query
  const int t0 = range * tiles_per_block;
  const int t1 = min(ntiles, t0 + tiles_per_block);
  const int S = t1 > t0 ? (t1 - t0) * NST : 0;

  // ---- resident query fragments: B[k][col] of 32x32x16, lane holds k = 16 ks + 8 half + j ----
  uint4 bq[NKS];
  {
    const uint16_t* qrow = Qp + (int64_t)q * D + 8 * half;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) bq[ks] = *(const uint4*)(qrow + 16 * ks);
  }

  // ---- LDS-DMA pattern: wave-instruction i (0..15) fills slot bytes [1024 i, +1024) = rows
  // 8i..8i+7; lane -> (row 8i + lane/8, slot lane%8) <- chunk slot ^ ((row>>1)&7); wave w issues
  // i = w + 4u, u = 0..3.  Issued through inline asm: the compiler then cannot see a VMEM op
  // writing LDS, so it no longer drains the whole queue (s_waitcnt vmcnt(0)) before every LDS
  // read; ordering is ours: counted vmcnt + s_barrier before a slot is read.
  int rowoff[k3GPW], choff[k3GPW];
#pragma unroll
  for (int u = 0; u < k3GPW; ++u) {
    const int r = 8 * (w + 4 * u) + (lane >> 3);
    rowoff[u] = r;
    choff[u] = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  int laneoff[k3GPW];  // element offset of this lane's 16 B inside a [128 rows][D] tile
#pragma unroll
  for (int u = 0; u < k3GPW; ++u) laneoff[u] = rowoff[u] * D + choff[u];
  // Stage gi -> LDS slot `slot`.  gi is clamped to the last stage so the tail of the stream issues
  // harmless duplicate loads into already-consumed slots: every stage issues exactly k3GPW
  // LDS-DMA ops per wave, the counted waits stay exact, and the tile body has no branches.
  auto issue = [&](int gi, int slot) {
    gi = gi < S ? gi : S - 1;
    const int ti = gi / NST;
    const int si = gi - ti * NST;
    const uint16_t* tbase = X + (int64_t)(t0 + ti) * k3M * D + si * k3BK;
    const uint32_t dst = lds_base + (uint32_t)(slot * k3Slot) + (uint32_t)(w * 1024);
#pragma unroll
    for (int u = 0; u < k3GPW; ++u) glds_asm(tbase + laneoff[u], __builtin_amdgcn_readfirstlane(dst + u * 4096));
  };
  // shared thresholds of this query group -> LDS (every wave, 64 lanes x 16 B = 1 KB; identical data)
  auto issue_tau = [&]() { glds_asm(tau + qg + lane * 4, __builtin_amdgcn_readfirstlane(lds_base + k3TauOff)); };

  uint64_t L[KL];
#pragma unroll
  for (int i = 0; i < KL; ++i) L[i] = 0ull;
  uint32_t published = 0u;
  const int sw = (l32 >> 1) & 7;
  const int a_base = l32 * 128;

  // fragment reads of k-step kk from LDS slot `slot`: 4 row sub-tiles of 32 rows, 16 B per lane
  auto read_frags = [&](int slot, int kk, uint4 (&f)[4]) {
    const uint8_t* sa = lds + slot * k3Slot + a_base + (((2 * kk + half) ^ sw) << 4);
#pragma unroll
    for (int m = 0; m < 4; ++m) f[m] = *(const uint4*)(sa + m * 32 * 128);
  };

  if (S == 0) return;  // (cannot happen with the host plan; whole workgroup exits together)
  issue_tau();
  // the resident query loads must land before the LDS-DMA stream starts counting
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < NKS; ++i) {  // hipcc stops tracking the fragments' loads (mfc::launder, k_mfma_common.h)
    typedef int v4i __attribute__((ext_vector_type(4)));
    v4i t = __builtin_bit_cast(v4i, bq[i]);
    asm volatile("" : "+v"(t));
    bq[i] = __builtin_bit_cast(uint4, t);
  }
#pragma unroll
  for (int p = 0; p < k3Ring; ++p) issue(p, p);
  asm volatile("s_waitcnt vmcnt(28)" ::: "memory");  // stage 0 landed (stages 1..7 in flight)
  asm volatile("s_barrier" ::: "memory");

  uint4 fa[4], fb[4];
  read_frags(0, 0, fa);

  v3f32x16 acc[4];
  for (int tile = t0; tile < t1; ++tile) {
    const int gbase = (tile - t0) * NST;
#pragma unroll
    for (int s = 0; s < NST; ++s) {
      const int g = gbase + s;
      const int slot = g % k3Ring;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        if (kk == 3) {
          // stage g+1 landed for this wave (younger: stages g+2..g+7 = 24 ops); all waves are
          // done reading slot g%8 (its k-step 3 fragments were read above) -> stage g+8 may land
          asm volatile("s_waitcnt vmcnt(24) lgkmcnt(0)" ::: "memory");
          asm volatile("s_barrier" ::: "memory");
          if (s == NST - 1) issue_tau();  // refreshed thresholds for the next tile's epilogue
          issue(g + k3Ring, slot);
        }
        // prefetch the next k-step's fragments (crossing into stage g+1 at kk == 3)
        if (kk < 3)
          read_frags(slot, kk + 1, (kk & 1) ? fa : fb);
        else
          read_frags((g + 1) % k3Ring, 0, (kk & 1) ? fa : fb);
        uint4 (&cur)[4] = (kk & 1) ? fb : fa;
#ifndef RFX_K3_NO_SGB
        // pin the interleave: this k-step's 4 prefetch reads go out ahead of its 4 MFMAs
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
#endif
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          if (s == 0 && kk == 0)
            acc[m] = mfma3<DT>(cur[m], bq[4 * s + kk], v3f32x16{});
          else
            acc[m] = mfma3<DT>(cur[m], bq[4 * s + kk], acc[m]);
        }
      }
    }

    // ---- epilogue: fold this tile's 256 rows into the lane list ----
    const int rbase = tile * k3M + 4 * half;
    if (mask) {  // metadata filter (uniform branch): excluded rows -> NaN
#pragma unroll
      for (int m = 0; m < 4; ++m) mask_acc16(acc[m], acc_row_bits(mask, rbase + m * 32, nrows));
    }
    float mx = -__builtin_inff();
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < 16; r += 2) mx = max3f(mx, acc[m][r], acc[m][r + 1]);  // NaN-ignoring max
    const uint32_t shared_o = *(const uint32_t*)(lds + k3TauOff + (w * k3QW + l32) * 4);
    const uint32_t own_o = (uint32_t)(L[KL - 1] >> 32);
    const uint32_t thr_o = own_o > shared_o ? own_o : shared_o;
    const float thr = thr_o ? unord3(thr_o) : -__builtin_inff();
    if (mx >= thr) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float s = acc[m][r];
          if (s >= thr) {  // NaN (tombstoned rows, rows past the end) never passes
            const int row = rbase + m * 32 + (r & 3) + 8 * (r >> 2);
            const uint64_t key = ((uint64_t)ord3(s) << 32) | (uint32_t)(~(uint32_t)row);
            if (key > L[KL - 1]) key_insert3<KL>(L, key);
          }
        }
      const uint32_t pub = (uint32_t)(L[KL - 1] >> 32);
      if (pub > published && pub > shared_o) {
        __hip_atomic_fetch_max(tau + q, pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        published = pub;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if (q < nq) {
    const int64_t o = ((int64_t)q * n_lists + (int64_t)range * 2 + half) * KL;
#pragma unroll
    for (int i = 0; i < KL; ++i) {
      const uint64_t key = L[i];
      cand_s[o + i] = key ? unord3((uint32_t)(key >> 32)) : -__builtin_inff();
      cand_r[o + i] = key ? (int)(~(uint32_t)key) : kEmptyRow;
    }
  }
}

// one translation unit per (dtype, D) instantiates the kernel for the lane-list sizes KL in {4, 10, 16}
#define RFX_K3_INSTANTIATE(DTV, DV, NAME)                                                                  \
  int NAME(int kl, dim3 grid, hipStream_t st, const uint16_t* X, int nrows, const uint16_t* Qp, int nq,      \
           int tiles_per_block, int ntiles, uint32_t* tau, float* cs, int* cr, int64_t n_lists,            \
           const uint32_t* mask) {                                                                         \
    if (kl == 4)                                                                                         \
      hipLaunchKernelGGL((scan_mfma3_kernel<DTV, 4, DV>), grid, dim3(256), 0, st, X, nrows, Qp, nq,        \
                         tiles_per_block, ntiles, tau, cs, cr, n_lists, mask);                           \
    else if (kl == 10)                                                                                   \
      hipLaunchKernelGGL((scan_mfma3_kernel<DTV, 10, DV>), grid, dim3(256), 0, st, X, nrows, Qp, nq,       \
                         tiles_per_block, ntiles, tau, cs, cr, n_lists, mask);                           \
    else if (kl == 16)                                                                                   \
      hipLaunchKernelGGL((scan_mfma3_kernel<DTV, 16, DV>), grid, dim3(256), 0, st, X, nrows, Qp, nq,       \
                         tiles_per_block, ntiles, tau, cs, cr, n_lists, mask);                           \
    else                                                                                                 \
      return -1;                                                                                         \
    return 0;                                                                                            \
  }

}  // namespace k3
}  // namespace rfx
