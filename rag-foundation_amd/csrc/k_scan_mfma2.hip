// k_scan_mfma2.hip — batched scan for large query batches (nq > 128): 256 rows × 256 queries.
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551),
// BASELINE.json config 3 (10M×768 bf16, nq=256, k=10).  Same contract as k_scan_mfma.hip
// (fused scan + per-query top-k, scores never written to HBM); this variant is built for HBM
// bandwidth:
//   * tile = 256 corpus rows × 256 queries, K streamed in BK=32 stages (16 KB of corpus rows +
//     16 KB of query rows per stage, 1:1 HBM:L2 bytes).  Both operands arrive by LDS-DMA
//     (global_load_lds_dwordx4): corpus stages into a 5-slot ring (4 stages = 64 KB of HBM reads
//     in flight per CU), query stages (L2-resident, shorter latency) into a 4-slot ring.  One
//     counted `s_waitcnt vmcnt(10)` + raw `s_barrier` per stage; LDS 145 KB.
//   * 8 waves as 2 (rows) × 4 (queries); each wave owns 128 rows × 64 queries = 4×2 sub-tiles
//     of v_mfma_f32_32x32x16_{bf16,f16} (128 accumulator VGPRs).
//   * LDS image rows are 64 B = 4 slots of 16 B; chunk c of row r lives in slot
//     c ^ ((r>>2)&3): conflict-free 32-row ds_read_b128 fragment reads.  LDS-DMA writes
//     linearly, so the permutation goes on the per-lane SOURCE address.
//   * Top-k: lane l always holds queries (l&31)+32n, so it keeps a sorted list of KL 64-bit keys
//     (orderable score << 32 | ~row: one unsigned compare implements "score desc, row asc") per
//     query.  A score is only considered if it reaches max(own KL-th score, tau[q]), where tau[q]
//     is a per-query threshold shared by all workgroups through device-scope atomicMax: every
//     value ever published is the KL-th best of some subset of rows, hence a lower bound of the
//     global k-th best, so a stale read only filters less — results stay exact.
// Algorithmic bytes per tile: 256 * D * 2 (corpus rows, read once).
#include "rfx_device.h"
#include "rfx_kernels.h"

namespace rfx {

typedef __attribute__((ext_vector_type(8))) __bf16 v2bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 v2f16x8;
typedef __attribute__((ext_vector_type(16))) float v2f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned v2u32x4;

template <int DT>
__device__ __forceinline__ v2f32x16 mfma2(const uint4& a, const uint4& b, const v2f32x16& c) {
  if constexpr (DT == RFX_BF16)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v2bf16x8, a), __builtin_bit_cast(v2bf16x8, b),
                                                   c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v2f16x8, a), __builtin_bit_cast(v2f16x8, b), c,
                                                  0, 0, 0);
}

// float -> uint32 whose unsigned order is the float order (finite values and +-inf)
__device__ __forceinline__ uint32_t ord32(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unord32(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
__device__ __forceinline__ uint64_t mkkey(float s, int row) {
  return ((uint64_t)ord32(s) << 32) | (uint32_t)(~(uint32_t)row);
}

// NaN-ignoring 3-way max as plain fmaxf (hipcc emits v_max3_f32 and pads the MFMA->VALU hazard an
// inline-asm reader of an accumulator would not get).
__device__ __forceinline__ float vmax3(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

constexpr int kB2M = 256, kB2N = 256, kB2K = 32;
constexpr int kRowB = kB2K * 2;                    // 64 B per operand row per stage
constexpr int kSlot = kB2M * kRowB;                // 16 KB (corpus or query slot)
constexpr int kRingA = 5;                          // corpus: 4 stages in flight (64 KB of HBM reads)
constexpr int kRingB = 4;                          // queries (L2-resident): 3 stages in flight
constexpr int kTauOff = (kRingA + kRingB) * kSlot;   // 144 KB
constexpr int kLds = kTauOff + kB2N * 4;             // + 1 KB shared thresholds

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

__device__ __forceinline__ void glds16(const void* src, uint8_t* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

// MODE (diagnostic builds only, via rfx_dbg_scan_variant): 0 full; 1 no top-k epilogue;
// 2 loads + LDS reads only (no MFMA, no epilogue); 3 no query-row loads; 4 no corpus-row loads;
// 5 MFMA + LDS reads + barriers only (the rings are filled once, then never reloaded; no epilogue);
// 6 corpus loads only (no query reloads, no MFMA, no epilogue); 7 query loads only (ditto).
template <int DT, int KL, int MODE = 0>
__global__ __launch_bounds__(512) void scan_mfma2_kernel(const uint16_t* __restrict__ X, int nrows, int D,
                                                         const uint16_t* __restrict__ Qp, int nq, int tiles_per_block,
                                                         int ntiles, uint32_t* __restrict__ tau,
                                                         float* __restrict__ cand_s, int* __restrict__ cand_r,
                                                         int64_t n_lists, const uint32_t* __restrict__ mask) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[kLds];

  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int wm = w >> 2, wn = w & 3;  // 2 × 4 wave grid
  const int half = lane >> 5, l32 = lane & 31;
  const int qb = blockIdx.y * kB2N;
  const int t0 = blockIdx.x * tiles_per_block;
  const int t1 = min(ntiles, t0 + tiles_per_block);
  const int nk = D / kB2K;
  const int S = t1 > t0 ? (t1 - t0) * nk : 0;

  // LDS-DMA pattern (per 16 KB slot): wave-instruction j (0..15) fills bytes [1024 j, 1024 j+1024)
  // = operand rows 16j..16j+15; lane -> (row 16j + lane/4, slot lane%4) <- source chunk
  // slot ^ ((row>>2)&3).  Wave w issues j = w and w+8 for each operand.
  const int r0 = 16 * w + (lane >> 2), r1 = 16 * (w + 8) + (lane >> 2);
  const int c0 = (lane & 3) ^ ((r0 >> 2) & 3), c1 = (lane & 3) ^ ((r1 >> 2) & 3);
  const uint16_t* qsrc0 = Qp + (int64_t)(qb + r0) * D + c0 * 8;
  const uint16_t* qsrc1 = Qp + (int64_t)(qb + r1) * D + c1 * 8;

  auto issue_a = [&](int st) {
    const int tl = st / nk;
    const int koff = (st - tl * nk) * kB2K;
    const int row_base = (t0 + tl) * kB2M;
    int ra = row_base + r0, rb = row_base + r1;
    ra = ra < nrows ? ra : nrows - 1;
    rb = rb < nrows ? rb : nrows - 1;
    uint8_t* dst = lds + (st % kRingA) * kSlot;
    if (MODE == 4 || ((MODE == 5 || MODE == 7) && st >= kRingA)) return;
    glds16(X + (int64_t)ra * D + koff + c0 * 8, dst + w * 1024);
    glds16(X + (int64_t)rb * D + koff + c1 * 8, dst + (w + 8) * 1024);
  };
  auto issue_b = [&](int st) {
    const int tl = st / nk;
    const int koff = (st - tl * nk) * kB2K;
    uint8_t* dst = lds + kRingA * kSlot + (st % kRingB) * kSlot;
    if (MODE == 3 || ((MODE == 5 || MODE == 6) && st >= kRingB)) return;
    glds16(qsrc0 + koff, dst + w * 1024);
    glds16(qsrc1 + koff, dst + (w + 8) * 1024);
  };
  // shared thresholds of this query block -> LDS (one wave-instruction, wave 0)
  auto issue_tau = [&]() {
    if (w == 0) glds16(tau + qb + lane * 4, lds + kTauOff);
  };

  v2f32x16 acc[4][2];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;

  uint64_t L[2][KL];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int i = 0; i < KL; ++i) L[n][i] = 0ull;
  uint32_t published[2] = {0u, 0u};
  uint32_t* tau_q[2] = {tau + qb + wn * 64 + l32, tau + qb + wn * 64 + 32 + l32};
  const int tau_lds[2] = {kTauOff + (wn * 64 + l32) * 4, kTauOff + (wn * 64 + 32 + l32) * 4};

  int a_off[4], b_off[2], a_sw[4], b_sw[2];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int r = wm * 128 + m * 32 + l32;
    a_off[m] = r * kRowB;
    a_sw[m] = (r >> 2) & 3;
  }
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const int q = wn * 64 + n * 32 + l32;
    b_off[n] = kRingA * kSlot + q * kRowB;
    b_sw[n] = (q >> 2) & 3;
  }

  // prologue in steady-state order: A0 | B0 A1 | B1 A2 | B2 A3   (top of stage s issues B(s+3), A(s+4))
  issue_tau();
  if (S > 0) issue_a(0);
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    if (p < S) issue_b(p);
    if (p + 1 < S) issue_a(p + 1);
  }

  for (int st = 0; st < S; ++st) {
    // A(st) and B(st) landed for this wave: newer are A(st+1..st+3), B(st+1..st+2) = 10 ops
    if (st + 3 < S)
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (st % nk == 0 && st > 0) issue_tau();  // refresh at each tile start (read >= 5 stages later)
    if (st + 3 < S) issue_b(st + 3);
    if (st + 4 < S) issue_a(st + 4);

    const uint8_t* sa = lds + (st % kRingA) * kSlot;
    const uint8_t* sb = lds + (st % kRingB) * kSlot;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 2 + half;
      uint4 a[4], b[2];
#pragma unroll
      for (int m = 0; m < 4; ++m) a[m] = *(const uint4*)(sa + a_off[m] + ((c ^ a_sw[m]) << 4));
#pragma unroll
      for (int n = 0; n < 2; ++n) b[n] = *(const uint4*)(sb + b_off[n] + ((c ^ b_sw[n]) << 4));
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          if constexpr (MODE == 2 || MODE == 6 || MODE == 7)
            asm volatile("" ::"v"(__builtin_bit_cast(v2u32x4, a[m])), "v"(__builtin_bit_cast(v2u32x4, b[n])));
          else
            acc[m][n] = mfma2<DT>(a[m], b[n], acc[m][n]);
        }
    }

    if ((MODE == 1 || MODE == 2 || MODE >= 5) && st % nk == nk - 1) {
      float t = 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            t += acc[m][n][r];
            acc[m][n][r] = 0.f;
          }
      if (t == 12345.678f) L[0][0] = 1;  // keeps the MFMA results live
    }
    if ((MODE == 0 || MODE == 3 || MODE == 4) && st % nk == nk - 1) {
      // ---- epilogue: fold this tile's 256 rows into the lane lists ----
      if (nk < 5) {  // the tile's threshold DMA may be younger than 4 stages: drain + barrier
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_barrier" ::: "memory");
      }
      const int tile = t0 + st / nk;
      const int rbase = tile * kB2M + wm * 128 + 4 * half;
      const bool full_tile = tile * kB2M + kB2M <= nrows;
      if (mask) {  // metadata filter (uniform branch): excluded rows -> NaN
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const uint32_t bits = acc_row_bits(mask, rbase + m * 32, nrows);
#pragma unroll
          for (int n = 0; n < 2; ++n) mask_acc16(acc[m][n], bits);
        }
      }
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        float mx = -__builtin_inff();
        if (full_tile) {
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int r = 0; r < 16; r += 2) mx = vmax3(mx, acc[m][n][r], acc[m][n][r + 1]);
        } else {
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = rbase + m * 32 + (r & 3) + 8 * (r >> 2);
              mx = vmax3(mx, row < nrows ? acc[m][n][r] : -__builtin_inff(), -__builtin_inff());
            }
        }
        const uint32_t shared_thr = *(const uint32_t*)(lds + tau_lds[n]);
        const uint32_t own = (uint32_t)(L[n][KL - 1] >> 32);
        const uint32_t thr = own > shared_thr ? own : shared_thr;
        if (mx == mx && ord32(mx) >= thr) {
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = rbase + m * 32 + (r & 3) + 8 * (r >> 2);
              const float s = acc[m][n][r];
              if (row < nrows && s == s && ord32(s) >= thr) {
                const uint64_t key = mkkey(s, row);
                if (key > L[n][KL - 1]) key_insert<KL>(L[n], key);
              }
            }
          // publish this list's KL-th score: a lower bound of the query's global k-th best
          const uint32_t pub = (uint32_t)(L[n][KL - 1] >> 32);
          if (pub > published[n] && pub > shared_thr) {
            __hip_atomic_fetch_max(tau_q[n], pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            published[n] = pub;
          }
        }
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- emit lane lists: query q, list id (block, wm, half) ----
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const int q = qb + wn * 64 + n * 32 + l32;
    if (q < nq) {
      const int64_t lid = (int64_t)blockIdx.x * 4 + wm * 2 + half;
      const int64_t o = ((int64_t)q * n_lists + lid) * KL;
#pragma unroll
      for (int i = 0; i < KL; ++i) {
        const uint64_t key = L[n][i];
        cand_s[o + i] = key ? unord32((uint32_t)(key >> 32)) : -__builtin_inff();
        cand_r[o + i] = key ? (int)(~(uint32_t)key) : kEmptyRow;
      }
    }
  }
}

MfmaPlan plan_scan_mfma2(int64_t nrows, int D, int dtype, int64_t nq, int k) {
  MfmaPlan p{};
  p.ok = (dtype == RFX_BF16 || dtype == RFX_F16) && D % 64 == 0 && nrows > 0;
  p.k_lane = k <= 4 ? 4 : (k <= 8 ? 8 : (k <= 10 ? 10 : (k <= 16 ? 16 : -1)));
  if (p.k_lane < 0) p.ok = false;
  p.bn = kB2N;
  p.q_blocks = (int)((nq + kB2N - 1) / kB2N);
  p.nq_pad = (int64_t)p.q_blocks * kB2N;
  const int64_t ntiles = std::max<int64_t>((nrows + kB2M - 1) / kB2M, 1);
  int64_t blocks = std::min<int64_t>(ntiles, 256);
  p.tiles_per_block = (int)((ntiles + blocks - 1) / blocks);
  p.blocks = (int)((ntiles + p.tiles_per_block - 1) / p.tiles_per_block);
  p.lists_per_block = 4;
  p.n_lists = (int64_t)p.blocks * 4;
  return p;
}

int launch_scan_mfma2_dbg(const MfmaPlan& p, int mode, const void* X, int nrows, int D, const void* Qpad, int nq,
                          uint32_t* tau, float* cs, int* cr, hipStream_t st) {
  if (!p.ok || p.k_lane != 10) return -1;
  const int ntiles = (nrows + kB2M - 1) / kB2M;
  if (hipMemsetAsync(tau, 0, (size_t)p.nq_pad * sizeof(uint32_t), st) != hipSuccess) return -2;
  dim3 grid(p.blocks, p.q_blocks);
  const uint16_t* Xh = (const uint16_t*)X;
  const uint16_t* Qh = (const uint16_t*)Qpad;
#define RFX_M2(MV)                                                                                        \
  if (mode == MV) {                                                                                       \
    hipLaunchKernelGGL((scan_mfma2_kernel<RFX_BF16, 10, MV>), grid, dim3(512), 0, st, Xh, nrows, D, Qh, nq, \
                       p.tiles_per_block, ntiles, tau, cs, cr, p.n_lists, nullptr);                       \
    return 0;                                                                                             \
  }
  RFX_M2(0) RFX_M2(1) RFX_M2(2) RFX_M2(3) RFX_M2(4) RFX_M2(5) RFX_M2(6) RFX_M2(7)
#undef RFX_M2
  return -1;
}

int launch_scan_mfma2(const MfmaPlan& p, const void* X, int nrows, int D, int dtype, const void* Qpad, int nq,
                      uint32_t* tau, float* cs, int* cr, hipStream_t st, const uint32_t* mask) {
  if (!p.ok) return -1;
  const int ntiles = (nrows + kB2M - 1) / kB2M;
  if (hipMemsetAsync(tau, 0, (size_t)p.nq_pad * sizeof(uint32_t), st) != hipSuccess) return -2;
  dim3 grid(p.blocks, p.q_blocks);
  const uint16_t* Xh = (const uint16_t*)X;
  const uint16_t* Qh = (const uint16_t*)Qpad;
#define RFX_KL2(DTV, KV)                                                                                  \
  if (dtype == DTV && p.k_lane == KV) {                                                                   \
    hipLaunchKernelGGL((scan_mfma2_kernel<DTV, KV>), grid, dim3(512), 0, st, Xh, nrows, D, Qh, nq,         \
                       p.tiles_per_block, ntiles, tau, cs, cr, p.n_lists, mask);                          \
    return 0;                                                                                             \
  }
  RFX_KL2(RFX_BF16, 4) RFX_KL2(RFX_BF16, 8) RFX_KL2(RFX_BF16, 10) RFX_KL2(RFX_BF16, 16)
  RFX_KL2(RFX_F16, 4) RFX_KL2(RFX_F16, 8) RFX_KL2(RFX_F16, 10) RFX_KL2(RFX_F16, 16)
#undef RFX_KL2
  return -1;
}

}  // namespace rfx
