// k_scan_mfma.hip — batched query×corpus scan on MFMA with a fused per-query top-k.
//
// Path: the retrieval half of GeminiRag.ask_stream (backend/app/services/gemini_rag.py:517-551)
// for batched queries (BASELINE.json config 3: 10M×768 bf16, nq=256, k=10).  The score matrix
// (nq × rows) is never written to HBM: every 128-row tile's scores stay in the MFMA accumulators
// and are folded into lane-resident top-k lists.
//
// Structure (one 512-thread workgroup per CU, persistent over a contiguous range of row tiles):
//   * tile = BM (128) corpus rows × BN (64/128/256) queries; 8 waves as WM×WN, each wave owns
//     (BM/WM) rows × (BN/WN) queries = MS×NS sub-tiles of 32×32 (v_mfma_f32_32x32x16_{bf16,f16}).
//   * K is streamed in BK=64 stages.  Both operands (corpus rows from HBM, query rows from L2)
//     arrive by LDS-DMA (global_load_lds_dwordx4) into a 3-slot ring: stage t+2 is in flight
//     while stage t is consumed; one counted `s_waitcnt vmcnt` + raw `s_barrier` per stage.
//   * LDS image per operand row: 128 B = 8 slots of 16 B; chunk c of row r sits in slot
//     c ^ ((r>>1)&7), which makes the 32-row ds_read_b128 fragment reads conflict-free.  The
//     LDS-DMA writes linearly, so the permutation is applied to the per-lane SOURCE address.
//   * Epilogue per tile: lane l of a wave always holds query (l&31)+32n, so each lane keeps a
//     sorted top-KL list per query in registers and only inserts scores that beat its own
//     KL-th entry (rare after warm-up).  Per query a block emits WM*2 lane lists.
// Algorithmic bytes per tile: BM*D*2 (corpus) — queries are L2-resident (nq*D*2 per batch).
#include "rfx_device.h"
#include "rfx_kernels.h"

namespace rfx {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

template <int DT>
__device__ __forceinline__ f32x16_t mfma32(const uint4& a, const uint4& b, const f32x16_t& c) {
  if constexpr (DT == RFX_BF16)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                   __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a),
                                                  __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
}

constexpr int kBM = 128;
constexpr int kBK = 64;

template <int BN>
struct MfmaGeom {
  static constexpr int WN = BN == 256 ? 4 : 2;
  static constexpr int WM = 8 / WN;
  static constexpr int WROWS = kBM / WM;
  static constexpr int WQ = BN / WN;
  static constexpr int MS = WROWS / 32;
  static constexpr int NS = WQ / 32;
  static constexpr int STAGE_ROWS = kBM + BN;
  static constexpr int STAGE_BYTES = STAGE_ROWS * kBK * 2;
  static constexpr int GPW = STAGE_ROWS / 8 / 8;  // LDS-DMA wave-instructions per wave per stage
  static_assert(MS >= 1 && NS >= 1, "geometry");
  static_assert((STAGE_ROWS / 8) % 8 == 0, "stage rows must split evenly over 8 waves");
};

// counted wait on this wave's outstanding vector-memory ops (LDS-DMA included)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}

template <int KL>
__device__ __forceinline__ void list_insert(float (&ls)[KL], int (&lr)[KL], float s, int r) {
  float cs = s;
  int cr = r;
#pragma unroll
  for (int i = 0; i < KL; ++i) {
    const bool b = better(cs, cr, ls[i], lr[i]);
    const float ts = ls[i];
    const int tr = lr[i];
    ls[i] = b ? cs : ts;
    lr[i] = b ? cr : tr;
    cs = b ? ts : cs;
    cr = b ? tr : cr;
  }
}

// MODE (diagnostic builds only, reached through rfx_dbg_scan_variant): 0 = full kernel,
// 1 = no top-k epilogue (accumulators folded into one value), 2 = no MFMA (data movement only).
template <int DT, int BN, int KL, int MODE = 0>
__global__ __launch_bounds__(512) void scan_mfma_kernel(const uint16_t* __restrict__ X, int nrows, int D,
                                                        const uint16_t* __restrict__ Qp, int nq,
                                                        int tiles_per_block, int ntiles,
                                                        float* __restrict__ cand_s, int* __restrict__ cand_r,
                                                        int64_t n_lists, const uint32_t* __restrict__ mask) {
  using G = MfmaGeom<BN>;
  __shared__ __attribute__((aligned(1024))) uint8_t lds[3 * G::STAGE_BYTES];

  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int wm = w / G::WN, wn = w % G::WN;
  const int qb = blockIdx.y * BN;
  const int t0 = blockIdx.x * tiles_per_block;
  const int t1 = min(ntiles, t0 + tiles_per_block);
  const int nk = D / kBK;
  const int S = t1 > t0 ? (t1 - t0) * nk : 0;

  // ---- LDS-DMA source pattern for this wave's GPW instructions per stage ----
  // instruction i covers stage rows 8i..8i+7; lane -> (row 8i + lane/8, slot lane%8) which
  // holds source chunk (slot ^ ((row>>1)&7)).
  const uint16_t* src_base[G::GPW];
  bool src_is_a[G::GPW];
#pragma unroll
  for (int u = 0; u < G::GPW; ++u) {
    const int i = w + 8 * u;
    const int sr = 8 * i + (lane >> 3);
    const int slot = lane & 7;
    if (sr < kBM) {
      const int chunk = slot ^ ((sr >> 1) & 7);
      src_base[u] = X + chunk * 8;  // + row * D added per tile
      src_is_a[u] = true;
    } else {
      const int r = sr - kBM;
      const int chunk = slot ^ ((r >> 1) & 7);
      src_base[u] = Qp + (int64_t)(qb + r) * D + chunk * 8;
      src_is_a[u] = false;
    }
  }

  auto issue = [&](int st) {
    const int tile = t0 + st / nk;
    const int ks = st - (st / nk) * nk;
    uint8_t* dst = lds + (st % 3) * G::STAGE_BYTES;
#pragma unroll
    for (int u = 0; u < G::GPW; ++u) {
      const int i = w + 8 * u;
      const uint16_t* src;
      if (src_is_a[u]) {
        int row = tile * kBM + 8 * i + (lane >> 3);
        row = row < nrows ? row : nrows - 1;
        src = src_base[u] + (int64_t)row * D + ks * kBK;
      } else {
        src = src_base[u] + ks * kBK;
      }
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(dst + i * 1024), 16, 0, 0);
    }
  };

  f32x16_t acc[G::MS][G::NS];
#pragma unroll
  for (int m = 0; m < G::MS; ++m)
#pragma unroll
    for (int n = 0; n < G::NS; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;

  float ls[G::NS][KL];
  int lr[G::NS][KL];
#pragma unroll
  for (int n = 0; n < G::NS; ++n)
#pragma unroll
    for (int i = 0; i < KL; ++i) {
      ls[n][i] = -__builtin_inff();
      lr[n][i] = kEmptyRow;
    }

  const int half = lane >> 5, l32 = lane & 31;

  if (S > 0) issue(0);
  if (S > 1) issue(1);
  for (int st = 0; st < S; ++st) {
    if (st + 1 < S)
      wait_vmcnt<G::GPW>();
    else
      wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (st + 2 < S) issue(st + 2);

    const uint8_t* As = lds + (st % 3) * G::STAGE_BYTES;
    const uint8_t* Bs = As + kBM * 128;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int c = kk * 2 + half;
      uint4 a[G::MS], b[G::NS];
#pragma unroll
      for (int m = 0; m < G::MS; ++m) {
        const int r = wm * G::WROWS + m * 32 + l32;
        a[m] = *(const uint4*)(As + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int n = 0; n < G::NS; ++n) {
        const int q = wn * G::WQ + n * 32 + l32;
        b[n] = *(const uint4*)(Bs + q * 128 + ((c ^ ((q >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int m = 0; m < G::MS; ++m)
#pragma unroll
        for (int n = 0; n < G::NS; ++n) {
          if constexpr (MODE == 2) {
            acc[m][n][0] += __uint_as_float(a[m].x ^ b[n].y);
          } else {
            acc[m][n] = mfma32<DT>(a[m], b[n], acc[m][n]);
          }
        }
    }

    if (MODE != 0 && st % nk == nk - 1) {
      float t = 0.f;
#pragma unroll
      for (int m = 0; m < G::MS; ++m)
#pragma unroll
        for (int n = 0; n < G::NS; ++n) {
#pragma unroll
          for (int r = 0; r < 16; ++r) t += acc[m][n][r];
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;
        }
      if (t == 12345.678f) ls[0][0] = t;  // keeps the MFMA results live
    }
    if (MODE == 0 && st % nk == nk - 1) {
      // ---- epilogue: fold this tile's scores into the lane lists ----
      const int tile = t0 + st / nk;
      const int rbase = tile * kBM + wm * G::WROWS + 4 * half;
      if (mask) {  // metadata filter (uniform branch): excluded rows -> NaN
#pragma unroll
        for (int m = 0; m < G::MS; ++m) {
          const uint32_t bits = acc_row_bits(mask, rbase + m * 32, nrows);
#pragma unroll
          for (int n = 0; n < G::NS; ++n) mask_acc16(acc[m][n], bits);
        }
      }
#pragma unroll
      for (int n = 0; n < G::NS; ++n) {
        float mx = -__builtin_inff();
#pragma unroll
        for (int m = 0; m < G::MS; ++m)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rbase + m * 32 + (r & 3) + 8 * (r >> 2);
            mx = fmaxf(mx, row < nrows ? acc[m][n][r] : -__builtin_inff());
          }
        if (mx >= ls[n][KL - 1]) {
#pragma unroll
          for (int m = 0; m < G::MS; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = rbase + m * 32 + (r & 3) + 8 * (r >> 2);
              const float s = acc[m][n][r];
              if (row < nrows && better(s, row, ls[n][KL - 1], lr[n][KL - 1])) list_insert<KL>(ls[n], lr[n], s, row);
            }
        }
#pragma unroll
        for (int m = 0; m < G::MS; ++m)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;
      }
    }
  }

  // ---- emit lane lists: query q, list id (block, wm, half) ----
  const int lists_per_block = G::WM * 2;
#pragma unroll
  for (int n = 0; n < G::NS; ++n) {
    const int q = qb + wn * G::WQ + n * 32 + l32;
    if (q < nq) {
      const int64_t lid = (int64_t)blockIdx.x * lists_per_block + wm * 2 + half;
      const int64_t o = ((int64_t)q * n_lists + lid) * KL;
#pragma unroll
      for (int i = 0; i < KL; ++i) {
        cand_s[o + i] = ls[n][i];
        cand_r[o + i] = lr[n][i];
      }
    }
  }
}

static int mfma_k_lane(int k) {
  if (k <= 4) return 4;
  if (k <= 8) return 8;
  if (k <= 10) return 10;
  if (k <= 16) return 16;
  return -1;
}

MfmaPlan plan_scan_mfma(int64_t nrows, int D, int dtype, int64_t nq, int k) {
  MfmaPlan p{};
  p.ok = (dtype == RFX_BF16 || dtype == RFX_F16) && D % kBK == 0 && nrows > 0;
  p.k_lane = mfma_k_lane(k);
  if (p.k_lane < 0) p.ok = false;
  p.bn = nq <= 64 ? 64 : (nq <= 128 ? 128 : 256);
  p.q_blocks = (int)((nq + p.bn - 1) / p.bn);
  p.nq_pad = (int64_t)p.q_blocks * p.bn;
  const int64_t ntiles = std::max<int64_t>((nrows + kBM - 1) / kBM, 1);
  const int wg_per_cu = p.bn == 256 ? 1 : 2;
  int64_t blocks = std::min<int64_t>(ntiles, 256 * wg_per_cu);
  if (blocks < 1) blocks = 1;
  p.tiles_per_block = (int)((ntiles + blocks - 1) / blocks);
  p.blocks = (int)((ntiles + p.tiles_per_block - 1) / p.tiles_per_block);
  const int wm = p.bn == 256 ? 2 : 4;
  p.lists_per_block = wm * 2;
  p.n_lists = (int64_t)p.blocks * p.lists_per_block;
  return p;
}

__global__ void pad_queries_kernel(const uint8_t* __restrict__ Q, int64_t qbytes, int64_t total,
                                   uint8_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = i < qbytes ? Q[i] : 0;
}

void launch_pad_queries(const void* Q, int64_t nq, int64_t nq_pad, int D, int esz, void* out, hipStream_t st) {
  const int64_t qbytes = nq * D * esz, total = nq_pad * D * esz;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(pad_queries_kernel, dim3(blocks < 1 ? 1 : blocks), dim3(256), 0, st, (const uint8_t*)Q,
                     qbytes, total, (uint8_t*)out);
}

template <int DT, int BN>
static int launch_mfma_kl(const MfmaPlan& p, const uint16_t* X, int nrows, int D, const uint16_t* Qp, int nq,
                          float* cs, int* cr, hipStream_t st, const uint32_t* mask) {
  const int ntiles = (nrows + kBM - 1) / kBM;
  dim3 grid(p.blocks, p.q_blocks);
#define RFX_KL(KV)                                                                                     \
  if (p.k_lane == KV) {                                                                                \
    hipLaunchKernelGGL((scan_mfma_kernel<DT, BN, KV>), grid, dim3(512), 0, st, X, nrows, D, Qp, nq,     \
                       p.tiles_per_block, ntiles, cs, cr, p.n_lists, mask);                            \
    return 0;                                                                                          \
  }
  RFX_KL(4) RFX_KL(8) RFX_KL(10) RFX_KL(16)
#undef RFX_KL
  return -1;
}

template <int DT>
static int launch_mfma_bn(const MfmaPlan& p, const uint16_t* X, int nrows, int D, const uint16_t* Qp, int nq,
                          float* cs, int* cr, hipStream_t st, const uint32_t* mask) {
  if (p.bn == 64) return launch_mfma_kl<DT, 64>(p, X, nrows, D, Qp, nq, cs, cr, st, mask);
  if (p.bn == 128) return launch_mfma_kl<DT, 128>(p, X, nrows, D, Qp, nq, cs, cr, st, mask);
  return launch_mfma_kl<DT, 256>(p, X, nrows, D, Qp, nq, cs, cr, st, mask);
}

int launch_scan_mfma_dbg(const MfmaPlan& p, int mode, const void* X, int nrows, int D, const void* Qpad, int nq,
                         float* cs, int* cr, hipStream_t st) {
  if (!p.ok || p.bn != 256 || p.k_lane != 10) return -1;
  const int ntiles = (nrows + kBM - 1) / kBM;
  dim3 grid(p.blocks, p.q_blocks);
  const uint16_t* Xh = (const uint16_t*)X;
  const uint16_t* Qh = (const uint16_t*)Qpad;
  if (mode == 1)
    hipLaunchKernelGGL((scan_mfma_kernel<RFX_BF16, 256, 10, 1>), grid, dim3(512), 0, st, Xh, nrows, D, Qh, nq,
                       p.tiles_per_block, ntiles, cs, cr, p.n_lists, nullptr);
  else if (mode == 2)
    hipLaunchKernelGGL((scan_mfma_kernel<RFX_BF16, 256, 10, 2>), grid, dim3(512), 0, st, Xh, nrows, D, Qh, nq,
                       p.tiles_per_block, ntiles, cs, cr, p.n_lists, nullptr);
  else
    hipLaunchKernelGGL((scan_mfma_kernel<RFX_BF16, 256, 10, 0>), grid, dim3(512), 0, st, Xh, nrows, D, Qh, nq,
                       p.tiles_per_block, ntiles, cs, cr, p.n_lists, nullptr);
  return 0;
}

int launch_scan_mfma(const MfmaPlan& p, const void* X, int nrows, int D, int dtype, const void* Qpad, int nq,
                     float* cs, int* cr, hipStream_t st, const uint32_t* mask) {
  if (!p.ok) return -1;
  if (dtype == RFX_BF16)
    return launch_mfma_bn<RFX_BF16>(p, (const uint16_t*)X, nrows, D, (const uint16_t*)Qpad, nq, cs, cr, st, mask);
  return launch_mfma_bn<RFX_F16>(p, (const uint16_t*)X, nrows, D, (const uint16_t*)Qpad, nq, cs, cr, st, mask);
}

}  // namespace rfx
