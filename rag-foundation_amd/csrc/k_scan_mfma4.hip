// k_scan_mfma4.hip — plan + dispatch of the all-query-stationary batched scan (kernel:
// k_scan_mfma4.h, instantiated per dtype in k4_*.hip), and its profiling ablations.
#include "k_scan_mfma4.h"

namespace rfx {
namespace k4 {
#define RFX_K4_DECL(NAME)                                                                                 \
  int NAME(int kl, dim3 grid, hipStream_t st, const uint16_t* X, const uint16_t* Qp, int nq,                \
           int tiles_per_block, int ntiles, uint32_t* tau, float* cs, int* cr, int64_t n_lists);
RFX_K4_DECL(launch_bf16_768)
RFX_K4_DECL(launch_f16_768)
#undef RFX_K4_DECL
}  // namespace k4

// threshold table: [nq_pad][kTauW] u32 (k_scan_mfma4.h)
size_t tau_bytes_mfma4(const MfmaPlan& p) { return (size_t)p.nq_pad * k4::kTauW * sizeof(uint32_t); }

// 256 queries per workgroup, one workgroup per CU: grid (ranges, q_blocks) with ranges·q_blocks ≈ 256.
MfmaPlan plan_scan_mfma4(int64_t nrows, int D, int dtype, int64_t nq, int k) {
  MfmaPlan p{};
  p.ok = (dtype == RFX_BF16 || dtype == RFX_F16) && D == 768 && nrows > 0;
  p.k_lane = k <= 4 ? 4 : (k <= 10 ? 10 : -1);
  if (p.k_lane < 0) p.ok = false;
  p.bn = k4::kQG;
  p.q_blocks = (int)((nq + k4::kQG - 1) / k4::kQG);
  p.nq_pad = (int64_t)p.q_blocks * k4::kQG;
  if (p.q_blocks < 1 || p.q_blocks > 256) p.ok = false;
  const int64_t ntiles = std::max<int64_t>((nrows + k4::kTM - 1) / k4::kTM, 1);
  int64_t ranges = std::max<int64_t>(256 / std::max(p.q_blocks, 1), 1);
  ranges = std::min<int64_t>(ranges, ntiles);
  p.tiles_per_block = (int)((ntiles + ranges - 1) / ranges);
  p.blocks = (int)((ntiles + p.tiles_per_block - 1) / p.tiles_per_block);
  p.lists_per_block = 2;
  p.n_lists = (int64_t)p.blocks * 2;
  return p;
}

int launch_scan_mfma4(const MfmaPlan& p, const void* X, int nrows, int D, int dtype, const void* Qpad, int nq,
                      uint32_t* tau, float* cs, int* cr, hipStream_t st) {
  if (!p.ok || D != 768) return -1;
  const int ntiles = (nrows + k4::kTM - 1) / k4::kTM;
  if (hipMemsetAsync(tau, 0, tau_bytes_mfma4(p), st) != hipSuccess) return -2;
  dim3 grid(p.blocks, p.q_blocks);
  auto f = dtype == RFX_BF16 ? k4::launch_bf16_768 : k4::launch_f16_768;
  return f(p.k_lane, grid, st, (const uint16_t*)X, (const uint16_t*)Qpad, nq, p.tiles_per_block, ntiles, tau, cs, cr,
           p.n_lists);
}

// Profiling ablations (bf16, d 768, KL 10), MODE bit flags of scan_mfma4_kernel:
// 1 = no top-k epilogue, 2 = no MFMA, 4 = contiguous row range per block, 8 = no corpus stream,
// 16 = count top-k slow-path entries (cand_r[0]), 32 = τ refresh through L1, 64 = DMA pieces
// bunched after the barrier, 128 = fragment prefetch distance 1,
// 256 = corpus pieces all re-read tile 0.
int launch_scan_mfma4_dbg(const MfmaPlan& p, int mode, const void* X, int nrows, int dtype, const void* Qpad, int nq,
                          uint32_t* tau, float* cs, int* cr, hipStream_t st) {
  if (!p.ok) return -1;
  if (mode == 0) return launch_scan_mfma4(p, X, nrows, 768, dtype, Qpad, nq, tau, cs, cr, st);  // production plan
  if (p.k_lane != 10) return -1;
  const int ntiles = (nrows + k4::kTM - 1) / k4::kTM;
  if (hipMemsetAsync(tau, 0, tau_bytes_mfma4(p), st) != hipSuccess) return -2;
  dim3 grid(p.blocks, p.q_blocks);
  const uint16_t* Xh = (const uint16_t*)X;
  const uint16_t* Qh = (const uint16_t*)Qpad;
#define RFX_K4_DBG(M)                                                                                  \
  case M:                                                                                              \
    hipLaunchKernelGGL((k4::scan_mfma4_kernel<RFX_BF16, 10, 768, M>), grid, dim3(256), 0, st, Xh, Qh, nq, \
                       p.tiles_per_block, ntiles, tau, cs, cr, p.n_lists);                             \
    break;
  switch (mode) {
    RFX_K4_DBG(1)
    RFX_K4_DBG(2)
    RFX_K4_DBG(3)
    RFX_K4_DBG(4)
    RFX_K4_DBG(5)
    RFX_K4_DBG(6)
    RFX_K4_DBG(8)
    RFX_K4_DBG(9)
    RFX_K4_DBG(16)
    RFX_K4_DBG(32)
    RFX_K4_DBG(48)
    RFX_K4_DBG(64)
    RFX_K4_DBG(128)
    RFX_K4_DBG(192)
    RFX_K4_DBG(257)
    default:
      return -1;
  }
#undef RFX_K4_DBG
  return 0;
}

}  // namespace rfx
