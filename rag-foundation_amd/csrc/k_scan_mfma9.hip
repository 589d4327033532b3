// k_scan_mfma9.hip — plan + dispatch of the batched f32 scan (kernel: k_scan_mfma9.h, instantiated
// in k9_f32_768.hip).
#include "k_scan_mfma9.h"

namespace rfx {
namespace k9 {
int launch_f32_768(int kl, dim3 grid, hipStream_t st, const float* X, const float* Qp, int nq, int ntiles,
                   int ranges, int groups, int paired, uint32_t* tau, float* cs, int* cr, int64_t n_lists,
                   const uint32_t* mask, int mask_words, const uint32_t* gate);
}  // namespace k9

size_t tau_bytes_mfma9(const MfmaPlan& p) { return (size_t)p.nq_pad * k9::kTauW * sizeof(uint32_t); }

// f32 stores, 16 < nq: 128 queries per workgroup, G = ceil(nq / 128) query groups × R row ranges,
// R·G ≈ 256 (R a multiple of 8: the groups of a range share an XCD).  Below 17 queries the VALU
// scan's 8-query slices cost less than a 128-query MFMA pass (the kernel computes all 128 columns).
MfmaPlan plan_scan_mfma9(int64_t nrows, int D, int dtype, int64_t nq, int k) {
  MfmaPlan p{};
  p.ok = dtype == RFX_F32 && D == 768 && nrows > 0 && nq > 16;
  p.k_lane = k <= 4 ? 4 : (k <= 10 ? 10 : -1);
  if (p.k_lane < 0) p.ok = false;
  p.bn = k9::kQG;
  p.q_blocks = (int)((nq + k9::kQG - 1) / k9::kQG);
  p.nq_pad = (int64_t)p.q_blocks * k9::kQG;
  if (p.q_blocks < 1 || p.q_blocks > 32) p.ok = false;
  const int64_t ntiles = std::max<int64_t>((nrows + k9::kTM - 1) / k9::kTM, 1);
  int64_t ranges = std::max<int64_t>(256 / std::max(p.q_blocks, 1), 1);
  if (ranges >= 8) ranges = ranges / 8 * 8;
  ranges = std::min<int64_t>(ranges, ntiles);
  p.blocks = (int)ranges;
  p.tiles_per_block = (int)((ntiles + ranges - 1) / ranges);
  p.lists_per_block = k9::kListsPerBlock;
  p.n_lists = (int64_t)p.blocks * k9::kListsPerBlock;
  return p;
}

int launch_scan_mfma9(const MfmaPlan& p, const void* X, int nrows, int D, int dtype, const void* Qpad, int nq,
                      uint32_t* tau, float* cs, int* cr, hipStream_t st, const uint32_t* mask, const uint32_t* gate,
                      bool tau_zeroed) {
  static_assert(k9::kTauW == kFallbackTauW, "screen_queries_kernel zeroes this table for the gated fallback");
  if (!p.ok || D != 768 || dtype != RFX_F32) return -1;
  const int ntiles = (nrows + k9::kTM - 1) / k9::kTM;
  if (!tau_zeroed && hipMemsetAsync(tau, 0, tau_bytes_mfma9(p), st) != hipSuccess) return -2;
  const int paired = p.blocks % 8 == 0 ? 1 : 0;
  dim3 grid(p.blocks * p.q_blocks);
  return k9::launch_f32_768(p.k_lane, grid, st, (const float*)X, (const float*)Qpad, nq, ntiles, p.blocks,
                            p.q_blocks, paired, tau, cs, cr, p.n_lists, mask, (nrows + 31) / 32, gate);
}

}  // namespace rfx
