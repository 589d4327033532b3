// k_scan_mfma8.hip — plan + dispatch of the k-split d = 1024 batched scan (kernel: k_scan_mfma8.h,
// instantiated per dtype in k8_*.hip).  Same grid, lists and threshold table as kernel 7.
#include "k_scan_mfma8.h"

namespace rfx {
namespace k8 {
#define RFX_K8_DECL(NAME)                                                                                 \
  int NAME(int kl, dim3 grid, hipStream_t st, const uint16_t* X, const uint16_t* Qp, int nq, int ntiles,     \
           int ranges, int groups, int paired, uint32_t* tau, float* cs, int* cr, int64_t n_lists,        \
           const uint32_t* mask, int mask_words, const uint32_t* gate);
RFX_K8_DECL(launch_bf16_1024)
RFX_K8_DECL(launch_f16_1024)
#undef RFX_K8_DECL
}  // namespace k8

size_t tau_bytes_mfma8(const MfmaPlan& p) { return (size_t)p.nq_pad * k8::kTauW * sizeof(uint32_t); }

// 128 queries per workgroup: G = ceil(nq / 128) query groups × R row ranges, R a multiple of 8 so
// the G groups of a range share an XCD.  p.blocks = R, p.q_blocks = G; one-dimensional grid.
MfmaPlan plan_scan_mfma8(int64_t nrows, int D, int dtype, int64_t nq, int k) {
  MfmaPlan p{};
  p.ok = (dtype == RFX_BF16 || dtype == RFX_F16) && D == 1024 && nrows > 0;
  p.k_lane = k <= 4 ? 4 : (k <= 10 ? 10 : -1);
  if (p.k_lane < 0) p.ok = false;
  p.bn = k8::kQG;
  p.q_blocks = (int)((nq + k8::kQG - 1) / k8::kQG);
  p.nq_pad = (int64_t)p.q_blocks * k8::kQG;
  if (p.q_blocks < 1 || p.q_blocks > 32) p.ok = false;
  const int64_t ntiles = std::max<int64_t>((nrows + k8::kTM - 1) / k8::kTM, 1);
  int64_t ranges = std::max<int64_t>(256 / std::max(p.q_blocks, 1), 1);
  if (ranges >= 8) ranges = ranges / 8 * 8;
  ranges = std::min<int64_t>(ranges, ntiles);
  p.blocks = (int)ranges;
  p.tiles_per_block = (int)((ntiles + ranges - 1) / ranges);
  p.lists_per_block = k8::kListsPerBlock;
  p.n_lists = (int64_t)p.blocks * k8::kListsPerBlock;
  return p;
}

int launch_scan_mfma8(const MfmaPlan& p, const void* X, int nrows, int D, int dtype, const void* Qpad, int nq,
                      uint32_t* tau, float* cs, int* cr, hipStream_t st, const uint32_t* mask, const uint32_t* gate,
                      bool tau_zeroed) {
  static_assert(k8::kTauW == kFallbackTauW, "screen_queries_kernel zeroes this table for the gated fallback");
  if (!p.ok || D != 1024) return -1;
  const int ntiles = (nrows + k8::kTM - 1) / k8::kTM;
  if (!tau_zeroed && hipMemsetAsync(tau, 0, tau_bytes_mfma8(p), st) != hipSuccess) return -2;
  const int paired = p.blocks % 8 == 0 ? 1 : 0;
  dim3 grid(p.blocks * p.q_blocks);
  auto f = dtype == RFX_BF16 ? k8::launch_bf16_1024 : k8::launch_f16_1024;
  return f(p.k_lane, grid, st, (const uint16_t*)X, (const uint16_t*)Qpad, nq, ntiles, p.blocks, p.q_blocks,
           paired, tau, cs, cr, p.n_lists, mask, (nrows + 31) / 32, gate);
}

}  // namespace rfx
