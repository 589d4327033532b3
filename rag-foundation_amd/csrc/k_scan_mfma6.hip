// k_scan_mfma6.hip — plan + dispatch of the headline scan (kernel: k_scan_mfma6.h, instantiated per
// dtype in k6_*.hip).
#include "k_scan_mfma6.h"

namespace rfx {
namespace k6 {
#define RFX_K6_DECL(NAME)                                                                                 \
  int NAME(int kl, dim3 grid, hipStream_t st, const uint16_t* X, const uint16_t* Qp, int nq, int ntiles,     \
           uint32_t* tau, float* cs, int* cr, int64_t n_lists, const uint32_t* mask, const uint32_t* gate);
RFX_K6_DECL(launch_bf16_768)
RFX_K6_DECL(launch_f16_768)
#undef RFX_K6_DECL
}  // namespace k6

// threshold table: [nq_pad][kTauW] u32 (k_scan_mfma6.h)
size_t tau_bytes_mfma6(const MfmaPlan& p) { return (size_t)p.nq_pad * k6::kTauW * sizeof(uint32_t); }

// 256 queries per workgroup, one workgroup per CU: grid (ranges, q_blocks), ranges·q_blocks ≈ 256;
// block b of a query group scans tiles b, b + ranges, ...
MfmaPlan plan_scan_mfma6(int64_t nrows, int D, int dtype, int64_t nq, int k) {
  MfmaPlan p{};
  p.ok = (dtype == RFX_BF16 || dtype == RFX_F16) && D == 768 && nrows > 0;
  p.k_lane = k <= 4 ? 4 : (k <= 10 ? 10 : -1);
  if (p.k_lane < 0) p.ok = false;
  p.bn = k6::kQG;
  p.q_blocks = (int)((nq + k6::kQG - 1) / k6::kQG);
  p.nq_pad = (int64_t)p.q_blocks * k6::kQG;
  if (p.q_blocks < 1 || p.q_blocks > 256) p.ok = false;
  const int64_t ntiles = std::max<int64_t>((nrows + k6::kTM - 1) / k6::kTM, 1);
  int64_t ranges = std::max<int64_t>(256 / std::max(p.q_blocks, 1), 1);
  ranges = std::min<int64_t>(ranges, ntiles);
  p.blocks = (int)ranges;
  p.tiles_per_block = (int)((ntiles + ranges - 1) / ranges);
  p.lists_per_block = 2;
  p.n_lists = (int64_t)p.blocks * 2;
  return p;
}

int launch_scan_mfma6(const MfmaPlan& p, const void* X, int nrows, int D, int dtype, const void* Qpad, int nq,
                      uint32_t* tau, float* cs, int* cr, hipStream_t st, const uint32_t* mask, const uint32_t* gate,
                      bool tau_zeroed) {
  static_assert(k6::kTauW == kFallbackTauW, "screen_queries_kernel zeroes this table for the gated fallback");
  if (!p.ok || D != 768) return -1;
  const int ntiles = (nrows + k6::kTM - 1) / k6::kTM;
  if (!tau_zeroed && hipMemsetAsync(tau, 0, tau_bytes_mfma6(p), st) != hipSuccess) return -2;
  dim3 grid(p.blocks, p.q_blocks);
  auto f = dtype == RFX_BF16 ? k6::launch_bf16_768 : k6::launch_f16_768;
  return f(p.k_lane, grid, st, (const uint16_t*)X, (const uint16_t*)Qpad, nq, ntiles, tau, cs, cr, p.n_lists, mask, gate);
}

}  // namespace rfx
