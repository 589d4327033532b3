// k_scan_mfma3.hip — plan + dispatch of the query-stationary batched scan (kernel: k_scan_mfma3.h,
// instantiated per (dtype, d) in k3_*.hip).
#include "rfx_kernels.h"

namespace rfx {
namespace k3 {
#define RFX_K3_DECL(NAME)                                                                                  \
  int NAME(int kl, dim3 grid, hipStream_t st, const uint16_t* X, int nrows, const uint16_t* Qp, int nq,      \
           int tiles_per_block, int ntiles, uint32_t* tau, float* cs, int* cr, int64_t n_lists,            \
           const uint32_t* mask);
RFX_K3_DECL(launch_bf16_768)
RFX_K3_DECL(launch_bf16_1024)
RFX_K3_DECL(launch_f16_768)
RFX_K3_DECL(launch_f16_1024)
#undef RFX_K3_DECL
constexpr int kM = 128, kQG = 128;
}  // namespace k3

MfmaPlan plan_scan_mfma3(int64_t nrows, int D, int dtype, int64_t nq, int k) {
  MfmaPlan p{};
  p.ok = (dtype == RFX_BF16 || dtype == RFX_F16) && (D == 768 || D == 1024) && nrows > 0;
  p.k_lane = k <= 4 ? 4 : (k <= 10 ? 10 : (k <= 16 ? 16 : -1));
  if (p.k_lane < 0) p.ok = false;
  p.bn = k3::kQG;
  p.q_blocks = (int)((nq + k3::kQG - 1) / k3::kQG);
  p.nq_pad = (int64_t)p.q_blocks * k3::kQG;
  if (p.q_blocks < 1 || p.q_blocks > 256) p.ok = false;
  const int64_t ntiles = std::max<int64_t>((nrows + k3::kM - 1) / k3::kM, 1);
  int64_t ranges = std::max<int64_t>(256 / std::max(p.q_blocks, 1), 1);
  ranges = std::min<int64_t>(ranges, ntiles);
  p.tiles_per_block = (int)((ntiles + ranges - 1) / ranges);
  p.blocks = (int)((ntiles + p.tiles_per_block - 1) / p.tiles_per_block);
  p.lists_per_block = 2;
  p.n_lists = (int64_t)p.blocks * 2;
  return p;
}

int launch_scan_mfma3(const MfmaPlan& p, const void* X, int nrows, int D, int dtype, const void* Qpad, int nq,
                      uint32_t* tau, float* cs, int* cr, hipStream_t st, const uint32_t* mask) {
  if (!p.ok) return -1;
  const int ntiles = (nrows + k3::kM - 1) / k3::kM;
  if (hipMemsetAsync(tau, 0, (size_t)(p.nq_pad + 256) * sizeof(uint32_t), st) != hipSuccess) return -2;
  dim3 grid(p.blocks, p.q_blocks);
  const uint16_t* Xh = (const uint16_t*)X;
  const uint16_t* Qh = (const uint16_t*)Qpad;
  auto f = dtype == RFX_BF16 ? (D == 768 ? k3::launch_bf16_768 : k3::launch_bf16_1024)
                             : (D == 768 ? k3::launch_f16_768 : k3::launch_f16_1024);
  return f(p.k_lane, grid, st, Xh, nrows, Qh, nq, p.tiles_per_block, ntiles, tau, cs, cr, p.n_lists, mask);
}

}  // namespace rfx
