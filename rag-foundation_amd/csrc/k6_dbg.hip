// k6_dbg.hip — DEBUG BUILD ONLY (librfx_dbg.so, `make dbg`): ablations of the headline scan kernel
// (k_scan_mfma6.h MODE bits: 1 no top-k epilogue, 8 no corpus stream), via rfx_dbg_scan_variant.
#include "k_scan_mfma6.h"

namespace rfx {

int launch_scan_mfma6_dbg(const MfmaPlan& p, int mode, const void* X, int nrows, int dtype, const void* Qpad, int nq,
                          uint32_t* tau, float* cs, int* cr, hipStream_t st) {
  if (!p.ok || dtype != RFX_BF16) return -1;
  if (mode == 0) return launch_scan_mfma6(p, X, nrows, 768, dtype, Qpad, nq, tau, cs, cr, st, nullptr);
  if (mode == 70 || mode == 71) {  // lane lists of 4 (k <= 4) with a 6- or 7-slot ring
    if (p.k_lane != 4) return -1;
    const int ntiles = (nrows + k6::kTM - 1) / k6::kTM;
    if (hipMemsetAsync(tau, 0, (size_t)p.nq_pad * k6::kTauW * sizeof(uint32_t), st) != hipSuccess) return -2;
    const uint16_t* Xh = (const uint16_t*)X;
    const uint16_t* Qh = (const uint16_t*)Qpad;
    if (mode == 70)
      hipLaunchKernelGGL((k6::scan_mfma6_kernel<RFX_BF16, 4, 768, 0, 6>), dim3(p.blocks, p.q_blocks), dim3(512), 0, st,
                         Xh, Qh, nq, ntiles, tau, cs, cr, p.n_lists, nullptr, nullptr);
    else
      hipLaunchKernelGGL((k6::scan_mfma6_kernel<RFX_BF16, 4, 768, 0, 7>), dim3(p.blocks, p.q_blocks), dim3(512), 0, st,
                         Xh, Qh, nq, ntiles, tau, cs, cr, p.n_lists, nullptr, nullptr);
    return 0;
  }
  if (p.k_lane != 10) return -1;
  const int ntiles = (nrows + k6::kTM - 1) / k6::kTM;
  if (hipMemsetAsync(tau, 0, (size_t)p.nq_pad * k6::kTauW * sizeof(uint32_t), st) != hipSuccess) return -2;
  dim3 grid(p.blocks, p.q_blocks);
  const uint16_t* Xh = (const uint16_t*)X;
  const uint16_t* Qh = (const uint16_t*)Qpad;
#define RFX_K6_DBG(M)                                                                                  \
  case M:                                                                                              \
    hipLaunchKernelGGL((k6::scan_mfma6_kernel<RFX_BF16, 10, 768, M>), grid, dim3(512), 0, st, Xh, Qh, nq, \
                       ntiles, tau, cs, cr, p.n_lists, nullptr, nullptr);                                       \
    break;
  switch (mode) {
    RFX_K6_DBG(1)
    RFX_K6_DBG(8)
    RFX_K6_DBG(9)
    RFX_K6_DBG(16)
    RFX_K6_DBG(32)
    RFX_K6_DBG(48)
    RFX_K6_DBG(41)
    RFX_K6_DBG(64)
    RFX_K6_DBG(256)
    RFX_K6_DBG(320)
    RFX_K6_DBG(512)
    RFX_K6_DBG(1024)

    default:
      return -1;
  }
#undef RFX_K6_DBG
  return 0;
}

}  // namespace rfx
