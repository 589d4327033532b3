// k5_dbg.hip — DEBUG BUILD ONLY (librfx_dbg.so, `make dbg`): profiling ablations of the
// headline scan kernel (k_scan_mfma5.h MODE bits), reached through rfx_dbg_scan_variant.
#include "k_scan_mfma5.h"

namespace rfx {
namespace k5 {
size_t tau_bytes_dbg(const MfmaPlan& p) { return (size_t)p.nq_pad * kTauW * sizeof(uint32_t); }
}  // namespace k5

// Profiling ablations (bf16, d 768, KL 10), MODE bit flags of scan_mfma5_kernel:
// 1 = no top-k epilogue, 2 = no MFMA, 8 = no corpus stream, 16 = count top-k slow-path entries
// (cand_r[0]), 64 = DMA pieces bunched after the barrier, 128 = fragment prefetch distance 1,
// 256 = corpus pieces all re-read tile 0.
int launch_scan_mfma5_dbg(const MfmaPlan& p, int mode, const void* X, int nrows, int dtype, const void* Qpad, int nq,
                          uint32_t* tau, float* cs, int* cr, hipStream_t st) {
  if (!p.ok) return -1;
  if (mode == 0) return launch_scan_mfma5(p, X, nrows, 768, dtype, Qpad, nq, tau, cs, cr, st, nullptr);  // production plan
  if (p.k_lane != 10) return -1;
  const int ntiles = (nrows + k5::kTM - 1) / k5::kTM;
  if (hipMemsetAsync(tau, 0, k5::tau_bytes_dbg(p), st) != hipSuccess) return -2;
  dim3 grid(p.blocks, p.q_blocks);
  const uint16_t* Xh = (const uint16_t*)X;
  const uint16_t* Qh = (const uint16_t*)Qpad;
#define RFX_K5_DBG(M)                                                                                  \
  case M:                                                                                              \
    hipLaunchKernelGGL((k5::scan_mfma5_kernel<RFX_BF16, 10, 768, M>), grid, dim3(512), 0, st, Xh, Qh, nq, \
                       ntiles, tau, cs, cr, p.n_lists, nullptr);                                       \
    break;
  switch (mode) {
    RFX_K5_DBG(0)
    RFX_K5_DBG(1)
    RFX_K5_DBG(3)
    RFX_K5_DBG(9)
    RFX_K5_DBG(16)
    RFX_K5_DBG(64)
    RFX_K5_DBG(128)
    RFX_K5_DBG(192)
    RFX_K5_DBG(512)
    RFX_K5_DBG(1024)
    RFX_K5_DBG(2048)
    RFX_K5_DBG(4096)
    RFX_K5_DBG(8192)
    RFX_K5_DBG(16384)
    RFX_K5_DBG(32768)
    RFX_K5_DBG(65536)
    RFX_K5_DBG(131072)
    RFX_K5_DBG(131073)
    RFX_K5_DBG(131081)
    RFX_K5_DBG(262153)
    RFX_K5_DBG(262144)
    RFX_K5_DBG(393216)
    RFX_K5_DBG(393225)
    RFX_K5_DBG(524288)
    RFX_K5_DBG(1048576)
    RFX_K5_DBG(1179648)
    RFX_K5_DBG(257)
    RFX_K5_DBG(4194304)
    RFX_K5_DBG(4194320)
    RFX_K5_DBG(8388608)
    RFX_K5_DBG(8388624)
    default:
      return -1;
  }
#undef RFX_K5_DBG
  return 0;
}

}  // namespace rfx
