// valu_bf16.hip — instantiation unit of the VALU fused scan (k_scan_valu.h) for bf16 indices.
#include "k_scan_valu.h"

namespace rfx {
int launch_valu_bf16(const ValuPlan& p, const void* X, int nrows, int D, const void* Qf, int nq, float* cs, int* cr,
                     hipStream_t st, const uint32_t* mask, uint32_t* tau, const FusedOut& fo) {
  return launch_valu_dt<RFX_BF16>(p, X, nrows, D, Qf, nq, cs, cr, st, mask, tau, fo);
}
}  // namespace rfx
