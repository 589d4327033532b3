// k5_bf16_768.hip — instantiations of the two-waves-per-SIMD scan (k_scan_mfma5.h) for bf16, d=768.
#include "k_scan_mfma5.h"

namespace rfx {
namespace k5 {
RFX_K5_INSTANTIATE(RFX_BF16, 768, launch_bf16_768)
}  // namespace k5
}  // namespace rfx
