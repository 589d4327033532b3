// k5_f16_768.hip — instantiations of the two-waves-per-SIMD scan (k_scan_mfma5.h) for f16, d=768.
#include "k_scan_mfma5.h"

namespace rfx {
namespace k5 {
RFX_K5_INSTANTIATE(RFX_F16, 768, launch_f16_768)
}  // namespace k5
}  // namespace rfx
