// k4_f16_768.hip — instantiations of the all-query-stationary scan (k_scan_mfma4.h) for f16, d=768.
#include "k_scan_mfma4.h"

namespace rfx {
namespace k4 {
RFX_K4_INSTANTIATE(RFX_F16, 768, launch_f16_768)
}  // namespace k4
}  // namespace rfx
