// k4_bf16_768.hip — instantiations of the all-query-stationary scan (k_scan_mfma4.h) for bf16, d=768.
#include "k_scan_mfma4.h"

namespace rfx {
namespace k4 {
RFX_K4_INSTANTIATE(RFX_BF16, 768, launch_bf16_768)
}  // namespace k4
}  // namespace rfx
