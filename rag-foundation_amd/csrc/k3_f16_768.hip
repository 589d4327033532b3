// k3_f16_768.hip — instantiations of the query-stationary scan (k_scan_mfma3.h) for f16, d=768.
#include "k_scan_mfma3.h"

namespace rfx {
namespace k3 {
RFX_K3_INSTANTIATE(RFX_F16, 768, launch_f16_768)
}  // namespace k3
}  // namespace rfx
