// k3_f16_1024.hip — instantiations of the query-stationary scan (k_scan_mfma3.h) for f16, d=1024.
#include "k_scan_mfma3.h"

namespace rfx {
namespace k3 {
RFX_K3_INSTANTIATE(RFX_F16, 1024, launch_f16_1024)
}  // namespace k3
}  // namespace rfx
