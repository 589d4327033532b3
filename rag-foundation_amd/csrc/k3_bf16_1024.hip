// k3_bf16_1024.hip — instantiations of the query-stationary scan (k_scan_mfma3.h) for bf16, d=1024.
#include "k_scan_mfma3.h"

namespace rfx {
namespace k3 {
RFX_K3_INSTANTIATE(RFX_BF16, 1024, launch_bf16_1024)
}  // namespace k3
}  // namespace rfx
