// k8_f16_1024.hip — instantiation unit of the k-split d = 1024 scan kernel (k_scan_mfma8.h) for f16 rows.
#include "k_scan_mfma8.h"

namespace rfx {
namespace k8 {
RFX_K8_INSTANTIATE(RFX_F16, 1024, launch_f16_1024)
}  // namespace k8
}  // namespace rfx
