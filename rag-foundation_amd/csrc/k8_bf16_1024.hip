// k8_bf16_1024.hip — instantiation unit of the k-split d = 1024 scan kernel (k_scan_mfma8.h) for bf16 rows.
#include "k_scan_mfma8.h"

namespace rfx {
namespace k8 {
RFX_K8_INSTANTIATE(RFX_BF16, 1024, launch_bf16_1024)
}  // namespace k8
}  // namespace rfx
