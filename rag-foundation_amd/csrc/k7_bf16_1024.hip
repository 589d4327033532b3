// k7_bf16_1024.hip — instantiation unit of the d = 1024 scan kernel (k_scan_mfma7.h) for bf16 rows.
#include "k_scan_mfma7.h"

namespace rfx {
namespace k7 {
RFX_K7_INSTANTIATE(RFX_BF16, 1024, launch_bf16_1024)
}  // namespace k7
}  // namespace rfx
