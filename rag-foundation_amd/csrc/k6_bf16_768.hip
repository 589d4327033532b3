// k6_bf16_768.hip — instantiation unit of the headline scan kernel (k_scan_mfma6.h) for bf16 rows, d 768.
#include "k_scan_mfma6.h"

namespace rfx {
namespace k6 {
RFX_K6_INSTANTIATE(RFX_BF16, 768, launch_bf16_768)
}  // namespace k6
}  // namespace rfx
