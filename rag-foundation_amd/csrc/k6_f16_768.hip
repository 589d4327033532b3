// k6_f16_768.hip — instantiation unit of the headline scan kernel (k_scan_mfma6.h) for f16 rows, d 768.
#include "k_scan_mfma6.h"

namespace rfx {
namespace k6 {
RFX_K6_INSTANTIATE(RFX_F16, 768, launch_f16_768)
}  // namespace k6
}  // namespace rfx
