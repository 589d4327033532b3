// k9_f32_768.hip — instantiation unit of the batched f32 scan kernel (k_scan_mfma9.h), d 768.
#include "k_scan_mfma9.h"

namespace rfx {
namespace k9 {
RFX_K9_INSTANTIATE(768, launch_f32_768)
}  // namespace k9
}  // namespace rfx
