// k10_768.hip — instantiation unit of the int8 screen kernel (k_scan_screen.h) for d 768.
#include "k_scan_screen.h"

namespace rfx {
namespace k10 {
RFX_K10_INSTANTIATE(768, launch_768)
}  // namespace k10
}  // namespace rfx
