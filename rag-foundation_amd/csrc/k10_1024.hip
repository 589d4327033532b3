// k10_1024.hip — instantiation unit of the int8 screen kernel (k_scan_screen.h) for d 1024.
#include "k_scan_screen.h"

namespace rfx {
namespace k10 {
RFX_K10_INSTANTIATE(1024, launch_1024)
}  // namespace k10
}  // namespace rfx
