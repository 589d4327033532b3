// k10w2_1024.hip — instantiation unit of the 2-wave int8 screen kernel (k_scan_screen.h: 64 queries per
// workgroup, the micro-batches of 9..64 questions) for d 1024.
#include "k_scan_screen.h"

namespace rfx {
namespace k10 {
RFX_K10_INSTANTIATE_W2(1024, launch_1024_w2)
}  // namespace k10
}  // namespace rfx
