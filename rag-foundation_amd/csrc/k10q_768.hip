// k10q_768.hip — instantiation unit of the 64-queries-per-wave int8 screen kernel (k_scan_screen64.h), d 768.
#include "k_scan_screen64.h"

namespace rfx {
namespace k10q {
RFX_K10Q_INSTANTIATE(768, kRing768, launch_768)
}  // namespace k10q
}  // namespace rfx
