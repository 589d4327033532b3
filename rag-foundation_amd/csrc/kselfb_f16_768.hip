// select + in-launch exact fallback (k_select_fb.h), f16 rows at d 768
#include "k_select_fb.h"
namespace rfx {
namespace selfb {
RFX_SELFB_INSTANTIATE(RFX_F16, launch_f16_768)
}  // namespace selfb
}  // namespace rfx
