// select + in-launch exact fallback (k_select_fb.h), bf16 rows at d 768
#include "k_select_fb.h"
namespace rfx {
namespace selfb {
RFX_SELFB_INSTANTIATE(RFX_BF16, launch_bf16_768)
}  // namespace selfb
}  // namespace rfx
