// slide_power_f32.hip -- fp32 power rows of the hop = 1 sliding DFT (own translation unit: parallel build).
#include "sliding_core.h"

namespace wsp {
hipError_t launch_slide_group_f32(const SlideArgs &a, const SlideGroup &g, hipStream_t s) { return by_n<float>(a, g, s); }
}  // namespace wsp
