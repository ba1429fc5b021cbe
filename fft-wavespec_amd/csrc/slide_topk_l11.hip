// slide_topk_l11.hip -- hop = 1 top-k records by the sliding DFT at N = 2048 (own translation unit:
// parallel build).  Device code: sliding_core.h.
#include "sliding_core.h"

namespace wsp {
hipError_t launch_slide_topk_l11(const SlideArgs &a, hipStream_t s) { return topk_by_nf<11>(a, s); }
}  // namespace wsp
