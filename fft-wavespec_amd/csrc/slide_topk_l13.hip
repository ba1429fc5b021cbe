// slide_topk_l13.hip -- hop = 1 top-k records by the sliding DFT at N = 8192 (own translation unit:
// parallel build).  Device code: sliding_core.h.
#include "sliding_core.h"

namespace wsp {
hipError_t launch_slide_topk_l13(const SlideArgs &a, hipStream_t s) { return topk_by_nf<13>(a, s); }
}  // namespace wsp
