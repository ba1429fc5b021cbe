// slide_topk_l10.hip -- hop = 1 top-k records by the sliding DFT at N = 1024 (own translation unit:
// parallel build).  Device code: sliding_core.h.
#include "sliding_core.h"

namespace wsp {
hipError_t launch_slide_topk_l10(const SlideArgs &a, hipStream_t s) { return topk_by_nf<10>(a, s); }
}  // namespace wsp
