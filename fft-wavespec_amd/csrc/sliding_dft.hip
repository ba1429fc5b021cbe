// sliding_dft.hip -- hop = 1 batches by a seeded sliding DFT (gfx950): the library's entry points
// (power rows of one series or of a group of series, top-k records) and the fp64 power kernels.
// Device code and design notes: sliding_core.h.
#include "sliding_core.h"

namespace wsp {

hipError_t launch_slide_topk(const SlideArgs &a, hipStream_t s) {
    if (a.n_windows <= 0) return hipSuccess;
    if (a.f32 || a.seg < 1 || a.span < 1 || a.span > kSlideTopkMaxSpan || a.kmin < 0 || a.kmin + a.span > (1 << a.log2n) / 2 ||
        a.topk < 1 || a.topk > 64 || !a.ws)
        return hipErrorInvalidValue;
    switch (a.log2n) {
    case 9: return launch_slide_topk_l9(a, s);
    case 10: return launch_slide_topk_l10(a, s);
    case 11: return launch_slide_topk_l11(a, s);
    case 12: return launch_slide_topk_l12(a, s);
    case 13: return launch_slide_topk_l13(a, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_slide(const SlideArgs &a, hipStream_t s) {
    if (a.n_windows <= 0) return hipSuccess;
    SlideGroup g;
    g.n = 1;
    g.series[0] = a.series;
    g.out[0] = a.out;
    g.n_windows[0] = a.n_windows;
    return launch_slide_group(a, g, s);
}

hipError_t launch_slide_group(const SlideArgs &a, const SlideGroup &g, hipStream_t s) {
    if (g.n < 1 || g.n > kSlideGroupMax || a.log2n < kSlideMinLog2N || a.log2n > kSlideMaxLog2N)
        return hipErrorInvalidValue;
    for (int m = 0; m < g.n; ++m)
        if (g.n_windows[m] < 0 || !g.series[m] || !g.out[m]) return hipErrorInvalidValue;
    return a.f32 ? launch_slide_group_f32(a, g, s) : launch_slide_group_f64(a, g, s);
}

hipError_t launch_slide_group_f64(const SlideArgs &a, const SlideGroup &g, hipStream_t s) { return by_n<double>(a, g, s); }

}  // namespace wsp
