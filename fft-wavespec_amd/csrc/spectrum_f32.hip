// spectrum_f32.hip -- fp32 instantiations of the spectrum kernel for log2 N < 12 (C3 path: N = 4096 in
// spectrum_f32_hi.hip; detrend and window arithmetic stay fp64, see spectrum_core.h).
#include "spectrum_dispatch.h"

namespace wsp {

hipError_t launch_spectrum_f32(const SpectrumLaunch &L, hipStream_t stream) {
    if (L.log2n >= core::kSplitLog2N) return launch_spectrum_f32_hi(L, stream);
    return core::dispatch_n_range<float, core::kSetBase, 5, core::kSplitLog2N - 1>(L, stream);
}

}  // namespace wsp
