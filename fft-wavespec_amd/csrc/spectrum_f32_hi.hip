// spectrum_f32_hi.hip -- fp32 instantiations of the spectrum kernel for log2 N >= 12 (C3's N = 4096).
#include "spectrum_dispatch.h"

namespace wsp {

hipError_t launch_spectrum_f32_hi(const SpectrumLaunch &L, hipStream_t stream) {
    return core::dispatch_n_range<float, core::kSetBase, core::kSplitLog2N, kMaxLog2N>(L, stream);
}

}  // namespace wsp
