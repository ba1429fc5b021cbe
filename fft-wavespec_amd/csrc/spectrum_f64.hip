// spectrum_f64.hip -- fp64 instantiations of the spectrum kernel for log2 N < 12 + the precision and
// output switch of launch_spectrum (kernel design: spectrum_core.h; log2 N >= 12: spectrum_f64_hi.hip).
#include "spectrum_dispatch.h"

namespace wsp {

hipError_t launch_spectrum(const SpectrumLaunch &L, hipStream_t stream) {
    if (L.f32) return launch_spectrum_f32(L, stream);
    if (L.output == kOutPhase || L.output == kOutTopKPhase) return launch_spectrum_phase(L, stream);
    if (L.log2n >= core::kSplitLog2N) return launch_spectrum_f64_hi(L, stream);
    return core::dispatch_n_range<double, core::kSetBase, 5, core::kSplitLog2N - 1>(L, stream);
}

}  // namespace wsp
