// spectrum_f64.hip -- fp64 instantiations of the spectrum kernel + the
// precision switch of launch_spectrum (kernel design: spectrum_core.h).
#include "spectrum_dispatch.h"

namespace wsp {

hipError_t launch_spectrum(const SpectrumLaunch &L, hipStream_t stream) {
    if (L.f32) return launch_spectrum_f32(L, stream);
    if (L.output == kOutPhase || L.output == kOutTopKPhase) return launch_spectrum_phase(L, stream);
    return core::dispatch_n<double>(L, stream);
}

}  // namespace wsp
