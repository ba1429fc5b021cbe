// spectrum_f64.hip -- fp64 instantiations of the spectrum kernel + the
// precision switch of launch_spectrum (kernel design: spectrum_core.h).
#include "spectrum_dispatch.h"

namespace wsp {

hipError_t launch_spectrum(const SpectrumLaunch &L, hipStream_t stream) {
    return L.f32 ? launch_spectrum_f32(L, stream) : core::dispatch_n<double>(L, stream);
}

}  // namespace wsp
