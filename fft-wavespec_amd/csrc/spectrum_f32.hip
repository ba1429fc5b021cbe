// spectrum_f32.hip -- fp32 instantiations of the spectrum kernel (C3 path;
// detrend and window arithmetic stay fp64, see spectrum_core.h).
#include "spectrum_dispatch.h"

namespace wsp {

hipError_t launch_spectrum_f32(const SpectrumLaunch &L, hipStream_t stream) {
    return core::dispatch_n<float>(L, stream);
}

}  // namespace wsp
