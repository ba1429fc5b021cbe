// spectrum_phase.hip -- fp64 instantiations of the spectrum kernel with the
// phase outputs (kOutPhase: [P | unwrapped phase | group delay] rows;
// kOutTopKPhase: top-k records with the phase and delay of each bin).  A
// translation unit of its own so the instantiations compile in parallel.
#include "spectrum_dispatch.h"

namespace wsp {

hipError_t launch_spectrum_phase(const SpectrumLaunch &L, hipStream_t stream) {
    if (L.f32) return hipErrorInvalidValue;
    return core::dispatch_n<double, core::kSetPhase>(L, stream);
}

}  // namespace wsp
