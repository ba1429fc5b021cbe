// spectrum_phase.hip -- fp64 instantiations of the spectrum kernel with the
// phase outputs (kOutPhase: [P | unwrapped phase | group delay] rows;
// kOutTopKPhase: top-k records with the phase and delay of each bin), log2 N < 12;
// log2 N >= 12 in spectrum_phase_hi.hip.  Translation units of their own so the
// instantiations compile in parallel.
#include "spectrum_dispatch.h"

namespace wsp {

hipError_t launch_spectrum_phase(const SpectrumLaunch &L, hipStream_t stream) {
    if (L.f32) return hipErrorInvalidValue;
    if (L.log2n >= core::kSplitLog2N) return launch_spectrum_phase_hi(L, stream);
    return core::dispatch_n_range<double, core::kSetPhase, 5, core::kSplitLog2N - 1>(L, stream);
}

}  // namespace wsp
