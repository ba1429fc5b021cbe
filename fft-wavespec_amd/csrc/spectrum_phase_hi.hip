// spectrum_phase_hi.hip -- the phase outputs' instantiations for log2 N >= 12 (ns_phase, ns_topk_phase).
#include "spectrum_dispatch.h"

namespace wsp {

hipError_t launch_spectrum_phase_hi(const SpectrumLaunch &L, hipStream_t stream) {
    return core::dispatch_n_range<double, core::kSetPhase, core::kSplitLog2N, kMaxLog2N>(L, stream);
}

}  // namespace wsp
