// spectrum_f64_hi.hip -- fp64 instantiations of the spectrum kernel for log2 N >= 12 (the north star's
// N = 4096 among them), a translation unit of its own so the library builds in parallel.
#include "spectrum_dispatch.h"

namespace wsp {

hipError_t launch_spectrum_f64_hi(const SpectrumLaunch &L, hipStream_t stream) {
    return core::dispatch_n_range<double, core::kSetBase, core::kSplitLog2N, kMaxLog2N>(L, stream);
}

}  // namespace wsp
