// kalman_kernels.hip -- launch of the per-window Kalman 4D detrend pre-pass
// (device code and design notes: kalman_core.h).
#include "kalman_core.h"

namespace wsp {
using kcore::KP;
using kcore::kalman_detrend_kernel;

namespace {

int cu_count() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 256;
    return cus > 0 ? cus : 256;
}

// One lane per window, 64 windows per wave.  Up to one wave per SIMD
// (4 x CUs x 64 windows) every SIMD gets exactly one wave: 4-wave workgroups
// with an LDS reservation that admits one workgroup per CU.  Larger batches
// use single-wave workgroups so that two waves can share a SIMD.
template <typename T, int FL> hipError_t launch_t(const KalmanLaunch &L, const KP &kp, hipStream_t stream) {
    constexpr int J = sizeof(T) == 4 ? 32 : 16;  // steps per tile; divides every window length >= 32
    constexpr size_t kStatic = 4 * 64 * (J + 1) * sizeof(T);
    const int cus = cu_count();
    const bool spread = L.variant != 1 && L.n_windows <= 4LL * 64 * cus;
    if (spread) {
        const size_t reserve = 84 * 1024 - kStatic;  // > half of the CU's 160 KiB: one workgroup per CU
        const unsigned grid = (unsigned)((L.n_windows + 255) / 256);
        hipLaunchKernelGGL((kalman_detrend_kernel<T, T, J, 64, J, FL, true, 4, true>), dim3(grid), dim3(256), reserve, stream,
                           static_cast<const T *>(L.series), static_cast<T *>(L.detrended), L.hop, L.n_windows, L.n, kp,
                           (unsigned *)nullptr);
    } else {
        const unsigned grid = (unsigned)((L.n_windows + 63) / 64);
        hipLaunchKernelGGL((kalman_detrend_kernel<T, T, J, 64, J, FL, true, 1, true>), dim3(grid), dim3(64), 0, stream,
                           static_cast<const T *>(L.series), static_cast<T *>(L.detrended), L.hop, L.n_windows, L.n, kp,
                           (unsigned *)nullptr);
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_kalman_detrend(const KalmanLaunch &L, hipStream_t stream) {
    if (L.n_windows <= 0) return hipSuccess;
    KP kp;
    static_assert(sizeof(KP) == 16 * sizeof(double), "KP layout");
    __builtin_memcpy(&kp, L.params, sizeof(kp));
    // the reference defaults (adaptive boost + clip, no EMA) run branch-free;
    // other flag sets read them per step.  L.variant = 1 forces single-wave
    // workgroups (ablation).
    constexpr int kFixed = kcore::kKfAdapt | kcore::kKfClip;
    const bool fixed = kcore::kalman_flags(kp) == kFixed;
    if (L.f32) return fixed ? launch_t<float, kFixed>(L, kp, stream) : launch_t<float, kcore::kKfRuntime>(L, kp, stream);
    return fixed ? launch_t<double, kFixed>(L, kp, stream) : launch_t<double, kcore::kKfRuntime>(L, kp, stream);
}

}  // namespace wsp
