// kalman_kernels.hip -- launch of the per-window Kalman 4D detrend pre-pass
// (device code and design notes: kalman_core.h).
#include "kalman_core.h"

namespace wsp {
using kcore::KP;
using kcore::kalman_detrend_kernel;

hipError_t launch_kalman_detrend(const KalmanLaunch &L, hipStream_t stream) {
    if (L.n_windows <= 0) return hipSuccess;
    KP kp;
    static_assert(sizeof(KP) == 16 * sizeof(double), "KP layout");
    __builtin_memcpy(&kp, L.params, sizeof(kp));
    // J = 32 (f32) / 16 (f64) steps per tile divides every window length >= 32.
    // Half-filled waves when one window per lane would leave a single wave per
    // SIMD (batches up to 256 CUs x 4 SIMDs x 64 lanes); L.variant overrides.
    const bool half = L.variant == 1 || (L.variant == 0 && L.n_windows <= 256LL * 4 * 64);
    const int wpw = half ? 32 : 64;
    const unsigned grid = (unsigned)((L.n_windows + wpw - 1) / wpw);
#define KLAUNCH(T, K, W)                                                                                          \
    hipLaunchKernelGGL((kalman_detrend_kernel<T, K, sizeof(T) == 4 ? 32 : 16, W, sizeof(T) == 4 ? 32 : 16>), dim3(grid), dim3(64), 0, stream, \
                       static_cast<const T *>(L.series), static_cast<T *>(L.detrended), L.hop, L.n_windows, L.n, kp)
    if (L.f32) {
        if (half) KLAUNCH(float, float, 32);
        else KLAUNCH(float, float, 64);
    } else {
        if (half) KLAUNCH(double, double, 32);
        else KLAUNCH(double, double, 64);
    }
#undef KLAUNCH
    return hipGetLastError();
}

}  // namespace wsp
