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

// fp32 plans with the reference default flags: two time segments per lane as packed pairs
// (kalman_pk2_kernel), stepped in the Newton basis when the floor guard's premises hold (nb2_ok).  Single-wave workgroups: at ~300 VGPRs a SIMD holds one wave of it anyway,
// so the dispatcher cannot stack two on one SIMD, and no wave waits at another's barrier
// (kalman_bench time, C3: 0.55-0.58 ms against 0.60-0.65 ms for 4-wave workgroups, 0.78-0.81 ms
// for the four-segment lane-pair kernel at two waves per SIMD, 0.69 ms sequential).
constexpr int kFoldMaxPairs = 2176;  // window pairs in LDS: N <= 4096 (17 KiB beside the 17 KiB tile, 4 waves per CU)

hipError_t launch_pk2(const KalmanLaunch &L, const KP &kp, hipStream_t stream) {
    const dim3 grid((unsigned)((L.n_windows + 63) / 64));
    const bool fold = kalman_folds_window(L);
    int l0 = 0, seg_off = 0;
    kalman_pair_geometry(L.n, &l0, &seg_off);
    const size_t lds = fold ? (size_t)l0 * 2 * sizeof(float) : 0;
    auto args = [&](auto kernel) {
        hipLaunchKernelGGL(kernel, grid, dim3(64), lds, stream, static_cast<const float *>(L.series),
                           static_cast<float *>(L.detrended), L.hop, L.n_windows, L.n, kp, (unsigned *)nullptr,
                           fold ? L.window_pairs : (const float *)nullptr);
    };
    if (L.variant == 7)  // the detrended rows written through to memory (A/B, round 5)
        args(kcore::kalman_pk2_kernel<32, 1, kcore::kPk2Warm, true, 16>);
    else if (L.variant == 8 || !kcore::nb2_ok(kp))  // the original basis with the reference's floors
        args(kcore::kalman_pk2_kernel<32, 1>);
    else  // the Newton basis, floors proven no-ops (guarded; kalman_core.h kstep_nb2)
        args(kcore::kalman_pk2_kernel<32, 1, kcore::kPk2Warm, true, 0, 1>);
    return hipGetLastError();
}

bool pk2_path(const KalmanLaunch &L, const KP &kp) {
    constexpr int kFixed = kcore::kKfAdapt | kcore::kKfClip;
    return L.f32 && kcore::kalman_flags(kp) == kFixed && (L.variant == 0 || L.variant == 7 || L.variant == 8 || L.variant == 9) &&
           kcore::pk2_fits(L.n);
}

}  // namespace

void kalman_pair_geometry(int n, int *l0, int *seg_off) {
    *l0 = (n + kcore::kPk2Warm) / 2;
    *seg_off = *l0 - kcore::kPk2Warm;
}

bool kalman_folds_window(const KalmanLaunch &L) {
    if (!L.window_pairs || L.n_windows <= 0) return false;
    KP kp;
    __builtin_memcpy(&kp, L.params, sizeof(kp));
    int l0 = 0, seg_off = 0;
    kalman_pair_geometry(L.n, &l0, &seg_off);
    return pk2_path(L, kp) && l0 <= kFoldMaxPairs;
}

hipError_t launch_kalman_detrend(const KalmanLaunch &L, hipStream_t stream) {
    if (L.n_windows <= 0) return hipSuccess;
    KP kp;
    static_assert(sizeof(KP) == 16 * sizeof(double), "KP layout");
    __builtin_memcpy(&kp, L.params, sizeof(kp));
    // the reference defaults (adaptive boost + clip, no EMA) run branch-free;
    // other flag sets read them per step.  fp32 default-flag plans of N >= 1024
    // run two time segments per lane (kalman_pk2_kernel, Newton basis).  L.variant = 1 forces
    // single-wave workgroups, 2 the sequential fp32 filter, 8 the two-segment filter in the
    // original basis (ablations).
    constexpr int kFixed = kcore::kKfAdapt | kcore::kKfClip;
    const bool fixed = kcore::kalman_flags(kp) == kFixed;
    if (L.f32) {
        if (pk2_path(L, kp)) return launch_pk2(L, kp, stream);
        return fixed ? launch_t<float, kFixed>(L, kp, stream) : launch_t<float, kcore::kKfRuntime>(L, kp, stream);
    }
    return fixed ? launch_t<double, kFixed>(L, kp, stream) : launch_t<double, kcore::kKfRuntime>(L, kp, stream);
}

}  // namespace wsp
