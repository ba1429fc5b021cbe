// kalman_kernels.hip -- per-window Kalman 4D detrend pre-pass (gfx950).
//
// Restates ResetKalmanState / StepKalman4D of
// L/WaveSpecZZ_1.0.3-pla-kalman-fast.mq5:2015-2125 with a per-window reset
// (north-star "per-window Kalman detrend", builder-defined: reset(x0), then
// trend_j = step(x_j), d_j = x_j - trend_j; same call discipline as the
// reference call site :3354-3360).
//
// The filter is a data-dependent sequential recurrence (adaptive Q boost and
// innovation clipping depend on the innovation), so it runs one lane per
// window, in fp64 like the MQL5 source.  Its output -- the detrended window,
// rounded to the plan's element type -- feeds the spectrum kernel as a
// hop = N series.  See DESIGN.md "Kalman detrend" for why this is a
// separate pass and what fusing it would take.
#include "wsp_internal.h"

namespace wsp {
namespace {

struct KP {
    double follow, qp, qv, qa, qj, adapt, r, vp, vv, va, vj, iv, ia, ij, clip, ema;
};

template <typename T>
__global__ __launch_bounds__(64) void kalman_detrend_kernel(const T *__restrict__ series, T *__restrict__ dout,
                                                            int64_t hop, int64_t n_windows, int n, KP kp) {
    const int64_t w = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (w >= n_windows) return;
    const T *__restrict__ x = series + w * hop;
    T *__restrict__ d = dout + w * (int64_t)n;

    const double q_scale = fmax(0.05, kp.follow);
    const double Qp = fmax(1e-9, kp.qp * q_scale);
    const double Qv = fmax(1e-9, kp.qv * q_scale);
    const double Qa = fmax(1e-9, kp.qa * q_scale);
    const double Qj = fmax(1e-9, kp.qj * q_scale);
    const double R = fmax(1e-9, kp.r);

    // ResetKalmanState(first_meas) :2015-2029
    double pos = (double)x[0], vel = kp.iv, acc = kp.ia, jerk = kp.ij;
    double P00 = fmax(1e-9, kp.vp), P11 = fmax(1e-9, kp.vv), P22 = fmax(1e-9, kp.va), P33 = fmax(1e-9, kp.vj);
    double P01 = 0, P02 = 0, P03 = 0, P10 = 0, P12 = 0, P13 = 0, P20 = 0, P21 = 0, P23 = 0, P30 = 0, P31 = 0, P32 = 0;
    bool ema_ready = false;
    double ema_prev = 0.0;
    const double ema_alpha = kp.ema > 0.0 ? 2.0 / (kp.ema + 1.0) : 0.0;

    for (int j = 0; j < n; ++j) {
        const double z = (double)x[j];
        // StepKalman4D :2031-2125, expression order of the MQL5 source
        const double x0p = pos + vel + 0.5 * acc + (1.0 / 6.0) * jerk;
        const double x1p = vel + acc + 0.5 * jerk;
        const double x2p = acc + jerk;
        const double x3p = jerk;
        double P00p = P00 + P01 + 0.5 * P02 + (1.0 / 6.0) * P03 + P10 + P11 + 0.5 * P12 + (1.0 / 6.0) * P13 +
                      0.5 * P20 + 0.5 * P21 + 0.25 * P22 + (1.0 / 12.0) * P23 + (1.0 / 6.0) * P30 +
                      (1.0 / 6.0) * P31 + (1.0 / 12.0) * P32 + (1.0 / 36.0) * P33 + Qp;
        const double P01p = P01 + P02 + 0.5 * P03 + P11 + P12 + 0.5 * P13 + 0.5 * P21 + 0.5 * P22 + 0.25 * P23 +
                            (1.0 / 6.0) * P31 + (1.0 / 6.0) * P32 + (1.0 / 12.0) * P33;
        const double P02p = P02 + P03 + P12 + P13 + 0.5 * P22 + 0.5 * P23 + (1.0 / 6.0) * P32 + (1.0 / 6.0) * P33;
        const double P03p = P03 + P13 + 0.5 * P23 + (1.0 / 6.0) * P33;
        double P11p = P11 + 2.0 * P12 + P13 + P21 + 2.0 * P22 + P23 + 0.5 * P31 + 0.5 * P32 + 0.25 * P33 + Qv;
        const double P12p = P12 + P13 + P22 + P23 + 0.5 * P32 + 0.5 * P33;
        const double P13p = P13 + P23 + 0.5 * P33;
        double P22p = P22 + 2.0 * P23 + P33 + Qa;
        const double P23p = P23 + P33;
        double P33p = P33 + Qj;
        const double P10p = P01p, P20p = P02p, P30p = P03p;
        const double P21p = P12p, P31p = P13p, P32p = P23p;

        double y = z - x0p;
        double S = P00p + R;
        if (kp.adapt > 0.0) {
            const double sigma = sqrt(S);
            const double k = fmin(5.0, fabs(y) / sigma) * kp.adapt;
            const double boost = 1.0 + k;
            P00p += (boost - 1.0) * Qp;
            P11p += (boost - 1.0) * Qv;
            P22p += (boost - 1.0) * Qa;
            P33p += (boost - 1.0) * Qj;
            S = P00p + R;
        }
        if (kp.clip > 0.0) {
            const double lim = kp.clip * sqrt(S);
            if (y > lim) y = lim;
            if (y < -lim) y = -lim;
        }
        const double K0 = P00p / S, K1 = P10p / S, K2 = P20p / S, K3 = P30p / S;
        pos = x0p + K0 * y;
        vel = x1p + K1 * y;
        acc = x2p + K2 * y;
        jerk = x3p + K3 * y;

        P00 = fmax(1e-12, (1.0 - K0) * P00p);
        P01 = (1.0 - K0) * P01p;
        P02 = (1.0 - K0) * P02p;
        P03 = (1.0 - K0) * P03p;
        P10 = P10p - K1 * P00p;
        P11 = fmax(1e-12, P11p - K1 * P01p);
        P12 = P12p - K1 * P02p;
        P13 = P13p - K1 * P03p;
        P20 = P20p - K2 * P00p;
        P21 = P21p - K2 * P01p;
        P22 = fmax(1e-12, P22p - K2 * P02p);
        P23 = P23p - K2 * P03p;
        P30 = P30p - K3 * P00p;
        P31 = P31p - K3 * P01p;
        P32 = P32p - K3 * P02p;
        P33 = fmax(1e-12, P33p - K3 * P03p);

        double trend = pos;
        if (kp.ema > 0.0) {  // :2117-2123
            if (!ema_ready) { ema_prev = trend; ema_ready = true; }
            ema_prev = ema_alpha * trend + (1.0 - ema_alpha) * ema_prev;
            trend = ema_prev;
        }
        d[j] = T(z - trend);
    }
}

}  // namespace

hipError_t launch_kalman_detrend(const KalmanLaunch &L, hipStream_t stream) {
    if (L.n_windows <= 0) return hipSuccess;
    KP kp;
    static_assert(sizeof(KP) == 16 * sizeof(double), "KP layout");
    __builtin_memcpy(&kp, L.params, sizeof(kp));
    const unsigned grid = (unsigned)((L.n_windows + 63) / 64);
    if (L.f32)
        hipLaunchKernelGGL(kalman_detrend_kernel<float>, dim3(grid), dim3(64), 0, stream,
                           static_cast<const float *>(L.series), static_cast<float *>(L.detrended), L.hop,
                           L.n_windows, L.n, kp);
    else
        hipLaunchKernelGGL(kalman_detrend_kernel<double>, dim3(grid), dim3(64), 0, stream,
                           static_cast<const double *>(L.series), static_cast<double *>(L.detrended), L.hop,
                           L.n_windows, L.n, kp);
    return hipGetLastError();
}

}  // namespace wsp
