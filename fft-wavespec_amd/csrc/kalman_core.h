// kalman_core.h -- device code of the per-window Kalman 4D detrend pre-pass.
// Included by kalman_kernels.hip (library launch) and tools/kbench.hip.
//
// Restates ResetKalmanState / StepKalman4D of
// L/WaveSpecZZ_1.0.3-pla-kalman-fast.mq5:2015-2125 with a per-window reset
// (north-star "per-window Kalman detrend", builder-defined: reset(x0), then
// trend_j = step(x_j), d_j = x_j - trend_j; the call discipline of the
// reference call site :3354-3360).
//
// The filter has data-dependent gain (adaptive Q boost and innovation clip
// depend on the innovation), so every window is a sequential N-step
// recurrence: one lane per window.  What makes it fast:
//  * LDS-staged tiles of J steps x 64 windows: global traffic is fully
//    coalesced (one row = J contiguous samples per wave instruction) and the
//    next tile is prefetched into registers while the lanes run the current one;
//  * the covariance is carried as the 10 entries of the symmetric P (the
//    reference's 16-entry expansion is algebraically symmetric: each P_ij
//    update equals P_ji's), ~40 % fewer operations per step;
//  * the state is centred on the window's first sample (z' = z - x0, pos' =
//    pos - x0): the filter is exactly shift-equivariant (innovation, gain,
//    boost and clip depend only on differences), and centring lets the fp32
//    plan run the filter in fp32 without cancelling against the price level.
// Output: d = x - trend rounded to the plan's element type, consumed by the
// spectrum kernel as a hop = N series.
#pragma once
#include "wsp_internal.h"

namespace wsp {
namespace kcore {

struct KP {
    double follow, qp, qv, qa, qj, adapt, r, vp, vv, va, vj, iv, ia, ij, clip, ema;
};

// 1/sqrt: hardware v_rsq_f32 for the fp32 filter (1 ulp), exact for fp64
__device__ __forceinline__ float krsqrt(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ double krsqrt(double x) { return 1.0 / sqrt(x); }

// WPW windows per wave (64, or 32 so that two waves share a SIMD and hide each
// other's dependency stalls when the batch has only one window per lane).
template <typename T, typename K, int J, int WPW, int UNROLL = 2>
__global__ __launch_bounds__(64) void kalman_detrend_kernel(const T *__restrict__ series, T *__restrict__ dout,
                                                            int64_t hop, int64_t n_windows, int n, KP kp) {
    __shared__ T tile[WPW * (J + 1)];  // [window row][step], +1 pad: conflict-free row walks
    const int l = threadIdx.x;
    const int64_t w0 = (int64_t)blockIdx.x * WPW;
    const bool lane_on = l < WPW;

    const K q_scale = (K)fmax(0.05, kp.follow);
    const K Qp = (K)fmax(1e-9, kp.qp * (double)q_scale), Qv = (K)fmax(1e-9, kp.qv * (double)q_scale);
    const K Qa = (K)fmax(1e-9, kp.qa * (double)q_scale), Qj = (K)fmax(1e-9, kp.qj * (double)q_scale);
    const K R = (K)fmax(1e-9, kp.r);
    const K adapt = (K)kp.adapt, clip = (K)kp.clip;
    const bool use_adapt = kp.adapt > 0.0, use_clip = kp.clip > 0.0, use_ema = kp.ema > 0.0;
    const K ema_a = use_ema ? (K)(2.0 / (kp.ema + 1.0)) : K(0);

    // ResetKalmanState(first_meas) :2015-2029, centred: pos' = 0
    K pos = 0, vel = (K)kp.iv, acc = (K)kp.ia, jerk = (K)kp.ij;
    K p00 = (K)fmax(1e-9, kp.vp), p11 = (K)fmax(1e-9, kp.vv), p22 = (K)fmax(1e-9, kp.va), p33 = (K)fmax(1e-9, kp.vj);
    K p01 = 0, p02 = 0, p03 = 0, p12 = 0, p13 = 0, p23 = 0;
    bool ema_ready = false;
    K ema_prev = 0;
    T x0 = 0;

    // tile rows are windows w0 .. w0+63; row r, step j of chunk c = series[(w0+r)*hop + c*J + j].
    // One wave instruction moves RPI rows of J contiguous samples (coalesced).
    constexpr int RPI = 64 / J, NI = WPW / RPI;
    const int lrow = l / J, lcol = l % J;
    T reg[NI];
    const int nchunks = n / J;
    auto issue = [&](int c) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int64_t w = w0 + i * RPI + lrow;
            reg[i] = series[(w < n_windows ? w : 0) * hop + (int64_t)c * J + lcol];
        }
    };
    issue(0);
    for (int c = 0; c < nchunks; ++c) {
#pragma unroll
        for (int i = 0; i < NI; ++i) tile[(i * RPI + lrow) * (J + 1) + lcol] = reg[i];
        __syncthreads();
        if (c + 1 < nchunks) issue(c + 1);  // next tile in flight while the lanes filter this one
        const int lr = lane_on ? l : 0;
        if (c == 0) x0 = tile[lr * (J + 1)];
        T zrow[J];  // this window's J samples in registers: no LDS latency inside the recurrence
#pragma unroll
        for (int j = 0; j < J; ++j) zrow[j] = tile[lr * (J + 1) + j];
#pragma unroll UNROLL
        for (int j = 0; j < J; ++j) {
            const T zt = zrow[j];
            const K z = (K)(zt - x0);  // exact for prices within 2x of x0 (Sterbenz)
            // StepKalman4D :2031-2125 on the symmetric covariance
            const K x0p = pos + vel + K(0.5) * acc + K(1.0 / 6.0) * jerk;
            const K x1p = vel + acc + K(0.5) * jerk;
            const K x2p = acc + jerk;
            const K x3p = jerk;
            K P00p = p00 + K(2) * p01 + p02 + K(1.0 / 3.0) * p03 + p11 + p12 + K(1.0 / 3.0) * p13 +
                     K(0.25) * p22 + K(1.0 / 6.0) * p23 + K(1.0 / 36.0) * p33 + Qp;
            const K P01p = p01 + p02 + K(0.5) * p03 + p11 + K(1.5) * p12 + K(2.0 / 3.0) * p13 + K(0.5) * p22 +
                           K(5.0 / 12.0) * p23 + K(1.0 / 12.0) * p33;
            const K P02p = p02 + p03 + p12 + p13 + K(0.5) * p22 + K(2.0 / 3.0) * p23 + K(1.0 / 6.0) * p33;
            const K P03p = p03 + p13 + K(0.5) * p23 + K(1.0 / 6.0) * p33;
            K P11p = p11 + K(3) * p12 + K(1.5) * p13 + K(2) * p22 + K(1.5) * p23 + K(0.25) * p33 + Qv;
            const K P12p = p12 + p13 + p22 + K(1.5) * p23 + K(0.5) * p33;
            const K P13p = p13 + p23 + K(0.5) * p33;
            K P22p = p22 + K(2) * p23 + p33 + Qa;
            const K P23p = p23 + p33;
            K P33p = p33 + Qj;

            K y = z - x0p;
            K S = P00p + R;
            if (use_adapt) {
                const K k = fmin(K(5), fabs(y) * krsqrt(S)) * adapt;  // boost - 1 = min(5,|y|/sigma) g
                P00p += k * Qp;
                P11p += k * Qv;
                P22p += k * Qa;
                P33p += k * Qj;
                S = P00p + R;
            }
            const K rs = krsqrt(S);
            if (use_clip) {
                const K lim = clip * (S * rs);  // clip * sqrt(S)
                y = fmin(fmax(y, -lim), lim);
            }
            const K inv = rs * rs;  // 1/S
            const K K0 = P00p * inv, K1 = P01p * inv, K2 = P02p * inv, K3 = P03p * inv;
            pos = x0p + K0 * y;
            vel = x1p + K1 * y;
            acc = x2p + K2 * y;
            jerk = x3p + K3 * y;
            // P_ij <- P_ij - K_i P_0j (symmetric), diagonal floors 1e-12
            p00 = fmax(K(1e-12), P00p - K0 * P00p);
            p01 = P01p - K1 * P00p;
            p02 = P02p - K2 * P00p;
            p03 = P03p - K3 * P00p;
            p11 = fmax(K(1e-12), P11p - K1 * P01p);
            p12 = P12p - K2 * P01p;
            p13 = P13p - K3 * P01p;
            p22 = fmax(K(1e-12), P22p - K2 * P02p);
            p23 = P23p - K3 * P02p;
            p33 = fmax(K(1e-12), P33p - K3 * P03p);

            K trend = pos;
            if (use_ema) {  // :2117-2123
                if (!ema_ready) {
                    ema_prev = trend;
                    ema_ready = true;
                }
                ema_prev = ema_a * trend + (K(1) - ema_a) * ema_prev;
                trend = ema_prev;
            }
            zrow[j] = T(z - trend);
        }
        if (lane_on) {
#pragma unroll
            for (int j = 0; j < J; ++j) tile[l * (J + 1) + j] = zrow[j];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int64_t w = w0 + i * RPI + lrow;
            if (w < n_windows) dout[w * (int64_t)n + (int64_t)c * J + lcol] = tile[(i * RPI + lrow) * (J + 1) + lcol];
        }
        __syncthreads();
    }
}

}  // namespace kcore

}  // namespace wsp
