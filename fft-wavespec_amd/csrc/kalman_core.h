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
#include <type_traits>

#include "wsp_internal.h"

namespace wsp {
namespace kcore {

struct KP {
    double follow, qp, qv, qa, qj, adapt, r, vp, vv, va, vj, iv, ia, ij, clip, ema;
};

// 1/sqrt: hardware v_rsq_f32 for the fp32 filter (1 ulp), exact for fp64
__device__ __forceinline__ float krsqrt(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ double krsqrt(double x) { return 1.0 / sqrt(x); }
// clamp to [-lim, lim]: one v_med3_f32 for the fp32 filter
__device__ __forceinline__ float kclamp(float y, float lim) { return __builtin_amdgcn_fmed3f(y, -lim, lim); }
__device__ __forceinline__ double kclamp(double y, double lim) { return fmin(fmax(y, -lim), lim); }

// Tile IO through buffer descriptors based at the workgroup's first window:
// 32-bit lane offsets (no 64-bit address VALU per access), and the
// descriptor's range check (on the lane offset, which carries the row) drops
// stores to rows past the batch end instead of a branch per row; loads of such
// rows read 0 or in-range samples that no output uses.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t kbuf(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float kload(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, float) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0));
}
__device__ __forceinline__ double kload(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, double) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0));
}
__device__ __forceinline__ void kstore(float v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)voff, (int)soff, 0);
}
__device__ __forceinline__ void kstore(double v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, (int)voff, (int)soff, 0);
}

// Filter flags as a compile-time constant (FL >= 0: bit 0 adaptive Q boost,
// bit 1 innovation clip, bit 2 EMA blend) remove the per-step uniform branches
// so the scheduler can interleave consecutive steps; FL = -1 reads them from KP.
enum : int { kKfAdapt = 1, kKfClip = 2, kKfEma = 4, kKfRuntime = -1 };

inline int kalman_flags(const KP &kp) {
    return (kp.adapt > 0.0 ? kKfAdapt : 0) | (kp.clip > 0.0 ? kKfClip : 0) | (kp.ema > 0.0 ? kKfEma : 0);
}

// WPW windows per wave (64, or 32 so that two waves share a SIMD and hide each
// other's dependency stalls when the batch has only one window per lane).
// PKUP (fp32 filter): the update in normalised form, g = P_0./sqrt(S), with
// the state and covariance updates as packed pairs (v_pk_fma_f32), about 10
// fewer instructions per step (0.743 -> 0.678 ms at C3).
// TWO: predicted covariance through A = F P in two stages (32 instead of 41
// add/fma; F is the constant-jerk transition, P symmetric) instead of the
// reference's expanded sums -- same values, including the reference's
// extra terms in P11.
// WAVES: independent waves per workgroup (each its own WPW windows and LDS
// tile).  With WAVES = 4 and an LDS reservation that admits one workgroup per
// CU, a batch of at most 64 windows per SIMD runs exactly one wave on every
// SIMD; single-wave workgroups may be stacked two to a SIMD by the dispatcher
// while other SIMDs idle (measured: 0.76 ms back-to-back, 1.1 ms after a
// spectrum launch at C3).
template <typename T, typename K, int J, int WPW, int UNROLL = 2, int FL = kKfRuntime, bool TWO = false, int WAVES = 1,
          bool PKUP = false>
__global__ __launch_bounds__(64 * WAVES) void kalman_detrend_kernel(const T *__restrict__ series, T *__restrict__ dout,
                                                                    int64_t hop, int64_t n_windows, int n, KP kp) {
    __shared__ T tiles[WAVES][WPW * (J + 1)];  // per wave: [window row][step], +1 pad: conflict-free row walks
    // wave index through readfirstlane: provably uniform, so the descriptors stay scalar
    const int l = threadIdx.x % 64, wv = WAVES > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x / 64) : 0;
    T *tile = tiles[wv];
    const int64_t w0 = ((int64_t)blockIdx.x * WAVES + wv) * WPW;
    const bool lane_on = l < WPW;
    typedef float f2v __attribute__((ext_vector_type(2)));
    // packed-pair update for the fp32 filter (fp64 has no packed fma)
    constexpr bool PK = TWO && std::is_same<K, float>::value && PKUP;

    const K q_scale = (K)fmax(0.05, kp.follow);
    const K Qp = (K)fmax(1e-9, kp.qp * (double)q_scale), Qv = (K)fmax(1e-9, kp.qv * (double)q_scale);
    const K Qa = (K)fmax(1e-9, kp.qa * (double)q_scale), Qj = (K)fmax(1e-9, kp.qj * (double)q_scale);
    const K R = (K)fmax(1e-9, kp.r);
    const K adapt = (K)kp.adapt, clip = (K)kp.clip;
    const K gQp = adapt * Qp, gQv = adapt * Qv, gQa = adapt * Qa, gQj = adapt * Qj;
    const bool use_adapt = FL >= 0 ? (FL & kKfAdapt) != 0 : kp.adapt > 0.0;
    const bool use_clip = FL >= 0 ? (FL & kKfClip) != 0 : kp.clip > 0.0;
    const bool use_ema = FL >= 0 ? (FL & kKfEma) != 0 : kp.ema > 0.0;
    const K ema_a = use_ema ? (K)(2.0 / (kp.ema + 1.0)) : K(0);

    // ResetKalmanState(first_meas) :2015-2029, centred: pos' = 0
    K pos = 0, vel = (K)kp.iv, acc = (K)kp.ia, jerk = (K)kp.ij;
    K p00 = (K)fmax(1e-9, kp.vp), p11 = (K)fmax(1e-9, kp.vv), p22 = (K)fmax(1e-9, kp.va), p33 = (K)fmax(1e-9, kp.vj);
    K p01 = 0, p02 = 0, p03 = 0, p12 = 0, p13 = 0, p23 = 0;
    bool ema_ready = false;
    K ema_prev = 0;
    T x0 = 0;

    // tile rows are windows w0 .. w0+WPW-1; row r, step j of chunk c = series[(w0+r)*hop + c*J + j].
    // One wave instruction moves RPI rows of J contiguous samples (coalesced).  Offsets are
    // 32-bit: the host guarantees WPW*hop and WPW*n elements fit in 2 GiB.
    constexpr int RPI = 64 / J, NI = WPW / RPI;
    const int lrow = l / J, lcol = l % J;
    // rows <= 0: a wave of the last workgroup past the batch end; its descriptors are
    // empty (loads read 0, stores are dropped) and it keeps step with the barriers
    const int64_t rows = n_windows - w0 < WPW ? (n_windows > w0 ? n_windows - w0 : 0) : WPW;
    const auto rin = kbuf(series + (rows > 0 ? w0 * hop : 0), rows > 0 ? (uint32_t)(((rows - 1) * hop + n) * (int64_t)sizeof(T)) : 0u);
    const auto rout = kbuf(dout + w0 * (int64_t)n, (uint32_t)(rows * n * (int64_t)sizeof(T)));
    const uint32_t vin = (uint32_t)((lrow * hop + lcol) * (int64_t)sizeof(T));
    const uint32_t vout = (uint32_t)((lrow * n + lcol) * (int)sizeof(T));
    T reg[NI];
    const int nchunks = n / J;
    auto issue = [&](int c) {
        const uint32_t vc = vin + (uint32_t)(c * J * (int)sizeof(T));
#pragma unroll
        for (int i = 0; i < NI; ++i) reg[i] = kload(rin, vc + (uint32_t)(i * RPI * hop * (int64_t)sizeof(T)), 0u, T());
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
            K P00p, P01p, P02p, P03p, P11p, P12p, P13p, P22p, P23p, P33p;
            if constexpr (TWO) {
                // A = F P (rows of F: [1 1 1/2 1/6] [0 1 1 1/2] [0 0 1 1] [0 0 0 1]); only the
                // entries F A^T needs on and above the diagonal
                const K a00 = p00 + p01 + K(0.5) * p02 + K(1.0 / 6.0) * p03;
                const K a01 = p01 + p11 + K(0.5) * p12 + K(1.0 / 6.0) * p13;
                const K a02 = p02 + p12 + K(0.5) * p22 + K(1.0 / 6.0) * p23;
                const K a03 = p03 + p13 + K(0.5) * p23 + K(1.0 / 6.0) * p33;
                const K a11 = p11 + p12 + K(0.5) * p13;
                const K a12 = p12 + p22 + K(0.5) * p23;
                const K a13 = p13 + p23 + K(0.5) * p33;
                const K a22 = p22 + p23;
                const K a23 = p23 + p33;
                // Pp = A F^T
                P00p = a00 + a01 + K(0.5) * a02 + K(1.0 / 6.0) * a03 + Qp;
                P01p = a01 + a02 + K(0.5) * a03;
                P02p = a02 + a03;
                P03p = a03;
                // the reference's P11 prediction (:2052) is not (F P F^T)_11: it adds
                // p12 + p22 + (p13 + p23)/2 = a12 + p13/2, kept for parity
                P11p = a11 + K(2) * a12 + K(0.5) * (a13 + p13) + Qv;
                P12p = a12 + a13;
                P13p = a13;
                P22p = a22 + a23 + Qa;
                P23p = a23;
                P33p = p33 + Qj;
            } else {
                P00p = p00 + K(2) * p01 + p02 + K(1.0 / 3.0) * p03 + p11 + p12 + K(1.0 / 3.0) * p13 +
                       K(0.25) * p22 + K(1.0 / 6.0) * p23 + K(1.0 / 36.0) * p33 + Qp;
                P01p = p01 + p02 + K(0.5) * p03 + p11 + K(1.5) * p12 + K(2.0 / 3.0) * p13 + K(0.5) * p22 +
                       K(5.0 / 12.0) * p23 + K(1.0 / 12.0) * p33;
                P02p = p02 + p03 + p12 + p13 + K(0.5) * p22 + K(2.0 / 3.0) * p23 + K(1.0 / 6.0) * p33;
                P03p = p03 + p13 + K(0.5) * p23 + K(1.0 / 6.0) * p33;
                P11p = p11 + K(3) * p12 + K(1.5) * p13 + K(2) * p22 + K(1.5) * p23 + K(0.25) * p33 + Qv;
                P12p = p12 + p13 + p22 + K(1.5) * p23 + K(0.5) * p33;
                P13p = p13 + p23 + K(0.5) * p33;
                P22p = p22 + K(2) * p23 + p33 + Qa;
                P23p = p23 + p33;
                P33p = p33 + Qj;
            }

            K y = z - x0p;
            K S = P00p + R;
            if (use_adapt) {
                if constexpr (TWO) {  // boost - 1 = min(5,|y|/sigma) g, g folded into the Q terms
                    const K k = fmin(K(5), fabs(y) * krsqrt(S));
                    P00p += k * gQp;
                    P11p += k * gQv;
                    P22p += k * gQa;
                    P33p += k * gQj;
                } else {
                    const K k = fmin(K(5), fabs(y) * krsqrt(S)) * adapt;
                    P00p += k * Qp;
                    P11p += k * Qv;
                    P22p += k * Qa;
                    P33p += k * Qj;
                }
                S = P00p + R;
            }
            const K rs = krsqrt(S);
            if constexpr (PK) {
                // Normalised form: g_i = P_0i / sqrt(S), y_n = y / sqrt(S) clipped to +-clip, so
                // K_i y = g_i y_n and K_i P_0j = g_i g_j.  Pairs (g0, g1), (g2, g3) and the
                // symmetric update as four packed fma (v_pk_fma_f32: one issue for two lanes' worth).
                K yn = y * rs;
                if (use_clip) yn = kclamp(yn, clip);
                const f2v pa = {P00p, P01p}, pb = {P02p, P03p};
                const f2v g01 = pa * rs, g23 = pb * rs;
                const f2v s01 = f2v{x0p, x1p} + g01 * yn, s23 = f2v{x2p, x3p} + g23 * yn;
                pos = s01.x;
                vel = s01.y;
                acc = s23.x;
                jerk = s23.y;
                const f2v q0 = pa - g01 * g01.x, q1 = pb - g23 * g01.x;
                const f2v q2 = f2v{P12p, P13p} - g23 * g01.y, q3 = f2v{P22p, P23p} - g23 * g23.x;
                p00 = fmax(K(1e-12), q0.x);
                p01 = q0.y;
                p02 = q1.x;
                p03 = q1.y;
                p11 = fmax(K(1e-12), P11p - g01.y * g01.y);
                p12 = q2.x;
                p13 = q2.y;
                p22 = fmax(K(1e-12), q3.x);
                p23 = q3.y;
                p33 = fmax(K(1e-12), P33p - g23.y * g23.y);
            } else {
                if (use_clip) y = kclamp(y, clip * (S * rs));  // clip * sqrt(S)
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
            }

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
        for (int i = 0; i < NI; ++i)
            kstore(tile[(i * RPI + lrow) * (J + 1) + lcol], rout, vout + (uint32_t)((i * RPI * n + c * J) * (int)sizeof(T)), 0u);
        __syncthreads();
    }
}

}  // namespace kcore

}  // namespace wsp
