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
//  * the state is centred on the first sample b of the lane's current LDS tile
//    (z' = z - b, pos' = pos - b, re-centred every J steps): the filter is
//    exactly shift-equivariant (innovation, gain, boost and clip depend only on
//    differences; only pos and the EMA carry the level), and centring lets the
//    fp32 plan run the filter in fp32 without cancelling against the price
//    level -- or against a level jump earlier in the window.
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

// The filter state is re-centred on a sample every kRecentre steps (see kalman_detrend_kernel): at
// most this many steps carry a level move (a price jump) in pos before it is shifted out.  Every
// segment start and tile length is a multiple of it, so segments that meet at a hand-over sit on the
// same centre.
constexpr int kRecentre = 16;

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

// Filter state of one lane (centred on its tile's first sample) and the
// step constants.
template <typename K> struct KState {
    K pos, vel, acc, jerk;
    K p00, p01, p02, p03, p11, p12, p13, p22, p23, p33;
    K ema_prev;
    bool ema_ready;
};
template <typename K> struct KConst {
    K Qp, Qv, Qa, Qj, R, gQp, gQv, gQa, gQj, adapt, clip, ema_a;
    bool use_adapt, use_clip, use_ema;
};

template <typename K, int FL> __device__ __forceinline__ KConst<K> kconst(const KP &kp) {
    KConst<K> c;
    const K q_scale = (K)fmax(0.05, kp.follow);
    c.Qp = (K)fmax(1e-9, kp.qp * (double)q_scale);
    c.Qv = (K)fmax(1e-9, kp.qv * (double)q_scale);
    c.Qa = (K)fmax(1e-9, kp.qa * (double)q_scale);
    c.Qj = (K)fmax(1e-9, kp.qj * (double)q_scale);
    c.R = (K)fmax(1e-9, kp.r);
    c.adapt = (K)kp.adapt;
    c.clip = (K)kp.clip;
    c.gQp = c.adapt * c.Qp;
    c.gQv = c.adapt * c.Qv;
    c.gQa = c.adapt * c.Qa;
    c.gQj = c.adapt * c.Qj;
    c.use_adapt = FL >= 0 ? (FL & kKfAdapt) != 0 : kp.adapt > 0.0;
    c.use_clip = FL >= 0 ? (FL & kKfClip) != 0 : kp.clip > 0.0;
    c.use_ema = FL >= 0 ? (FL & kKfEma) != 0 : kp.ema > 0.0;
    c.ema_a = c.use_ema ? (K)(2.0 / (kp.ema + 1.0)) : K(0);
    return c;
}

// ResetKalmanState(first_meas) :2015-2029, centred: pos = first_meas - centre
template <typename K> __device__ __forceinline__ void kreset(KState<K> &s, const KP &kp, K pos0) {
    s.pos = pos0;
    s.vel = (K)kp.iv;
    s.acc = (K)kp.ia;
    s.jerk = (K)kp.ij;
    s.p00 = (K)fmax(1e-9, kp.vp);
    s.p11 = (K)fmax(1e-9, kp.vv);
    s.p22 = (K)fmax(1e-9, kp.va);
    s.p33 = (K)fmax(1e-9, kp.vj);
    s.p01 = s.p02 = s.p03 = s.p12 = s.p13 = s.p23 = K(0);
    s.ema_prev = K(0);
    s.ema_ready = false;
}

// StepKalman4D :2031-2125 on the symmetric covariance; returns the trend.
// TWO: predicted covariance through A = F P in two stages (32 instead of 41
// add/fma; F is the constant-jerk transition, P symmetric) instead of the
// reference's expanded sums -- same values, including the reference's extra
// terms in P11.  PK (fp32 filter): the update in normalised form, g = P_0./sqrt(S),
// with the state and covariance updates as packed pairs (v_pk_fma_f32), about 10
// fewer instructions per step (0.743 -> 0.678 ms at C3).
template <typename K, bool TWO, bool PKUP>
__device__ __forceinline__ K kstep(KState<K> &st, const KConst<K> &c, K z) {
    typedef float f2v __attribute__((ext_vector_type(2)));
    constexpr bool PK = TWO && std::is_same<K, float>::value && PKUP;
    const K pos = st.pos, vel = st.vel, acc = st.acc, jerk = st.jerk;
    const K p00 = st.p00, p01 = st.p01, p02 = st.p02, p03 = st.p03, p11 = st.p11, p12 = st.p12, p13 = st.p13,
            p22 = st.p22, p23 = st.p23, p33 = st.p33;
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
        P00p = a00 + a01 + K(0.5) * a02 + K(1.0 / 6.0) * a03 + c.Qp;
        P01p = a01 + a02 + K(0.5) * a03;
        P02p = a02 + a03;
        P03p = a03;
        // the reference's P11 prediction (:2052) is not (F P F^T)_11: it adds
        // p12 + p22 + (p13 + p23)/2 = a12 + p13/2, kept for parity
        P11p = a11 + K(2) * a12 + K(0.5) * (a13 + p13) + c.Qv;
        P12p = a12 + a13;
        P13p = a13;
        P22p = a22 + a23 + c.Qa;
        P23p = a23;
        P33p = p33 + c.Qj;
    } else {
        P00p = p00 + K(2) * p01 + p02 + K(1.0 / 3.0) * p03 + p11 + p12 + K(1.0 / 3.0) * p13 + K(0.25) * p22 +
               K(1.0 / 6.0) * p23 + K(1.0 / 36.0) * p33 + c.Qp;
        P01p = p01 + p02 + K(0.5) * p03 + p11 + K(1.5) * p12 + K(2.0 / 3.0) * p13 + K(0.5) * p22 +
               K(5.0 / 12.0) * p23 + K(1.0 / 12.0) * p33;
        P02p = p02 + p03 + p12 + p13 + K(0.5) * p22 + K(2.0 / 3.0) * p23 + K(1.0 / 6.0) * p33;
        P03p = p03 + p13 + K(0.5) * p23 + K(1.0 / 6.0) * p33;
        P11p = p11 + K(3) * p12 + K(1.5) * p13 + K(2) * p22 + K(1.5) * p23 + K(0.25) * p33 + c.Qv;
        P12p = p12 + p13 + p22 + K(1.5) * p23 + K(0.5) * p33;
        P13p = p13 + p23 + K(0.5) * p33;
        P22p = p22 + K(2) * p23 + p33 + c.Qa;
        P23p = p23 + p33;
        P33p = p33 + c.Qj;
    }

    K y = z - x0p;
    K S = P00p + c.R;
    if (c.use_adapt) {
        if constexpr (TWO) {  // boost - 1 = min(5,|y|/sigma) g, g folded into the Q terms
            const K k = fmin(K(5), fabs(y) * krsqrt(S));
            P00p += k * c.gQp;
            P11p += k * c.gQv;
            P22p += k * c.gQa;
            P33p += k * c.gQj;
        } else {
            const K k = fmin(K(5), fabs(y) * krsqrt(S)) * c.adapt;
            P00p += k * c.Qp;
            P11p += k * c.Qv;
            P22p += k * c.Qa;
            P33p += k * c.Qj;
        }
        S = P00p + c.R;
    }
    const K rs = krsqrt(S);
    if constexpr (PK) {
        // Normalised form: g_i = P_0i / sqrt(S), y_n = y / sqrt(S) clipped to +-clip, so
        // K_i y = g_i y_n and K_i P_0j = g_i g_j.  Pairs (g0, g1), (g2, g3) and the
        // symmetric update as four packed fma (v_pk_fma_f32: one issue for two lanes' worth).
        K yn = y * rs;
        if (c.use_clip) yn = kclamp(yn, c.clip);
        const f2v pa = {P00p, P01p}, pb = {P02p, P03p};
        const f2v g01 = pa * rs, g23 = pb * rs;
        const f2v s01 = f2v{x0p, x1p} + g01 * yn, s23 = f2v{x2p, x3p} + g23 * yn;
        st.pos = s01.x;
        st.vel = s01.y;
        st.acc = s23.x;
        st.jerk = s23.y;
        const f2v q0 = pa - g01 * g01.x, q1 = pb - g23 * g01.x;
        const f2v q2 = f2v{P12p, P13p} - g23 * g01.y, q3 = f2v{P22p, P23p} - g23 * g23.x;
        st.p00 = fmax(K(1e-12), q0.x);
        st.p01 = q0.y;
        st.p02 = q1.x;
        st.p03 = q1.y;
        st.p11 = fmax(K(1e-12), P11p - g01.y * g01.y);
        st.p12 = q2.x;
        st.p13 = q2.y;
        st.p22 = fmax(K(1e-12), q3.x);
        st.p23 = q3.y;
        st.p33 = fmax(K(1e-12), P33p - g23.y * g23.y);
    } else {
        if (c.use_clip) y = kclamp(y, c.clip * (S * rs));  // clip * sqrt(S)
        const K inv = rs * rs;  // 1/S
        const K K0 = P00p * inv, K1 = P01p * inv, K2 = P02p * inv, K3 = P03p * inv;
        st.pos = x0p + K0 * y;
        st.vel = x1p + K1 * y;
        st.acc = x2p + K2 * y;
        st.jerk = x3p + K3 * y;
        // P_ij <- P_ij - K_i P_0j (symmetric), diagonal floors 1e-12
        st.p00 = fmax(K(1e-12), P00p - K0 * P00p);
        st.p01 = P01p - K1 * P00p;
        st.p02 = P02p - K2 * P00p;
        st.p03 = P03p - K3 * P00p;
        st.p11 = fmax(K(1e-12), P11p - K1 * P01p);
        st.p12 = P12p - K2 * P01p;
        st.p13 = P13p - K3 * P01p;
        st.p22 = fmax(K(1e-12), P22p - K2 * P02p);
        st.p23 = P23p - K3 * P02p;
        st.p33 = fmax(K(1e-12), P33p - K3 * P03p);
    }

    K trend = st.pos;
    if (c.use_ema) {  // :2117-2123
        if (!st.ema_ready) {
            st.ema_prev = trend;
            st.ema_ready = true;
        }
        st.ema_prev = c.ema_a * trend + (K(1) - c.ema_a) * st.ema_prev;
        trend = st.ema_prev;
    }
    return trend;
}

// Segments of one window's filter.  SEG = 1: one lane runs the window's N steps.
// SEG = 2 (parallel in time): lane pair (l, l + 32) splits window l: the first
// lane runs samples [0, L0) from the reset as usual, the second lane starts
// cold -- ResetKalmanState at sample L0 - WU -- runs WU warm-up steps without
// output, then samples [L0, N), L0 = (N + WU)/2 so that both run L0 steps.  The
// filter forgets its initial state: a cold start contracts onto the sequential
// filter's trajectory (oracle.numpy_kalman_trend: 4e-16 after 256 steps on the
// C3 data) until rounding makes the two states identical, after which the
// deterministic recurrence keeps them identical.  The result is VERIFIED, not
// assumed: at the end the first lane's state after sample L0 - 1 is compared
// BIT FOR BIT with the second lane's state after its warm-up (all 14 values,
// + the EMA state when enabled); if any differs, the second lanes of the wave
// re-run [L0, N) from the first lanes' state.  Either way every output is
// bit-identical to the one-lane filter's.  Twice the lanes per window: at C3's
// 65536 windows the filter gets two waves per SIMD instead of one lone wave,
// which issues VALU every 2 instead of every 4 cycles (MI355X_MICROARCH.md,
// vector issue cost), at (N + WU)/2N of the steps per lane.
constexpr int kSegWarm = 512;
template <typename K> __device__ __forceinline__ bool kclose(K a, K b) {
    return __builtin_bit_cast(typename std::conditional<sizeof(K) == 4, unsigned, unsigned long long>::type, a) ==
           __builtin_bit_cast(typename std::conditional<sizeof(K) == 4, unsigned, unsigned long long>::type, b);
}
template <typename K> __device__ __forceinline__ K kxor32(K v) {  // value of lane l ^ 32
    if constexpr (sizeof(K) == 4) {
        return __builtin_bit_cast(K, __shfl_xor(__builtin_bit_cast(int, v), 32, 64));
    } else {
        const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
        const int lo = __shfl_xor((int)(unsigned)u, 32, 64), hi = __shfl_xor((int)(unsigned)(u >> 32), 32, 64);
        return __builtin_bit_cast(K, (unsigned long long)(unsigned)lo | ((unsigned long long)(unsigned)hi << 32));
    }
}

// WPW windows per wave (64, or 32 so that two waves share a SIMD and hide each
// other's dependency stalls when the batch has only one window per lane).
// WAVES: independent waves per workgroup (each its own WPW windows and LDS
// tile).  With WAVES = 4 and an LDS reservation that admits one workgroup per
// CU, a batch of at most 64 windows per SIMD runs exactly one wave on every
// SIMD; single-wave workgroups may be stacked two to a SIMD by the dispatcher
// while other SIMDs idle (measured: 0.76 ms back-to-back, 1.1 ms after a
// spectrum launch at C3).  SEG = 2 requires WPW = 32 (lane pairs l, l + 32).
// `fallbacks` (tools only, may be null): waves that re-ran their second segments.
template <typename T, typename K, int J, int WPW, int UNROLL = 2, int FL = kKfRuntime, bool TWO = false, int WAVES = 1,
          bool PKUP = false, int SEG = 1, int WU = kSegWarm>
__global__ __launch_bounds__(64 * WAVES) void kalman_detrend_kernel(const T *__restrict__ series, T *__restrict__ dout,
                                                                    int64_t hop, int64_t n_windows, int n, KP kp,
                                                                    unsigned *fallbacks = nullptr, double *dbg = nullptr) {
    static_assert(SEG == 1 || (SEG == 2 && WPW == 32), "two segments pair lanes l and l + 32");
    __shared__ T tiles[WAVES][64 * (J + 1)];  // per wave: [row][step], +1 pad: conflict-free row walks
    // wave index through readfirstlane: provably uniform, so the descriptors stay scalar
    const int l = threadIdx.x % 64, wv = WAVES > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x / 64) : 0;
    T *tile = tiles[wv];
    const int64_t w0 = ((int64_t)blockIdx.x * WAVES + wv) * WPW;
    // rows of the tile: SEG = 1, row r = window r; SEG = 2, row r = segment r / 32 of window r % 32
    constexpr int ROWS = 64;
    const bool lane_on = SEG == 2 || l < WPW;
    const KConst<K> kc = kconst<K, FL>(kp);
    // segment geometry (SEG = 2): both lanes run L0 steps; the second lane's samples start at L0 - WU
    const int L0 = SEG == 2 ? (n + WU) / 2 : n;
    const int seg_off = L0 - WU;  // series offset of the second segment's first (warm-up) sample
    const int nchunks = L0 / J;
    constexpr int WUC = WU / J;  // warm-up chunks of the second segment
    static_assert(WU % 32 == 0, "whole tiles of warm-up");

    // tile rows are windows w0 .. w0+WPW-1 (x SEG); row r, step j of chunk c = series[(w0+wr)*hop + sr*seg_off +
    // c*J + j].  One wave instruction moves RPI rows of J contiguous samples (coalesced).  Offsets are
    // 32-bit: the host guarantees WPW*hop and WPW*n elements fit in 2 GiB.
    constexpr int RPI = 64 / J, NI = ROWS / RPI, NIS = NI / SEG;  // NIS instructions per segment
    const int lrow = l / J, lcol = l % J;
    // rows <= 0: a wave of the last workgroup past the batch end; its descriptors are
    // empty (loads read 0, stores are dropped) and it keeps step with the barriers
    const int64_t rows = n_windows - w0 < WPW ? (n_windows > w0 ? n_windows - w0 : 0) : WPW;
    const auto rin = kbuf(series + (rows > 0 ? w0 * hop : 0), rows > 0 ? (uint32_t)(((rows - 1) * hop + n) * (int64_t)sizeof(T)) : 0u);
    const auto rout = kbuf(dout + w0 * (int64_t)n, (uint32_t)(rows * n * (int64_t)sizeof(T)));
    const uint32_t vin = (uint32_t)((lrow * hop + lcol) * (int64_t)sizeof(T));
    const uint32_t vout = (uint32_t)((lrow * n + lcol) * (int)sizeof(T));
    // per-instruction row offsets (uniform): instruction i covers rows i*RPI + lrow
    auto in_row = [&](int i) { return (uint32_t)((((i % NIS) * RPI) * hop + (i / NIS) * (int64_t)seg_off) * (int64_t)sizeof(T)); };
    auto out_row = [&](int i) { return (uint32_t)((((i % NIS) * RPI) * (int64_t)n + (i / NIS) * (int64_t)seg_off) * (int64_t)sizeof(T)); };
    T reg[NI];
    auto issue = [&](int c) {
        const uint32_t vc = vin + (uint32_t)(c * J * (int)sizeof(T));
#pragma unroll
        for (int i = 0; i < NI; ++i) reg[i] = kload(rin, vc + in_row(i), 0u, T());
    };

    KState<K> st;
    T base = 0, base_at_warm = 0;  // the lane's current centre: the first sample of its current tile
    const int lr = lane_on ? l : 0;
    // filters chunks [c0, c1) of every lane; stores the rows of segment 0 for c >= s0 and of segment 1
    // for c >= s1 (SEG = 2: its warm-up chunks produce no output)
    auto run = [&](int c0, int c1, int s0, int s1, bool save_warm, KState<K> &warm) {
        issue(c0);
        for (int c = c0; c < c1; ++c) {
#pragma unroll
            for (int i = 0; i < NI; ++i) tile[(i * RPI + lrow) * (J + 1) + lcol] = reg[i];
            __syncthreads();
            if (c + 1 < c1) issue(c + 1);  // next tile in flight while the lanes filter this one
            T zrow[J];  // this row's J samples in registers: no LDS latency inside the recurrence
#pragma unroll
            for (int j = 0; j < J; ++j) zrow[j] = tile[lr * (J + 1) + j];
            // re-centre on the tile's first sample (shift-equivariance: only pos and the EMA carry the
            // level) and every kRecentre samples after it; the shift base - zrow[j] is exact for prices
            // within 2x of each other (Sterbenz)
            if (c == 0) {
                kreset<K>(st, kp, K(0));
            } else {
                const K sh = (K)(base - zrow[0]);
                st.pos += sh;
                st.ema_prev += sh;
            }
            base = zrow[0];
#pragma unroll UNROLL
            for (int j = 0; j < J; ++j) {
                if (j > 0 && j % kRecentre == 0) {  // and every kRecentre steps inside the tile
                    const K sh = (K)(base - zrow[j]);
                    st.pos += sh;
                    st.ema_prev += sh;
                    base = zrow[j];
                }
                const K z = (K)(zrow[j] - base);  // exact for prices within 2x of the centre (Sterbenz)
                const K trend = kstep<K, TWO, PKUP>(st, kc, z);
                zrow[j] = T(z - trend);
            }
            if constexpr (SEG == 2) {
                if (save_warm && c == WUC - 1) {  // the second lanes' state after sample L0 - 1
                    warm = st;
                    base_at_warm = base;
                }
            }
            if (lane_on) {
#pragma unroll
                for (int j = 0; j < J; ++j) tile[l * (J + 1) + j] = zrow[j];
            }
            __syncthreads();
            const uint32_t vc = vout + (uint32_t)(c * J * (int)sizeof(T));
#pragma unroll
            for (int i = 0; i < NI; ++i)
                if (c >= (i / NIS == 0 ? s0 : s1))
                    kstore(tile[(i * RPI + lrow) * (J + 1) + lcol], rout, vc + out_row(i), 0u);
            __syncthreads();
        }
    };
    KState<K> warm;
    if constexpr (SEG == 1) {
        run(0, nchunks, 0, 0, false, warm);
    } else {
        run(0, nchunks, 0, WUC, true, warm);
        // verify: the first lane's exact state after sample L0 - 1 against the second lane's warm-up state
        KState<K> ex;
        ex.pos = kxor32(st.pos), ex.vel = kxor32(st.vel), ex.acc = kxor32(st.acc), ex.jerk = kxor32(st.jerk);
        ex.p00 = kxor32(st.p00), ex.p01 = kxor32(st.p01), ex.p02 = kxor32(st.p02), ex.p03 = kxor32(st.p03);
        ex.p11 = kxor32(st.p11), ex.p12 = kxor32(st.p12), ex.p13 = kxor32(st.p13), ex.p22 = kxor32(st.p22);
        ex.p23 = kxor32(st.p23), ex.p33 = kxor32(st.p33), ex.ema_prev = kxor32(st.ema_prev);
        ex.ema_ready = __shfl_xor((int)st.ema_ready, 32, 64) != 0;
        bool ok = kclose(ex.pos, warm.pos) && kclose(ex.vel, warm.vel) && kclose(ex.acc, warm.acc) &&
                  kclose(ex.jerk, warm.jerk) && kclose(ex.p00, warm.p00) && kclose(ex.p01, warm.p01) &&
                  kclose(ex.p02, warm.p02) && kclose(ex.p03, warm.p03) && kclose(ex.p11, warm.p11) &&
                  kclose(ex.p12, warm.p12) && kclose(ex.p13, warm.p13) && kclose(ex.p22, warm.p22) &&
                  kclose(ex.p23, warm.p23) && kclose(ex.p33, warm.p33);
        if (kc.use_ema) ok = ok && ex.ema_ready == warm.ema_ready && kclose(ex.ema_prev, warm.ema_prev);
        if (l < 32) ok = true;  // only the second lanes' outputs depend on the check
        if (dbg && l >= 32 && w0 + (l - 32) < n_windows) {  // tools: exact state and warm-up state per window
            double *q = dbg + (w0 + l - 32) * 28;
            const K e[14] = {ex.pos, ex.vel, ex.acc, ex.jerk, ex.p00, ex.p01, ex.p02, ex.p03, ex.p11, ex.p12, ex.p13, ex.p22, ex.p23, ex.p33};
            const K wv2[14] = {warm.pos, warm.vel, warm.acc, warm.jerk, warm.p00, warm.p01, warm.p02, warm.p03, warm.p11, warm.p12, warm.p13, warm.p22, warm.p23, warm.p33};
            for (int k = 0; k < 14; ++k) {
                q[k] = (double)e[k];
                q[14 + k] = (double)wv2[k];
            }
        }
        if (__ballot(!ok)) {  // wave-uniform: the second lanes re-run [L0, N) from the exact state
            if (fallbacks && l == 0) atomicAdd(fallbacks, 1u);
            st = ex;
            // the exact state is centred on sample L0 - J (the first lanes' last tile), which is the
            // second lanes' own centre of tile WUC - 1
            base = base_at_warm;
            // chunks WUC .. nchunks-1 of the second segment; the first lanes recompute their own last
            // chunks' values, which are not stored (s0 past the end)
            run(WUC, nchunks, nchunks, WUC, false, warm);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Packed two-segment filter (fp32 plans, reference default flags: adaptive boost + clip, no EMA).
//
// At C3 the one-lane-per-window filter is one lone wave per SIMD, and a lone wave issues one VALU
// instruction per 4 cycles whether it is v_fma_f32 or v_pk_fma_f32 (MI355X_MICROARCH.md, issue
// cost): a packed instruction does two lanes' worth of filter work for the price of one.  The
// window's own recurrence has no pair structure left to pack (kstep PKUP packs what there is), so
// each lane runs TWO time segments of its window side by side as the halves of float2 registers:
//   .x  segment A: ResetKalmanState at sample 0, samples [0, L0)                 (exact)
//   .y  segment B: ResetKalmanState at sample L0 - WU, WU warm-up steps without output,
//                  then samples [L0, N)                                           L0 = (N + WU) / 2
// so that every step of the lane is one packed step of both (L0 steps instead of N).  The filter
// forgets its start (a cold start contracts onto the sequential trajectory; numpy, C3 data: 4e-16
// after 256 steps in fp64, 1-6 ulps in fp32).  The warm-up is VERIFIED per window: after its
// last step segment A holds the exact state at sample L0 - 1, which segment B reached after its
// warm-up (kept from then); every component must agree within 2^-16 relative plus an absolute
// floor of 2^-24 (|centre| + |pos|) -- half an fp32 ulp of the price level, below what an fp32
// series can resolve.  Any window that fails makes its wave re-run [L0, N) from segment A's
// exact state (wave-uniform branch), so a filter that has not converged is never used.  The
// outputs agree with the sequential fp32 filter to the fp32 rounding of the state (not bit for
// bit), i.e. well inside the f32 plan's parity bar (1e-5 of the spectrum); fp64 plans keep the
// sequential kernel.
typedef float kf2 __attribute__((ext_vector_type(2)));

struct KState2 {
    kf2 pos, vel, acc, jerk, p00, p01, p02, p03, p11, p12, p13, p22, p23, p33;
};

__device__ __forceinline__ kf2 krsq2(kf2 s) { return kf2{__builtin_amdgcn_rsqf(s.x), __builtin_amdgcn_rsqf(s.y)}; }
__device__ __forceinline__ kf2 kfloor2(kf2 v) { return kf2{fmaxf(1e-12f, v.x), fmaxf(1e-12f, v.y)}; }

// StepKalman4D :2031-2125 for both segments: the two-stage predict and the normalised update of
// kstep<float, true, true>, every operation a packed one except rsq / min / clamp / floor.
__device__ __forceinline__ kf2 kstep_pk2(KState2 &st, const KConst<float> &c, kf2 z) {
    const kf2 pos = st.pos, vel = st.vel, acc = st.acc, jerk = st.jerk;
    const kf2 p00 = st.p00, p01 = st.p01, p02 = st.p02, p03 = st.p03, p11 = st.p11, p12 = st.p12, p13 = st.p13,
              p22 = st.p22, p23 = st.p23, p33 = st.p33;
    const kf2 x0p = pos + vel + 0.5f * acc + (1.0f / 6.0f) * jerk;
    const kf2 x1p = vel + acc + 0.5f * jerk;
    const kf2 x2p = acc + jerk;
    const kf2 x3p = jerk;
    const kf2 a00 = p00 + p01 + 0.5f * p02 + (1.0f / 6.0f) * p03;
    const kf2 a01 = p01 + p11 + 0.5f * p12 + (1.0f / 6.0f) * p13;
    const kf2 a02 = p02 + p12 + 0.5f * p22 + (1.0f / 6.0f) * p23;
    const kf2 a03 = p03 + p13 + 0.5f * p23 + (1.0f / 6.0f) * p33;
    const kf2 a11 = p11 + p12 + 0.5f * p13;
    const kf2 a12 = p12 + p22 + 0.5f * p23;
    const kf2 a13 = p13 + p23 + 0.5f * p33;
    const kf2 a22 = p22 + p23;
    const kf2 a23 = p23 + p33;
    kf2 P00p = a00 + a01 + 0.5f * a02 + (1.0f / 6.0f) * a03 + c.Qp;
    const kf2 P01p = a01 + a02 + 0.5f * a03;
    const kf2 P02p = a02 + a03;
    const kf2 P03p = a03;
    kf2 P11p = a11 + 2.0f * a12 + 0.5f * (a13 + p13) + c.Qv;  // the reference's P11 (:2052), see kstep
    const kf2 P12p = a12 + a13;
    const kf2 P13p = a13;
    kf2 P22p = a22 + a23 + c.Qa;
    const kf2 P23p = a23;
    kf2 P33p = p33 + c.Qj;

    const kf2 y = z - x0p;
    kf2 S = P00p + c.R;
    const kf2 yr = y * krsq2(S);  // boost - 1 = min(5, |y|/sigma) g, g folded into gQ*
    const kf2 k = {fminf(5.0f, fabsf(yr.x)), fminf(5.0f, fabsf(yr.y))};
    P00p += k * c.gQp;
    P11p += k * c.gQv;
    P22p += k * c.gQa;
    P33p += k * c.gQj;
    S = P00p + c.R;
    const kf2 rs = krsq2(S);
    kf2 yn = y * rs;
    yn = kf2{__builtin_amdgcn_fmed3f(yn.x, -c.clip, c.clip), __builtin_amdgcn_fmed3f(yn.y, -c.clip, c.clip)};
    const kf2 g0 = P00p * rs, g1 = P01p * rs, g2 = P02p * rs, g3 = P03p * rs;
    st.pos = x0p + g0 * yn;
    st.vel = x1p + g1 * yn;
    st.acc = x2p + g2 * yn;
    st.jerk = x3p + g3 * yn;
    st.p00 = kfloor2(P00p - g0 * g0);
    st.p01 = P01p - g1 * g0;
    st.p02 = P02p - g2 * g0;
    st.p03 = P03p - g3 * g0;
    st.p11 = kfloor2(P11p - g1 * g1);
    st.p12 = P12p - g2 * g1;
    st.p13 = P13p - g3 * g1;
    st.p22 = kfloor2(P22p - g2 * g2);
    st.p23 = P23p - g3 * g2;
    st.p33 = kfloor2(P33p - g3 * g3);
    return st.pos;
}

// ---------------------------------------------------------------------------------------------
// The same step in the Newton (forward-difference) basis, the fp32 default since round 6.
//
// F = exp(N) (N the shift) is similar to the Jordan block Jd = I + N: F = T Jd T^-1 with
//   T^-1 = [[1, 0, 0, 0], [0, 1, 1/2, 1/6], [0, 0, 1, 1], [0, 0, 0, 1]],
// i.e. u = T^-1 x holds the forward differences of the cubic (u0 = pos, u1 = vel + acc/2 +
// jerk/6, u2 = acc + jerk, u3 = jerk).  In u the state predict is three neighbour sums and the
// covariance predict P' <- Jd P' Jd^T fifteen adds (instead of 6 and 35 operations); T's first
// row is e0, so S, gain, boost, clip and the normalised update keep their form.  What the
// reference adds beyond F P F^T carries over as:
//  * the P11 prediction of :2052 adds e = P12 + P22 + (P13 + P23)/2 of the ORIGINAL basis; T^-1 e1
//    = e1, so in u it is e added to P'11, e = P'12 - P'13/2 + P'22/2 - 11/12 P'23 + P'33/3;
//  * Q = diag(Qp, Qv, Qa, Qj) becomes Q' = T^-1 Q T^-T: Qp on 00 plus six entries of the 1..3 block
//    (KNb below), boosted as a whole by b = 1 + min(5, |y|/sigma) adapt;
//  * the diagonal floors max(1e-12, P_ii) (:2110-2114) act on the original basis and are NOT
//    applied.  Instead they are proven no-ops: while e >= -Qv/2 at every step, the predicted P
//    dominates diag(Qp, Qv/2, Qa, Qj) (F P F^T and bQ are PSD, e e1e1^T takes at most Qv/2), so the
//    updated P = (P_p^-1 + e0 e0^T/R)^-1 >= diag(Qp R/(Qp + R), Qv/2, Qa, Qj) -- above 1e-12 by the
//    host's gate (nb2_ok: all of them >= 2^-20, far above fp32 rounding of P).  The kernel keeps
//    min(e) per lane (one v_min3 per two steps and segment) and a wave with e < -Qv/2 anywhere
//    re-runs in the original basis with the floors (kalman_pk2_kernel NB = false).
// CPU model and checks of the algebra against the oracle: tests/test_kalman_newton.py.
struct KNb {
    float Qp, Q11, Q12, Q13, Q22, Q23, Q33, R, QpR, adapt, clip, emin;  // emin: -Qv/2
};
inline bool nb2_ok(const KP &kp) {
    const double qs = kp.follow > 0.05 ? kp.follow : 0.05;
    auto fl = [](double v) { return v > 1e-9 ? v : 1e-9; };
    const double Qp = fl(kp.qp * qs), Qv = fl(kp.qv * qs), Qa = fl(kp.qa * qs), Qj = fl(kp.qj * qs), R = fl(kp.r);
    double m = Qp * R / (Qp + R);
    m = m < Qv / 2 ? m : Qv / 2;
    m = m < Qa ? m : Qa;
    m = m < Qj ? m : Qj;
    return m >= 0x1p-20;
}
__device__ __forceinline__ KNb knb_const(const KP &kp) {
    const double qs = fmax(0.05, kp.follow);
    const double Qp = fmax(1e-9, kp.qp * qs), Qv = fmax(1e-9, kp.qv * qs), Qa = fmax(1e-9, kp.qa * qs),
                 Qj = fmax(1e-9, kp.qj * qs), R = fmax(1e-9, kp.r);
    KNb c;
    c.Qp = (float)Qp;
    c.Q11 = (float)(Qv + Qa / 4 + Qj / 36);
    c.Q12 = (float)(Qa / 2 + Qj / 6);
    c.Q13 = (float)(Qj / 6);
    c.Q22 = (float)(Qa + Qj);
    c.Q23 = (float)Qj;
    c.Q33 = (float)Qj;
    c.R = (float)R;
    c.QpR = (float)(Qp + R);
    c.adapt = (float)kp.adapt;
    c.clip = (float)kp.clip;
    c.emin = (float)(-0.5 * Qv);
    return c;
}
// ResetKalmanState :2015-2029 in u (centred: u0 = 0): u = T^-1 (0, iv, ia, ij), P' = T^-1 P0 T^-T
__device__ __forceinline__ void knb_reset(KState2 &st, const KP &kp) {
    const double vp = fmax(1e-9, kp.vp), vv = fmax(1e-9, kp.vv), va = fmax(1e-9, kp.va), vj = fmax(1e-9, kp.vj);
    auto b = [](double v) { const float f = (float)v; return kf2{f, f}; };
    st.pos = kf2{0.f, 0.f};
    st.vel = b(kp.iv + kp.ia / 2 + kp.ij / 6);
    st.acc = b(kp.ia + kp.ij);
    st.jerk = b(kp.ij);
    st.p00 = b(vp);
    st.p01 = st.p02 = st.p03 = kf2{0.f, 0.f};
    st.p11 = b(vv + va / 4 + vj / 36);
    st.p12 = b(va / 2 + vj / 6);
    st.p13 = b(vj / 6);
    st.p22 = b(va + vj);
    st.p23 = b(vj);
    st.p33 = b(vj);
}
// One step of both segments in u; e (the reference's P11 term) leaves through `e` for the guard.
__device__ __forceinline__ kf2 kstep_nb2(KState2 &st, const KNb &c, kf2 z, kf2 &e) {
    const kf2 p00 = st.p00, p01 = st.p01, p02 = st.p02, p03 = st.p03, p11 = st.p11, p12 = st.p12, p13 = st.p13,
              p22 = st.p22, p23 = st.p23, p33 = st.p33;
    e = p12 - 0.5f * p13 + 0.5f * p22 - (11.0f / 12.0f) * p23 + (1.0f / 3.0f) * p33;
    const kf2 u0p = st.pos + st.vel, u1p = st.vel + st.acc, u2p = st.acc + st.jerk, u3p = st.jerk;
    // Jd P' Jd^T: C_ij = P_ij + P_i+1,j + P_i,j+1 + P_i+1,j+1 (15 adds)
    const kf2 c23 = p23 + p33, c22 = (p22 + p23) + c23, c13 = p13 + p23, b12 = p12 + p22, c12 = b12 + c13;
    const kf2 c11 = (p11 + p12) + b12, c03 = p03 + p13, b02 = p02 + p12, c02 = b02 + c03, b01 = p01 + p11;
    const kf2 c01 = b01 + b02, c00 = (p00 + p01) + b01;
    const kf2 y = z - u0p;
    const kf2 yr = y * krsq2(c00 + c.QpR);  // S before the boost: P00p (with Qp) + R
    const kf2 bq = kf2{fminf(5.0f, fabsf(yr.x)), fminf(5.0f, fabsf(yr.y))} * c.adapt + 1.0f;  // boost b
    const kf2 P00p = c00 + bq * c.Qp, P11p = (c11 + e) + bq * c.Q11, P12p = c12 + bq * c.Q12, P13p = c13 + bq * c.Q13;
    const kf2 P22p = c22 + bq * c.Q22, P23p = c23 + bq * c.Q23, P33p = p33 + bq * c.Q33;
    const kf2 rs = krsq2(P00p + c.R);
    kf2 yn = y * rs;
    yn = kf2{__builtin_amdgcn_fmed3f(yn.x, -c.clip, c.clip), __builtin_amdgcn_fmed3f(yn.y, -c.clip, c.clip)};
    const kf2 g0 = P00p * rs, g1 = c01 * rs, g2 = c02 * rs, g3 = c03 * rs;
    st.pos = u0p + g0 * yn;
    st.vel = u1p + g1 * yn;
    st.acc = u2p + g2 * yn;
    st.jerk = u3p + g3 * yn;
    st.p00 = P00p - g0 * g0;
    st.p01 = c01 - g1 * g0;
    st.p02 = c02 - g2 * g0;
    st.p03 = c03 - g3 * g0;
    st.p11 = P11p - g1 * g1;
    st.p12 = P12p - g2 * g1;
    st.p13 = P13p - g3 * g1;
    st.p22 = P22p - g2 * g2;
    st.p23 = P23p - g3 * g2;
    st.p33 = P33p - g3 * g3;
    return st.pos;
}

constexpr int kPk2Warm = 256;
// can the packed two-segment kernel take windows of n samples with tiles of J steps?
constexpr bool pk2_fits(int n, int J = 32, int WU = kPk2Warm) { return n >= 4 * WU && ((n + WU) / 2) % J == 0; }

__device__ __forceinline__ bool kagree(float a, float b, float floor_) {
    return fabsf(a - b) <= 0x1p-16f * (fabsf(a) + fabsf(b)) + floor_;
}

// WAVES independent waves per workgroup, each 64 windows (one per lane) and its own LDS tile of
// [window][step] (A, B) pairs, row stride J + 2 pairs (68 dwords at J = 32):
//  * global IO moves rows of J contiguous samples, 16 B per lane (8 lanes per row, 8 rows per wave
//    instruction), through buffer descriptors based at the wave's first window; the uniform row
//    offsets ride in soffset, the lane's offset in voffset (no address VALU per access);
//  * a lane's 4 samples of a segment-A row and of the segment-B row of the same window and
//    columns land as 4 (A, B) pairs = two ds_write_b128, and leave the same way;
//  * the filter reads two steps of both segments per ds_read_b128.
// With 68-dword rows every one of these LDS accesses is conflict-free: 16 lanes of a b128 access
// cover the 64 banks once (rows 4 banks apart, 8 lanes of a row 8 banks apart).
// ROT (default): the tile loop rotated so that the wait for tile c + 1's loads comes after tile c's
// stores on every path, and the main pass's stores unconditional (segment B's warm-up values land in
// segment A's region [L0 - WU, L0), which segment A overwrites later from the same wave): the loads
// then need vmcnt(#stores) instead of vmcnt(0) (gfx950 counts loads and stores in one in-order
// counter, and the unrotated loop's entry path and conditional stores forced a wait for the previous
// tile's stores every J steps).
// SCP: cache policy of the detrended rows' stores (16 = sc1: written through to memory, so none are left dirty in
// the XCDs' L2s for the writeback between the filter and the spectrum launch; 0 = plain)
// NB = 1: the Newton-basis step (kstep_nb2) with its floor guard; a wave whose guard fails re-runs the
// whole window pair in the original basis (the NB = 0 form) with the floors.  NB = 2 (tools): the
// guard forced to fail, so every wave takes that re-run; NB = 3 (tools): the tile IO without the
// filter.  `fallbacks` (tools): +1 per warm-up re-run, +65536 per guard re-run.
template <int J, int WAVES, int WU = kPk2Warm, bool ROT = true, int SCP = 0, int NB = 0>
// wpairs (optional): the window as (h_j, h_(j + seg_off)) pairs, j < L0, staged once into dynamic LDS (L0 x 8 B) and
// multiplied into both segments' detrended rows on their way out (the spectrum launch then takes no window).
__global__ __launch_bounds__(64 * WAVES) void kalman_pk2_kernel(const float *__restrict__ series, float *__restrict__ dout,
                                                                int64_t hop, int64_t n_windows, int n, KP kp,
                                                                unsigned *fallbacks = nullptr,
                                                                const float *__restrict__ wpairs = nullptr) {
    static_assert(J == 32 && WU % J == 0, "8 lanes x 4 samples per row, whole tiles of warm-up");
    constexpr int RS = J + 2;  // row stride in pairs
    __shared__ __attribute__((aligned(16))) kf2 tiles[WAVES][64 * RS];
    extern __shared__ __attribute__((aligned(16))) kf2 wlds[];  // window pairs (wpairs != nullptr)
    typedef float f4v __attribute__((ext_vector_type(4)));
    const int l = threadIdx.x % 64, wv = WAVES > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x / 64) : 0;
    kf2 *tile = tiles[wv];
    const int64_t w0 = ((int64_t)blockIdx.x * WAVES + wv) * 64;
    const KConst<float> kc = kconst<float, kKfAdapt | kKfClip>(kp);
    const int L0 = (n + WU) / 2, seg_off = L0 - WU, nchunks = L0 / J;
    constexpr int WUC = WU / J;
    const int rl = l / 8, q = l % 8;  // IO: row rl of the instruction's 8, samples 4q .. 4q + 3
    const int64_t rows = n_windows - w0 < 64 ? (n_windows > w0 ? n_windows - w0 : 0) : 64;
    const auto rin = kbuf(series + (rows > 0 ? w0 * hop : 0), rows > 0 ? (uint32_t)(((rows - 1) * hop + n) * (int64_t)sizeof(float)) : 0u);
    const auto rout = kbuf(dout + w0 * (int64_t)n, (uint32_t)(rows * n * (int64_t)sizeof(float)));
    const uint32_t vin = (uint32_t)((rl * hop + 4 * q) * (int64_t)sizeof(float));
    const uint32_t vout = (uint32_t)((rl * n + 4 * q) * (int)sizeof(float));
    // instruction g (0..7) of segment s: rows 8 g + rl; uniform byte offsets
    auto in_off = [&](int g, int s) { return (uint32_t)(((8 * g) * hop + s * (int64_t)seg_off) * (int64_t)sizeof(float)); };
    auto out_off = [&](int g, int s) { return (uint32_t)(((8 * g) * (int64_t)n + s * (int64_t)seg_off) * (int64_t)sizeof(float)); };
    auto ld4 = [&](uint32_t voff, uint32_t soff) {
        return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rin, (int)voff, (int)soff, 0));
    };
    auto st4 = [&](f4v v, uint32_t voff, uint32_t soff) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rout, (int)voff, (int)soff, SCP);
    };
    // segment B's warm-up rows (ROT stores them so that every tile issues the same stores, see above): through an
    // empty descriptor, which drops them -- the same vmcnt bookkeeping without their 6 % of the written bytes
    const auto rnull = kbuf(dout, 0u);
    auto st4_warm = [&](f4v v, uint32_t voff, uint32_t soff, bool drop) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), drop ? rnull : rout, (int)voff, (int)soff, SCP);
    };
    f4v ra[8], rb[8];
    auto issue = [&](int c) {
        const uint32_t vc = vin + (uint32_t)(c * J * (int)sizeof(float));
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            ra[g] = ld4(vc, in_off(g, 0));
            rb[g] = ld4(vc, in_off(g, 1));
        }
    };
    auto tpos = [&](int g) { return (8 * g + rl) * RS + 4 * q; };  // pair index of an IO lane's first sample

    const bool win = wpairs != nullptr;
    if (win) {  // the window pairs into LDS, once per workgroup
        for (int i = threadIdx.x; i < L0; i += 64 * WAVES) wlds[i] = reinterpret_cast<const kf2 *>(wpairs)[i];
        __syncthreads();
    }
    KNb kn;
    if constexpr (NB) kn = knb_const(kp);
    kf2 emin = {__builtin_inff(), __builtin_inff()};  // NB: min over the steps of e (floor guard)
    KState2 st;
    kf2 base = {0.f, 0.f};  // each segment's centre: the first sample of its current tile
    KState<float> warm;  // segment B's state after its warm-up
    auto stage = [&]() {  // the loaded rows of both segments -> (A, B) pairs in the tile
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            f4v *t = reinterpret_cast<f4v *>(tile + tpos(g));
            t[0] = f4v{ra[g].x, rb[g].x, ra[g].y, rb[g].y};
            t[1] = f4v{ra[g].z, rb[g].z, ra[g].w, rb[g].w};
        }
    };
    // one whole pass over the window pair, in the Newton basis (PNB) or the original one
    auto pass = [&](auto nb_tag) {
    constexpr bool PNB = decltype(nb_tag)::value;
    // store_a: segment A's rows are stored (main pass); segment B's always are (ROT: also during its
    // warm-up, into segment A's later region)
    auto run = [&](int c0, int c1, int sA, int sB, auto store_a) {
        constexpr bool SA = decltype(store_a)::value;
        issue(c0);
        if constexpr (ROT) {
            stage();
            __syncthreads();
            if (c0 + 1 < c1) issue(c0 + 1);
        }
        for (int c = c0; c < c1; ++c) {
            if constexpr (!ROT) {
                stage();
                __syncthreads();
                if (c + 1 < c1) issue(c + 1);  // next tile in flight while the lanes filter this one
            }
            kf2 zrow[J], eprev;
#pragma unroll
            for (int j = 0; j < J; j += 2) {
                const f4v v = *reinterpret_cast<const f4v *>(tile + l * RS + j);
                zrow[j] = kf2{v.x, v.y};
                zrow[j + 1] = kf2{v.z, v.w};
            }
            // Re-centre both segments on a sample every kRecentre steps (the tile's first, then
            // inside the tile).  StepKalman4D is exactly shift-equivariant (only pos carries the
            // level: innovation, gain, boost and clip see differences), so moving the centre is
            // exact up to one rounding of pos per move, and pos stays at the size of the local
            // excursion instead of the distance from sample 0: a 0.5 level jump inside a window
            // then costs fp32 ~20x less (2-4e-5 -> 1-3e-6 of the spectrum,
            // scripts/kalman_f32_emulation.py).  base - zrow[j] is exact (Sterbenz).
            if (c == 0 && PNB) {
                knb_reset(st, kp);
            } else if (c == 0) {  // (sample 0, sample L0 - WU): both segments reset at their first sample
                KState<float> a;
                kreset<float>(a, kp, 0.f);
                st.pos = kf2{0.f, 0.f};
                st.vel = kf2{a.vel, a.vel}, st.acc = kf2{a.acc, a.acc}, st.jerk = kf2{a.jerk, a.jerk};
                st.p00 = kf2{a.p00, a.p00}, st.p11 = kf2{a.p11, a.p11}, st.p22 = kf2{a.p22, a.p22}, st.p33 = kf2{a.p33, a.p33};
                st.p01 = st.p02 = st.p03 = st.p12 = st.p13 = st.p23 = kf2{0.f, 0.f};
            } else {
                st.pos += base - zrow[0];
            }
            base = zrow[0];
#pragma unroll
            for (int j = 0; j < J; ++j) {
                if (j > 0 && j % kRecentre == 0) {  // and every kRecentre steps inside the tile
                    st.pos += base - zrow[j];
                    base = zrow[j];
                }
                const kf2 z = zrow[j] - base;  // exact for prices within 2x of the centre (Sterbenz)
                if constexpr (NB == 3) {  // tools: the tile IO alone (no filter)
                    zrow[j] = z;
                } else if constexpr (PNB) {
                    kf2 e;
                    const kf2 trend = kstep_nb2(st, kn, z, e);
                    zrow[j] = z - trend;
                    if (j % 2 == 0) {
                        eprev = e;
                    } else {  // one v_min3 per two steps and segment
                        emin.x = fminf(emin.x, fminf(eprev.x, e.x));
                        emin.y = fminf(emin.y, fminf(eprev.y, e.y));
                    }
                } else {
                    const kf2 trend = kstep_pk2(st, kc, z);
                    zrow[j] = z - trend;
                }
            }
            if (c == WUC - 1) {
                warm.pos = st.pos.y, warm.vel = st.vel.y, warm.acc = st.acc.y, warm.jerk = st.jerk.y;
                warm.p00 = st.p00.y, warm.p01 = st.p01.y, warm.p02 = st.p02.y, warm.p03 = st.p03.y;
                warm.p11 = st.p11.y, warm.p12 = st.p12.y, warm.p13 = st.p13.y, warm.p22 = st.p22.y;
                warm.p23 = st.p23.y, warm.p33 = st.p33.y;
            }
            if (win) {  // window values of samples c J + j (segment A) and seg_off + c J + j (B): broadcast LDS reads
#pragma unroll
                for (int j = 0; j < J; j += 2) {
                    const f4v h = *reinterpret_cast<const f4v *>(wlds + c * J + j);
                    zrow[j] *= kf2{h.x, h.y};
                    zrow[j + 1] *= kf2{h.z, h.w};
                }
            }
#pragma unroll
            for (int j = 0; j < J; j += 2)
                *reinterpret_cast<f4v *>(tile + l * RS + j) = f4v{zrow[j].x, zrow[j].y, zrow[j + 1].x, zrow[j + 1].y};
            __syncthreads();
            const uint32_t vc = vout + (uint32_t)(c * J * (int)sizeof(float));
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const f4v *t = reinterpret_cast<const f4v *>(tile + tpos(g));
                const f4v u = t[0], v = t[1];
                if (ROT ? SA : c >= sA) st4(f4v{u.x, u.z, v.x, v.z}, vc, out_off(g, 0));
                if (ROT || c >= sB) st4_warm(f4v{u.y, u.w, v.y, v.w}, vc, out_off(g, 1), c < sB);
            }
            __syncthreads();
            if constexpr (ROT) {
                if (c + 1 < c1) {
                    stage();  // waits for tile c + 1's loads only: this tile's stores stay in flight
                    __syncthreads();
                    if (c + 2 < c1) issue(c + 2);
                }
            }
        }
    };
    run(0, nchunks, 0, WUC, std::true_type{});
    if constexpr (NB == 3) return;  // tools: IO only, nothing to verify
    // segment A now holds the exact state after sample L0 - 1; segment B held its estimate of it.
    // Both are centred on sample L0 - kRecentre: segment A's last tile is segment B's tile WUC - 1.
    const float fl = 0x1p-24f * (fabsf(base.x) + fabsf(st.pos.x));
    const bool ok = kagree(st.pos.x, warm.pos, fl) && kagree(st.vel.x, warm.vel, fl) && kagree(st.acc.x, warm.acc, fl) &&
                    kagree(st.jerk.x, warm.jerk, fl) && kagree(st.p00.x, warm.p00, 0.f) && kagree(st.p01.x, warm.p01, 0.f) &&
                    kagree(st.p02.x, warm.p02, 0.f) && kagree(st.p03.x, warm.p03, 0.f) && kagree(st.p11.x, warm.p11, 0.f) &&
                    kagree(st.p12.x, warm.p12, 0.f) && kagree(st.p13.x, warm.p13, 0.f) && kagree(st.p22.x, warm.p22, 0.f) &&
                    kagree(st.p23.x, warm.p23, 0.f) && kagree(st.p33.x, warm.p33, 0.f);
    if (__ballot(!ok)) {  // wave-uniform: segment B's outputs [L0, N) again, from the exact state
        if (fallbacks && l == 0) atomicAdd(fallbacks, 1u);
        st.pos.y = st.pos.x, st.vel.y = st.vel.x, st.acc.y = st.acc.x, st.jerk.y = st.jerk.x;
        st.p00.y = st.p00.x, st.p01.y = st.p01.x, st.p02.y = st.p02.x, st.p03.y = st.p03.x;
        st.p11.y = st.p11.x, st.p12.y = st.p12.x, st.p13.y = st.p13.x, st.p22.y = st.p22.x;
        st.p23.y = st.p23.x, st.p33.y = st.p33.x;
        base.y = base.x;
        run(WUC, nchunks, nchunks, WUC, std::false_type{});  // only segment B stores
    }
    };
    if constexpr (NB == 0) {
        pass(std::false_type{});
    } else {
        pass(std::true_type{});
        // the floors were no-ops iff e >= -Qv/2 throughout (kstep_nb2); else the exact original-basis pass
        if (__ballot(NB == 2 || fminf(emin.x, emin.y) < kn.emin)) {
            if (fallbacks && l == 0) atomicAdd(fallbacks, 65536u);
            pass(std::false_type{});
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Four segments per window over a lane pair (fp32, default flags).  One wave per SIMD issues an
// instruction every ~5.5 cycles whatever its form, two waves per SIMD retire a packed one every
// ~3.6 (tools/valu_probe.hip, profiles/r02/valu_probe.log): the packed filter above is issue-bound
// at one wave per SIMD.  Here a wave holds 32 windows: lane l < 32 runs segments 0 and 1 of window
// l as a packed pair, lane l + 32 segments 2 and 3, so C3's 65536 windows are 2048 waves -- two per
// SIMD at <= 256 VGPRs.  Segment k starts cold at sample k S (S = L - WU; L = (N + 3 WU)/4 steps per
// lane), runs WU warm-up steps, then outputs [k S + WU, k S + L) (segment 0: [0, L)).  Hand-offs
// are verified in order, each against the exact (or already verified) state of the segment
// before it: 0 -> 1 and 2 -> 3 in-lane, 1 -> 2 across the pair (lane l -> l + 32); a failed check
// re-runs that segment's outputs from its predecessor's final state before the next check is made.
constexpr bool pk4_fits(int n, int J = 16, int WU = kPk2Warm) { return n >= 4 * WU && ((n + 3 * WU) / 4) % J == 0; }

__device__ __forceinline__ KState<float> kget(const KState2 &s, int h) {
    KState<float> r;
    auto g = [h](kf2 v) { return h ? v.y : v.x; };
    r.pos = g(s.pos), r.vel = g(s.vel), r.acc = g(s.acc), r.jerk = g(s.jerk);
    r.p00 = g(s.p00), r.p01 = g(s.p01), r.p02 = g(s.p02), r.p03 = g(s.p03), r.p11 = g(s.p11);
    r.p12 = g(s.p12), r.p13 = g(s.p13), r.p22 = g(s.p22), r.p23 = g(s.p23), r.p33 = g(s.p33);
    return r;
}
__device__ __forceinline__ void kset(KState2 &s, int h, const KState<float> &r) {
    auto p = [h](kf2 &v, float x) {
        if (h) v.y = x;
        else v.x = x;
    };
    p(s.pos, r.pos), p(s.vel, r.vel), p(s.acc, r.acc), p(s.jerk, r.jerk);
    p(s.p00, r.p00), p(s.p01, r.p01), p(s.p02, r.p02), p(s.p03, r.p03), p(s.p11, r.p11);
    p(s.p12, r.p12), p(s.p13, r.p13), p(s.p22, r.p22), p(s.p23, r.p23), p(s.p33, r.p33);
}
// the warm-up check of kalman_pk2_kernel: every component within 2^-16 relative, the state
// additionally within 2^-24 (|centre| + |pos|) absolute
__device__ __forceinline__ bool kagree_state(const KState<float> &e, const KState<float> &w, float centre) {
    const float fl = 0x1p-24f * (fabsf(centre) + fabsf(e.pos));
    return kagree(e.pos, w.pos, fl) && kagree(e.vel, w.vel, fl) && kagree(e.acc, w.acc, fl) && kagree(e.jerk, w.jerk, fl) &&
           kagree(e.p00, w.p00, 0.f) && kagree(e.p01, w.p01, 0.f) && kagree(e.p02, w.p02, 0.f) && kagree(e.p03, w.p03, 0.f) &&
           kagree(e.p11, w.p11, 0.f) && kagree(e.p12, w.p12, 0.f) && kagree(e.p13, w.p13, 0.f) && kagree(e.p22, w.p22, 0.f) &&
           kagree(e.p23, w.p23, 0.f) && kagree(e.p33, w.p33, 0.f);
}
__device__ __forceinline__ KState<float> kxor32_state(const KState<float> &s) {
    KState<float> r;
    r.pos = kxor32(s.pos), r.vel = kxor32(s.vel), r.acc = kxor32(s.acc), r.jerk = kxor32(s.jerk);
    r.p00 = kxor32(s.p00), r.p01 = kxor32(s.p01), r.p02 = kxor32(s.p02), r.p03 = kxor32(s.p03), r.p11 = kxor32(s.p11);
    r.p12 = kxor32(s.p12), r.p13 = kxor32(s.p13), r.p22 = kxor32(s.p22), r.p23 = kxor32(s.p23), r.p33 = kxor32(s.p33);
    return r;
}

// Single-wave workgroups (2 per SIMD by the 256-VGPR bound); tile and IO as kalman_pk2_kernel with
// tile row r = lane r, at J = 16 steps per tile (the J = 32 form spills at 256 VGPRs): 4 lanes per
// row, IO instruction g (0..3) moves tile rows 16 g .. 16 g + 15 = windows 16 (g % 2) + rl,
// segments 2 (g / 2) and 2 (g / 2) + 1.  Row stride J + 2 = 18 pairs: the filter's ds_read_b128 /
// ds_write_b128 (16 lanes, 16 rows) cover the 64 banks once; the IO accesses are 2-way.
template <int J, int WU = kPk2Warm>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void kalman_pk4_kernel(
    const float *__restrict__ series, float *__restrict__ dout, int64_t hop, int64_t n_windows, int n, KP kp,
    unsigned *fallbacks = nullptr) {
    static_assert((J == 16 || J == 32) && WU % J == 0, "4 samples per lane, whole tiles of warm-up");
    constexpr int RS = J + 2, LPR = J / 4, RPI = 64 / LPR, NG = 64 / RPI;  // lanes per row, rows per instruction
    __shared__ __attribute__((aligned(16))) kf2 tile[64 * RS];
    typedef float f4v __attribute__((ext_vector_type(4)));
    const int l = threadIdx.x;
    const bool hi = l >= 32;
    const int64_t w0 = (int64_t)blockIdx.x * 32;
    const KConst<float> kc = kconst<float, kKfAdapt | kKfClip>(kp);
    const int L = (n + 3 * WU) / 4, S = L - WU, nchunks = L / J;
    constexpr int WUC = WU / J;
    const int rl = l / LPR, q = l % LPR;
    const int64_t rows = n_windows - w0 < 32 ? (n_windows > w0 ? n_windows - w0 : 0) : 32;
    const auto rin = kbuf(series + (rows > 0 ? w0 * hop : 0), rows > 0 ? (uint32_t)(((rows - 1) * hop + n) * (int64_t)sizeof(float)) : 0u);
    const auto rout = kbuf(dout + w0 * (int64_t)n, (uint32_t)(rows * n * (int64_t)sizeof(float)));
    const uint32_t vin = (uint32_t)((rl * hop + 4 * q) * (int64_t)sizeof(float));
    const uint32_t vout = (uint32_t)((rl * n + 4 * q) * (int)sizeof(float));
    // instruction g: tile rows RPI g + rl = windows RPI (g % (NG/2)) + rl, segment pair g / (NG/2)
    auto in_off = [&](int g, int s) {
        return (uint32_t)(((RPI * (g % (NG / 2))) * hop + (2 * (g / (NG / 2)) + s) * (int64_t)S) * (int64_t)sizeof(float));
    };
    auto out_off = [&](int g, int s) {
        return (uint32_t)(((RPI * (g % (NG / 2))) * (int64_t)n + (2 * (g / (NG / 2)) + s) * (int64_t)S) * (int64_t)sizeof(float));
    };
    auto ld4 = [&](uint32_t voff, uint32_t soff) {
        return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rin, (int)voff, (int)soff, 0));
    };
    auto st4 = [&](f4v v, uint32_t voff, uint32_t soff) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rout, (int)voff, (int)soff, 0);
    };
    f4v ra[NG], rb[NG];
    auto issue = [&](int c) {
        const uint32_t vc = vin + (uint32_t)(c * J * (int)sizeof(float));
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            ra[g] = ld4(vc, in_off(g, 0));
            rb[g] = ld4(vc, in_off(g, 1));
        }
    };
    auto tpos = [&](int g) { return (RPI * g + rl) * RS + 4 * q; };

    KState2 st, warm2;
    kf2 base = {0.f, 0.f}, wbase = {0.f, 0.f};  // segment centres (first sample of the current tile), at WUC - 1
    // sm: segments whose rows this pass stores (segment k from chunk 0 if k == 0, else from WUC)
    auto run = [&](int c0, int c1, unsigned sm) {
        issue(c0);
        for (int c = c0; c < c1; ++c) {
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                f4v *t = reinterpret_cast<f4v *>(tile + tpos(g));
                t[0] = f4v{ra[g].x, rb[g].x, ra[g].y, rb[g].y};
                t[1] = f4v{ra[g].z, rb[g].z, ra[g].w, rb[g].w};
            }
            __syncthreads();
            if (c + 1 < c1) issue(c + 1);
            kf2 zrow[J];
#pragma unroll
            for (int j = 0; j < J; j += 2) {
                const f4v v = *reinterpret_cast<const f4v *>(tile + l * RS + j);
                zrow[j] = kf2{v.x, v.y};
                zrow[j + 1] = kf2{v.z, v.w};
            }
            if (c == 0) {  // every segment resets at its first sample; re-centred per tile (kalman_pk2_kernel)
                KState<float> a;
                kreset<float>(a, kp, 0.f);
                st.pos = kf2{0.f, 0.f};
                st.vel = kf2{a.vel, a.vel}, st.acc = kf2{a.acc, a.acc}, st.jerk = kf2{a.jerk, a.jerk};
                st.p00 = kf2{a.p00, a.p00}, st.p11 = kf2{a.p11, a.p11}, st.p22 = kf2{a.p22, a.p22}, st.p33 = kf2{a.p33, a.p33};
                st.p01 = st.p02 = st.p03 = st.p12 = st.p13 = st.p23 = kf2{0.f, 0.f};
            } else {
                st.pos += base - zrow[0];
            }
            base = zrow[0];
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const kf2 z = zrow[j] - base;
                const kf2 trend = kstep_pk2(st, kc, z);
                zrow[j] = z - trend;
            }
            if (c == WUC - 1) {
                warm2 = st;
                wbase = base;
            }
#pragma unroll
            for (int j = 0; j < J; j += 2)
                *reinterpret_cast<f4v *>(tile + l * RS + j) = f4v{zrow[j].x, zrow[j].y, zrow[j + 1].x, zrow[j + 1].y};
            __syncthreads();
            const uint32_t vc = vout + (uint32_t)(c * J * (int)sizeof(float));
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                const f4v *t = reinterpret_cast<const f4v *>(tile + tpos(g));
                const f4v u = t[0], v = t[1];
                const int k0 = 2 * (g / (NG / 2)), k1 = k0 + 1;
                if ((sm >> k0 & 1) && c >= (k0 == 0 ? 0 : WUC)) st4(f4v{u.x, u.z, v.x, v.z}, vc, out_off(g, 0));
                if ((sm >> k1 & 1) && c >= WUC) st4(f4v{u.y, u.w, v.y, v.w}, vc, out_off(g, 1));
            }
            __syncthreads();
        }
    };
    run(0, nchunks, 0xfu);
    const KState2 fin = st;
    // 0 -> 1 (lanes < 32): segment 1's warm-up against segment 0's exact final state
    KState<float> s1 = kget(fin, 1);
    // (a predecessor's last tile is its successor's tile WUC - 1: both states sit on the successor's wbase)
    if (__ballot(!hi && !kagree_state(kget(fin, 0), kget(warm2, 1), wbase.y))) {
        if (fallbacks && l == 0) atomicAdd(fallbacks, 1u);
        kset(st, 1, kget(fin, 0));
        base.y = wbase.y;
        run(WUC, nchunks, 0x2u);
        s1 = kget(st, 1);
    }
    // 1 -> 2 (across the pair): segment 2's warm-up (lane l + 32) against segment 1's final (lane l)
    s1 = kxor32_state(s1);
    KState<float> s2 = kget(fin, 0);
    if (__ballot(hi && !kagree_state(s1, kget(warm2, 0), wbase.x))) {
        if (fallbacks && l == 0) atomicAdd(fallbacks, 1u);
        kset(st, 0, s1);
        base.x = wbase.x;
        run(WUC, nchunks, 0x4u);
        s2 = kget(st, 0);
    }
    // 2 -> 3 (lanes >= 32)
    if (__ballot(hi && !kagree_state(s2, kget(warm2, 1), wbase.y))) {
        if (fallbacks && l == 0) atomicAdd(fallbacks, 1u);
        kset(st, 1, s2);
        base.y = wbase.y;
        run(WUC, nchunks, 0x8u);
    }
}

}  // namespace kcore

}  // namespace wsp
