// spectrum_dispatch.h -- host-side argument setup and template dispatch of
// the spectrum kernel (one instantiation per N, detrend, output, window class).
#pragma once
#include <cmath>
#include <type_traits>

#include "spectrum_core.h"

namespace wsp {
namespace core {

// Window coefficients of L/WaveSpecZZ_1.0.2.mq5:884-922 as a0 + a1 cos th + a2 cos 2th.
inline int window_class(int window, double *a0, double *a1, double *a2) {
    *a0 = 1.0, *a1 = 0.0, *a2 = 0.0;
    switch (window) {
    case 1: *a0 = 0.5, *a1 = -0.5; return kWinCos;                  // Hann 0.5(1 - cos)
    case 2: *a0 = 0.54, *a1 = -0.46; return kWinCos;                // Hamming
    case 3: *a0 = 0.42, *a1 = -0.5, *a2 = 0.08; return kWinCos2;    // Blackman
    case 4: return kWinBartlett;
    default: return kWinNone;
    }
}

template <typename T> SpecArgs<T> make_args(const SpectrumLaunch &L, int wpb) {
    SpecArgs<T> a{};
    a.series = static_cast<const T *>(L.series);
    a.out = static_cast<T *>(L.out);
    a.tw = static_cast<const cpx<T> *>(L.twiddle);
    a.hop = L.hop;
    a.n_windows = L.n_windows;
    a.n_groups = (L.n_windows + wpb - 1) / wpb;
    // pair loads (x[2n], x[2n+1]) as one 16-B (f64) / 8-B (f32) access; gfx950 under ROCm runs in
    // unaligned-access mode, so element-aligned pairs (odd hop) are legal -- L.vec_mode 1 forces
    // the two-scalar path for A/B
    a.vec = L.vec_mode == 1 ? 0 : L.vec_mode == 2 ? 1 : ((L.hop % 2 == 0) && (reinterpret_cast<uintptr_t>(L.series) % (2 * sizeof(T)) == 0));
    // overlapping windows re-read samples from L2/MALL: keep them cacheable
    a.nt = L.nt_mode == 2 || (L.nt_mode == 0 && L.hop >= (int64_t(1) << L.log2n));
    const int wclass = window_class(L.window, &a.a0, &a.a1, &a.a2);
    if (wclass == kWinCos || wclass == kWinCos2) {
        // cosine windows carry the R2C step's factor 1/2 (spectrum_kernel: kS1, kS2)
        a.a0 *= 0.5;
        a.a1 *= 0.5;
        a.a2 *= 0.5;
    }
    const int n = 1 << L.log2n;
    const int m = n / 2;
    const int log2m = L.log2n - 1;
    const int q = log2m - 3;
    const int r0 = q / 4 > 0 ? 16 : (q % 4 ? (1 << (q % 4)) : 8);
    const long double two_pi = 6.283185307179586476925286766559005768L;
    const long double th = two_pi / (long double)(n - 1);
    a.inv_theta = (double)th;
    a.inv_nm1 = 1.0 / (double)(n - 1);
    a.cs = (double)cosl(th * (long double)(2 * (m / r0)));
    a.ss = (double)sinl(th * (long double)(2 * (m / r0)));
    a.co = (double)cosl(th);
    a.so = (double)sinl(th);
    a.topk = L.topk;
    a.kmin = L.kmin;
    a.kmax = L.kmax;
    a.alpha = L.iir_alpha;
    a.c = L.iir_c;
    for (int j = 0; j < 8; ++j) a.apow[j] = L.iir_apow[j];
    return a;
}

// Library default (profiles/r01/kbench_*.log, interleaved rounds): real/imag
// split LDS exchange (17.5 KiB, 3 waves/SIMD -> 6 workgroups/CU), no register
// prefetch, non-temporal 16-B stores of the LDS-staged power row, 32768
// workgroups grid-striding.  Sample loads are non-temporal only when windows
// do not overlap (a.nt).  The IIR path (33 KiB detrend staging caps it at 4
// workgroups/CU anyway) and the packed output (spills at 168 VGPRs) keep the
// AoS exchange at 2 waves/SIMD.
// Round-1 additions on every path (profiles/r01/kbench_hop1_n*.log, kbench_ns_b64.log): single-wave
// workgroups when a window fits one wave (no cross-wave s_barrier), Hann/Hamming by the 3-term
// recurrence, and -- split exchange -- single ds_read_b64 reads instead of the compiler's
// ds_read2_b64 pairs: hop = 1 at N = 512/1024/2048/4096 -7/-8/-7/-3 %, north star -2.5 %.
constexpr int kCommonVar = kVarNoPrefetch | kVarNtStore | kVarWave1 | kVarWinRec;
constexpr int kDefaultVar = kCommonVar | kVarSplitLds | kVarLdsB64;
constexpr int kDefaultGrid = 32768;
template <typename T, int LOG2N, int DETREND, int OUT> constexpr int default_var() {
    // the f32 mean path converts every sample to fp64 for the reduction and spills at 168;
    // N > 4096 runs one 256/512-thread workgroup per window, where the split exchange cannot
    // raise occupancy (LDS and VGPRs allow 2 waves/SIMD either way)
    // (the phase outputs keep the round-1 starting point: their register budget is the tightest)
    // (the top-k scan stages only its band, which fits the split slot when it spans at most about half
    // of the bins: dispatch_win falls back to the AoS slot for wider bands)
    // (top-k: the split exchange where one wave scans the band, N = 2048 / 4096 without detrend;
    // elsewhere its scan paths spill at 168 VGPRs)
    // (top-k + phase: the same split-exchange one-wave scan, then one wave for the winners' phases, round 4;
    // dispatch_win falls back to the AoS form when bins 0 .. kmax + 1 do not fit the split slot)
    if constexpr (OUT == kOutTopK || OUT == kOutTopKPhase)
        return (DETREND == kDetrendNone && (LOG2N == 11 || LOG2N == 12)) ? kDefaultVar
               : OUT == kOutTopK                                          ? kCommonVar
                                                                          : (kVarNoPrefetch | kVarNtStore);
    // (phase record: the AoS form; the split form, wsp_plan_set_variant 2, measured slower, round 5)
    return (OUT == kOutPhase) ? (kVarNoPrefetch | kVarNtStore)
           : (DETREND == kDetrendIir || OUT != kOutPower || (sizeof(T) == 4 && DETREND == kDetrendMean) || LOG2N > 12)
               ? kCommonVar
               : kDefaultVar;
}
// Can the split-exchange top-k instantiation take a band of `span` bins?  Its one-wave scan holds
// at most 8 bins per lane, and the band is staged in the window's split slot (SLOT elements of T).
template <typename T, int LOG2N, int VAR> constexpr bool band_fits(int span) {
    return !(VAR & kVarSplitLds) ||
           (span <= 64 * 8 && (int64_t)span * (int64_t)sizeof(cpx<T>) <= (int64_t)Geo<LOG2N>::SLOT * (int64_t)sizeof(T));
}
// The split-exchange top-k + phase form stages bins 0 .. kmax + 1 and its phase wave covers 64 x 16 bins.
template <typename T, int LOG2N, int VAR> constexpr bool phase_prefix_fits(int kmax, int span) {
    return !(VAR & kVarSplitLds) ||
           (span <= 64 * 8 && kmax + 2 <= 64 * 16 &&
            (int64_t)(kmax + 2) * (int64_t)sizeof(cpx<T>) <= (int64_t)Geo<LOG2N>::SLOT * (int64_t)sizeof(T));
}

// Non-temporal sample loads as a compile-time variant (kVarNtLoad) where the windows do not overlap:
// the run-time form (a.nt) costs the north-star kernel 4 % (539-540 vs 518 us per launch on one box,
// kbench store mode, profiles/r02/kbench_ns_ntload.log).  Instantiated for the power and top-k outputs at
// N >= 1024 without the IIR detrend (the phase outputs measured within noise of the run-time form and would
// double the longest translation unit); elsewhere a.nt still selects the loads at run time.
template <typename T, int LOG2N, int DETREND, int OUT, int VAR> constexpr bool ct_nt_variant() {
    return !(VAR & kVarNtLoad) && (OUT == kOutPower || OUT == kOutTopK) && LOG2N >= 10 && DETREND != kDetrendIir;
}

template <typename T, int LOG2N, int DETREND, int OUT, int WCLASS, int VAR = default_var<T, LOG2N, DETREND, OUT>()>
hipError_t launch_one(const SpectrumLaunch &L, hipStream_t stream) {
    if constexpr (ct_nt_variant<T, LOG2N, DETREND, OUT, VAR>()) {
        if (L.nt_mode == 2 || (L.nt_mode == 0 && L.hop >= (int64_t(1) << LOG2N)))
            return launch_one<T, LOG2N, DETREND, OUT, WCLASS, VAR | kVarNtLoad>(L, stream);
    }
    using G = Blk<LOG2N, VAR>;
    const SpecArgs<T> a = make_args<T>(L, G::WPB);
    int64_t grid = L.grid > 0 ? L.grid : kDefaultGrid;
    if (grid > a.n_groups) grid = a.n_groups;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((spectrum_kernel<T, LOG2N, DETREND, OUT, WCLASS, VAR>), dim3((unsigned)grid), dim3(G::BLOCK),
                       0, stream, a);
    return hipGetLastError();
}

template <typename T, int LOG2N, int DETREND, int OUT>
hipError_t dispatch_win(const SpectrumLaunch &L, hipStream_t s) {
    double a0, a1, a2;
    if constexpr (OUT == kOutTopKPhase && (default_var<T, LOG2N, DETREND, OUT>() & kVarSplitLds) != 0) {
        constexpr int kAos = kVarNoPrefetch | kVarNtStore;
        if (L.variant == 1 || !phase_prefix_fits<T, LOG2N, default_var<T, LOG2N, DETREND, OUT>()>(L.kmax, L.kmax - L.kmin + 1)) {
            switch (window_class(L.window, &a0, &a1, &a2)) {
            case kWinCos: return launch_one<T, LOG2N, DETREND, OUT, kWinCos, kAos>(L, s);
            case kWinCos2: return launch_one<T, LOG2N, DETREND, OUT, kWinCos2, kAos>(L, s);
            case kWinBartlett: return launch_one<T, LOG2N, DETREND, OUT, kWinBartlett, kAos>(L, s);
            default: return launch_one<T, LOG2N, DETREND, OUT, kWinNone, kAos>(L, s);
            }
        }
    }
    // the split-exchange phase record (round 5, wsp_plan_set_variant 2 at N = 2048 / 4096 without IIR): 3 waves per
    // SIMD, but 1.36 against 1.15 ms for the AoS form at the north star (r05g) -- an ablation, not the default
    if constexpr (OUT == kOutPhase && (LOG2N == 11 || LOG2N == 12) && DETREND != kDetrendIir) {
        if (L.variant == 2) {
            switch (window_class(L.window, &a0, &a1, &a2)) {
            case kWinCos: return launch_one<T, LOG2N, DETREND, OUT, kWinCos, kDefaultVar>(L, s);
            case kWinCos2: return launch_one<T, LOG2N, DETREND, OUT, kWinCos2, kDefaultVar>(L, s);
            case kWinBartlett: return launch_one<T, LOG2N, DETREND, OUT, kWinBartlett, kDefaultVar>(L, s);
            default: return launch_one<T, LOG2N, DETREND, OUT, kWinNone, kDefaultVar>(L, s);
            }
        }
    }
    if constexpr (OUT == kOutTopK && (default_var<T, LOG2N, DETREND, OUT>() & kVarSplitLds) != 0) {
        if (!band_fits<T, LOG2N, default_var<T, LOG2N, DETREND, OUT>()>(L.kmax - L.kmin + 1)) {
            switch (window_class(L.window, &a0, &a1, &a2)) {
            case kWinCos: return launch_one<T, LOG2N, DETREND, OUT, kWinCos, kCommonVar>(L, s);
            case kWinCos2: return launch_one<T, LOG2N, DETREND, OUT, kWinCos2, kCommonVar>(L, s);
            case kWinBartlett: return launch_one<T, LOG2N, DETREND, OUT, kWinBartlett, kCommonVar>(L, s);
            default: return launch_one<T, LOG2N, DETREND, OUT, kWinNone, kCommonVar>(L, s);
            }
        }
    }
    switch (window_class(L.window, &a0, &a1, &a2)) {
    case kWinCos: return launch_one<T, LOG2N, DETREND, OUT, kWinCos>(L, s);
    case kWinCos2: return launch_one<T, LOG2N, DETREND, OUT, kWinCos2>(L, s);
    case kWinBartlett: return launch_one<T, LOG2N, DETREND, OUT, kWinBartlett>(L, s);
    default: return launch_one<T, LOG2N, DETREND, OUT, kWinNone>(L, s);
    }
}

// OSET selects the output modes one translation unit instantiates:
// kSetBase = power / packed / top-k, kSetPhase = the fp64 phase outputs.
enum OutSet : int { kSetBase = 0, kSetPhase = 1 };

template <typename T, int LOG2N, int DETREND, int OSET>
hipError_t dispatch_out(const SpectrumLaunch &L, hipStream_t s) {
    if constexpr (OSET == kSetPhase) {
        switch (L.output) {
        case kOutPhase: return dispatch_win<T, LOG2N, DETREND, kOutPhase>(L, s);
        case kOutTopKPhase: return dispatch_win<T, LOG2N, DETREND, kOutTopKPhase>(L, s);
        default: return hipErrorInvalidValue;
        }
    } else {
        switch (L.output) {
        case kOutPower: return dispatch_win<T, LOG2N, DETREND, kOutPower>(L, s);
        case kOutPacked: return dispatch_win<T, LOG2N, DETREND, kOutPacked>(L, s);
        case kOutTopK: return dispatch_win<T, LOG2N, DETREND, kOutTopK>(L, s);
        default: return hipErrorInvalidValue;
        }
    }
}

template <typename T, int LOG2N, int OSET> hipError_t dispatch_detrend(const SpectrumLaunch &L, hipStream_t s) {
    switch (L.detrend) {
    case kDetrendNone: return dispatch_out<T, LOG2N, kDetrendNone, OSET>(L, s);
    case kDetrendMean: return dispatch_out<T, LOG2N, kDetrendMean, OSET>(L, s);
    case kDetrendIir: return dispatch_out<T, LOG2N, kDetrendIir, OSET>(L, s);
    default: return hipErrorInvalidValue;
    }
}

template <typename T, int OSET = kSetBase> hipError_t dispatch_n(const SpectrumLaunch &L, hipStream_t s) {
    if (L.n_windows <= 0) return hipSuccess;
    switch (L.log2n) {
    case 5: return dispatch_detrend<T, 5, OSET>(L, s);
    case 6: return dispatch_detrend<T, 6, OSET>(L, s);
    case 7: return dispatch_detrend<T, 7, OSET>(L, s);
    case 8: return dispatch_detrend<T, 8, OSET>(L, s);
    case 9: return dispatch_detrend<T, 9, OSET>(L, s);
    case 10: return dispatch_detrend<T, 10, OSET>(L, s);
    case 11: return dispatch_detrend<T, 11, OSET>(L, s);
    case 12: return dispatch_detrend<T, 12, OSET>(L, s);
    case 13: return dispatch_detrend<T, 13, OSET>(L, s);
    case 14: return dispatch_detrend<T, 14, OSET>(L, s);
    default: return hipErrorInvalidValue;
    }
}

// The log2 N in [LO, HI] part of dispatch_n: the library compiles its instantiations in several
// translation units (spectrum_f64*.hip, spectrum_f32*.hip, spectrum_phase*.hip) so they build in parallel.
template <typename T, int OSET, int LO, int HI> hipError_t dispatch_n_range(const SpectrumLaunch &L, hipStream_t s) {
    if (L.n_windows <= 0) return hipSuccess;
    hipError_t e = hipErrorInvalidValue;
    auto one = [&](auto lg) {
        constexpr int G = decltype(lg)::value;
        if constexpr (G >= LO && G <= HI)
            if (L.log2n == G) e = dispatch_detrend<T, G, OSET>(L, s);
    };
    one(std::integral_constant<int, 5>{});
    one(std::integral_constant<int, 6>{});
    one(std::integral_constant<int, 7>{});
    one(std::integral_constant<int, 8>{});
    one(std::integral_constant<int, 9>{});
    one(std::integral_constant<int, 10>{});
    one(std::integral_constant<int, 11>{});
    one(std::integral_constant<int, 12>{});
    one(std::integral_constant<int, 13>{});
    one(std::integral_constant<int, 14>{});
    return e;
}
constexpr int kSplitLog2N = 12;  // first log2 N of the second translation unit of each precision / output set

}  // namespace core
}  // namespace wsp
