// spectrum_kernels.hip -- fused sliding-window power-spectrum kernel for
// gfx950 (MI355X, CDNA4).
//
// One launch = the whole hot path of WaveSpecZZ for a batch of windows:
//   gather (1.1.0:765-769) -> detrend (none 1.1.0:1239 / mean
//   L/WaveSpecZZ_gpu_wip.mq5:940-950 / IIR trend L/WaveSpecZZ_1.0.2.mq5:3040-3053)
//   -> window (L/WaveSpecZZ_1.0.2.mq5:884-935, precomputed table)
//   -> real FFT (replaces FourierTransformManual L/WaveSpecZZ_1.0.2.mq5:938-974
//      and the DLL's gpu_fft_real_forward, Include/imports.mqh:7)
//   -> |X_k|^2, k < N/2 (FftProcessor::Run 1.1.0:529-530) or the packed
//      out[2k]=Re, out[2k+1]=Im layout (1.1.0:522-528).
//
// Design (DESIGN.md "Kernel"):
//  * A window of N real samples is FFT'd as an M = N/2 point complex FFT of
//    z[n] = x[2n] + i x[2n+1] plus a real-to-complex post-twiddle.  Loading
//    (x[2n], x[2n+1]) as one 16-B double2 gives z[n] directly.
//  * M/16 threads per window, 16 complex points per thread in registers;
//    Stockham autosort passes of radix 16/8/4/2 with a final radix-8 pass;
//    LDS only for the transposes between passes (SoA re/im, +1 pad per 16).
//  * The final pass gives thread t butterflies {t, B-t} (thread 0: {0, B/2}),
//    so Z[k] and Z[M-k] -- the pair the real post-processing needs -- are in
//    the same thread: no extra LDS round trip for the R2C step.
//  * Every workgroup holds 2048 complex points (1 window at N=4096, 2048/M
//    windows at smaller N) and walks the batch with a grid-stride loop.
//  * Detrend arithmetic is fp64 in both precisions (prices ~1.1 minus a trend
//    of the same size: fp32 would cancel catastrophically).
#include "wsp_internal.h"

namespace wsp {
namespace {

template <typename T> struct cpx { T re, im; };
template <typename T> struct V2;
template <> struct V2<double> { using t = double2; };
template <> struct V2<float> { using t = float2; };

template <typename T> __device__ __forceinline__ cpx<T> cadd(cpx<T> a, cpx<T> b) { return {a.re + b.re, a.im + b.im}; }
template <typename T> __device__ __forceinline__ cpx<T> csub(cpx<T> a, cpx<T> b) { return {a.re - b.re, a.im - b.im}; }
template <typename T> __device__ __forceinline__ cpx<T> cmul(cpx<T> a, cpx<T> b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
template <typename T> __device__ __forceinline__ cpx<T> cconj(cpx<T> a) { return {a.re, -a.im}; }

// cos(2 pi k/16); sin(2 pi k/16) = cos16(k - 4).
__host__ __device__ constexpr double cos16(int k) {
    constexpr double C1 = 0.92387953251128675613, C2 = 0.70710678118654752440, C3 = 0.38268343236508977173;
    switch (k & 15) {
    case 0: return 1.0;   case 1: return C1;    case 2: return C2;    case 3: return C3;
    case 4: return 0.0;   case 5: return -C3;   case 6: return -C2;   case 7: return -C1;
    case 8: return -1.0;  case 9: return -C1;   case 10: return -C2;  case 11: return -C3;
    case 12: return 0.0;  case 13: return C3;   case 14: return C2;   default: return C1;
    }
}
__host__ __device__ constexpr double sin16(int k) { return cos16(k - 4); }

// a * W16^k, W16 = e^{-2 pi i/16}; k is a compile-time constant after
// unrolling, so the switch folds and trivial factors cost no multiply.
template <typename T> __device__ __forceinline__ cpx<T> mulw16(cpx<T> a, int k) {
    const T h = T(0.70710678118654752440);
    switch (k & 15) {
    case 0: return a;
    case 4: return {a.im, -a.re};
    case 8: return {-a.re, -a.im};
    case 12: return {-a.im, a.re};
    case 2: return {(a.re + a.im) * h, (a.im - a.re) * h};
    case 6: return {(a.im - a.re) * h, -(a.im + a.re) * h};
    case 10: return {-(a.re + a.im) * h, (a.re - a.im) * h};
    case 14: return {(a.re - a.im) * h, (a.im + a.re) * h};
    default: {
        const T c = T(cos16(k)), s = T(sin16(k));
        return {a.re * c + a.im * s, a.im * c - a.re * s};
    }
    }
}

template <int LOG2R> __host__ __device__ constexpr int bitrev(int i) {
    int r = 0;
    for (int b = 0; b < LOG2R; ++b) r |= ((i >> b) & 1) << (LOG2R - 1 - b);
    return r;
}

// In-register R-point DFT (R = 2,4,8,16), natural order in and out.
template <typename T, int R> __device__ __forceinline__ void dft(cpx<T> *a) {
    constexpr int LR = R == 2 ? 1 : R == 4 ? 2 : R == 8 ? 3 : 4;
    cpx<T> b[R];
#pragma unroll
    for (int i = 0; i < R; ++i) b[bitrev<LR>(i)] = a[i];
#pragma unroll
    for (int s = 1; s <= LR; ++s) {
        const int len = 1 << s, half = len >> 1;
#pragma unroll
        for (int i = 0; i < R; i += len) {
#pragma unroll
            for (int j = 0; j < half; ++j) {
                const cpx<T> u = b[i + j];
                const cpx<T> v = mulw16(b[i + j + half], j * (16 / len));
                b[i + j] = cadd(u, v);
                b[i + j + half] = csub(u, v);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < R; ++i) a[i] = b[i];
}

template <int LOG2N> struct Geo {
    static constexpr int N = 1 << LOG2N;
    static constexpr int M = N / 2;        // complex points
    static constexpr int LOG2M = LOG2N - 1;
    static constexpr int TPW = M / 16;     // threads per window
    static constexpr int WPB = kBlock / TPW;  // windows per workgroup
    static constexpr int SLOT = M + M / 16;   // padded complex slots per window
    static constexpr int Q = LOG2M - 3;
    static constexpr int N16 = Q / 4, REM = Q % 4;
    static constexpr int NPASS = N16 + (REM ? 1 : 0) + 1;
    static constexpr int B = M / 8;        // butterflies of the final radix-8 pass
    static constexpr int radix(int p) { return p < N16 ? 16 : ((REM && p == N16) ? (1 << REM) : 8); }
    static constexpr int ns(int p) {
        int s = 1;
        for (int i = 0; i < p; ++i) s *= radix(i);
        return s;
    }
    static_assert(TPW >= 1 && TPW <= kBlock, "window size out of range");
};

__device__ __forceinline__ int pad16(int i) { return i + (i >> 4); }
__device__ __forceinline__ int pad32(int i) { return i + (i >> 5); }

template <typename T> struct SpecArgs {
    const T *__restrict__ series;
    T *__restrict__ out;
    const T *__restrict__ win;
    const cpx<T> *__restrict__ tw;
    int64_t hop, n_windows, n_groups;
    double alpha, c;
    double apow[8];
};

// Stockham pass p (0 < p < NPASS-1): LDS -> registers -> twiddle -> DFT -> LDS.
template <typename T, int LOG2N, int PASS>
__device__ __forceinline__ void mid_pass(T *sre, T *sim, const cpx<T> *__restrict__ tw, int t) {
    using G = Geo<LOG2N>;
    constexpr int R = G::radix(PASS), Ns = G::ns(PASS), BPT = 16 / R;
    constexpr int M = G::M, N = G::N, TPW = G::TPW;
    cpx<T> v[16];
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
        const int b = t + TPW * q;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = pad16(b + (M / R) * r);
            v[q * R + r] = {sre[i], sim[i]};
        }
        const cpx<T> w = tw[(b % Ns) * (N / (Ns * R))];
        cpx<T> wr = w;
#pragma unroll
        for (int r = 1; r < R; ++r) {
            v[q * R + r] = cmul(v[q * R + r], wr);
            if (r + 1 < R) wr = cmul(wr, w);
        }
        dft<T, R>(&v[q * R]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
        const int b = t + TPW * q;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = pad16((b / Ns) * Ns * R + (b % Ns) + Ns * r);
            sre[i] = v[q * R + r].re;
            sim[i] = v[q * R + r].im;
        }
    }
    __syncthreads();
}

template <typename T, int LOG2N, int PASS>
__device__ __forceinline__ void mid_passes(T *sre, T *sim, const cpx<T> *__restrict__ tw, int t) {
    if constexpr (PASS < Geo<LOG2N>::NPASS - 1) {
        mid_pass<T, LOG2N, PASS>(sre, sim, tw, t);
        mid_passes<T, LOG2N, PASS + 1>(sre, sim, tw, t);
    }
}

template <typename T, int LOG2N, int DETREND, int OUT, bool VEC>
__global__ __launch_bounds__(kBlock, 2) void spectrum_kernel(SpecArgs<T> a) {
    using G = Geo<LOG2N>;
    using v2 = typename V2<T>::t;
    constexpr int N = G::N, M = G::M, TPW = G::TPW, WPB = G::WPB, SLOT = G::SLOT, B = G::B;
    constexpr int R0 = G::radix(0), BPT0 = 16 / R0;
    constexpr int kCplx = 2 * WPB * SLOT * (int)sizeof(T);
    constexpr int kRaw = DETREND == kDetrendIir ? WPB * (N + N / 32) * 8 : 0;
    constexpr int kMain = kCplx > kRaw ? kCplx : kRaw;
    constexpr int kScan = 16 * 8;
    __shared__ __attribute__((aligned(16))) char smem[kMain + kScan];
    double *scanbuf = reinterpret_cast<double *>(smem + kMain);

    const int tid = threadIdx.x;
    const int slot = tid / TPW;
    const int t = tid % TPW;
    T *sre = reinterpret_cast<T *>(smem) + slot * SLOT;
    T *sim = reinterpret_cast<T *>(smem) + WPB * SLOT + slot * SLOT;
    const bool has_win = a.win != nullptr;

    for (int64_t g = blockIdx.x; g < a.n_groups; g += gridDim.x) {
        const int64_t w = g * WPB + slot;
        const bool active = w < a.n_windows;
        const T *__restrict__ xw = a.series + (active ? w : 0) * a.hop;

        // ---- gather: pass-0 layout, element (q, r) = z[(t + TPW q) + (M/R0) r]
        double xa[16], xb[16];
#pragma unroll
        for (int q = 0; q < BPT0; ++q)
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                const int n = (t + TPW * q) + (M / R0) * r;
                if constexpr (VEC) {
                    const v2 p = *reinterpret_cast<const v2 *>(xw + 2 * n);
                    xa[q * R0 + r] = p.x;
                    xb[q * R0 + r] = p.y;
                } else {
                    xa[q * R0 + r] = xw[2 * n];
                    xb[q * R0 + r] = xw[2 * n + 1];
                }
            }

        // ---- detrend (fp64)
        if constexpr (DETREND == kDetrendMean) {
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < 16; ++i) s += xa[i] + xb[i];
            constexpr int SW = TPW < 64 ? TPW : 64;
#pragma unroll
            for (int off = SW / 2; off >= 1; off >>= 1) s += __shfl_xor(s, off, SW);
            if constexpr (TPW == 128) {
                if ((tid & 63) == 0) scanbuf[tid >> 6] = s;
                __syncthreads();
                s = scanbuf[0] + scanbuf[1];
            }
            const double mean = s / (double)N;
#pragma unroll
            for (int i = 0; i < 16; ++i) { xa[i] -= mean; xb[i] -= mean; }
        } else if constexpr (DETREND == kDetrendIir) {
            // t0 = c(x0+x0), tj = c(xj+x(j-1)) + alpha t(j-1), d = x - t.
            // Chunk of 32 samples per thread, affine carry scan across threads.
            double *raw = reinterpret_cast<double *>(smem) + slot * (N + N / 32);
            __syncthreads();  // previous group's LDS reads are complete
#pragma unroll
            for (int q = 0; q < BPT0; ++q)
#pragma unroll
                for (int r = 0; r < R0; ++r) {
                    const int n = (t + TPW * q) + (M / R0) * r;
                    raw[pad32(2 * n)] = xa[q * R0 + r];
                    raw[pad32(2 * n + 1)] = xb[q * R0 + r];
                }
            __syncthreads();
            const double alpha = a.alpha, c = a.c;
            double xc[33];
            xc[0] = raw[pad32(t == 0 ? 0 : 32 * t - 1)];
#pragma unroll
            for (int j = 0; j < 32; ++j) xc[j + 1] = raw[pad32(32 * t + j)];
            double tr = 0.0;
#pragma unroll
            for (int j = 0; j < 32; ++j) tr = c * (xc[j + 1] + xc[j]) + alpha * tr;
            // inclusive scan: v_t = sum_{s<=t} alpha^(32(t-s)) e_s
            constexpr int SW = TPW < 64 ? TPW : 64;
            const int lt = t & (SW - 1);
            double v = tr;
#pragma unroll
            for (int j = 0, d = 1; d < SW; ++j, d <<= 1) {
                const double up = __shfl_up(v, d, SW);
                if (lt >= d) v = a.apow[j] * up + v;
            }
            double carry = __shfl_up(v, 1, SW);
            if constexpr (TPW == 128) {
                if (t == 63) scanbuf[0] = v;
                __syncthreads();
                if (t >= 64) {
                    const double v0 = scanbuf[0];
                    double p = 1.0;
                    const int m = lt + 1;
#pragma unroll
                    for (int j = 0; j < 7; ++j)
                        if ((m >> j) & 1) p *= a.apow[j];
                    v = p * v0 + v;
                    carry = __shfl_up(v, 1, SW);
                    if (lt == 0) carry = v0;
                }
            }
            if (t == 0) carry = 0.0;
            tr = carry;
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                tr = c * (xc[j + 1] + xc[j]) + alpha * tr;
                raw[pad32(32 * t + j)] = xc[j + 1] - tr;
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < BPT0; ++q)
#pragma unroll
                for (int r = 0; r < R0; ++r) {
                    const int n = (t + TPW * q) + (M / R0) * r;
                    xa[q * R0 + r] = raw[pad32(2 * n)];
                    xb[q * R0 + r] = raw[pad32(2 * n + 1)];
                }
        }

        // ---- window + pass 0 (no twiddles: Ns = 1)
        cpx<T> v[16];
#pragma unroll
        for (int q = 0; q < BPT0; ++q)
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                const int n = (t + TPW * q) + (M / R0) * r;
                T da = T(xa[q * R0 + r]), db = T(xb[q * R0 + r]);
                if (has_win) {
                    const v2 wv = *reinterpret_cast<const v2 *>(a.win + 2 * n);
                    da *= wv.x;
                    db *= wv.y;
                }
                v[q * R0 + r] = {da, db};
            }
#pragma unroll
        for (int q = 0; q < BPT0; ++q) dft<T, R0>(&v[q * R0]);
        __syncthreads();  // previous group's final-pass LDS reads are done
#pragma unroll
        for (int q = 0; q < BPT0; ++q) {
            const int b = t + TPW * q;
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                const int i = pad16(b * R0 + r);
                sre[i] = v[q * R0 + r].re;
                sim[i] = v[q * R0 + r].im;
            }
        }
        __syncthreads();

        // ---- middle passes
        mid_passes<T, LOG2N, 1>(sre, sim, a.tw, t);

        // ---- final radix-8 pass: thread t owns butterflies {t, B-t} ({0, B/2} for t = 0)
        const int bq[2] = {t, t == 0 ? TPW : 2 * TPW - t};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int i = pad16(bq[q] + B * r);
                v[q * 8 + r] = {sre[i], sim[i]};
            }
            if constexpr (G::NPASS > 1) {
                const cpx<T> w = a.tw[2 * bq[q]];  // (b % Ns) * N/(Ns*8) with Ns = B
                cpx<T> wr = w;
#pragma unroll
                for (int r = 1; r < 8; ++r) {
                    v[q * 8 + r] = cmul(v[q * 8 + r], wr);
                    if (r + 1 < 8) wr = cmul(wr, w);
                }
            }
            dft<T, 8>(&v[q * 8]);
        }

        // ---- real-to-complex post-processing + |X|^2
        // X[k] = E + W_N^k O, E = (Z[k] + conj Z[M-k])/2, O = -i (Z[k] - conj Z[M-k])/2
        const cpx<T> wt = a.tw[t];
        const cpx<T> w16c = {T(cos16(1)), T(-sin16(1))};
        const cpx<T> w32 = {T(0.98078528040323044913), T(-0.19509032201612826785)};
        const cpx<T> wb[2] = {wt, t == 0 ? w32 : cmul(w16c, cconj(wt))};
        if (active) {
#pragma unroll
            for (int q = 0; q < 2; ++q)
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const cpx<T> A = v[q * 8 + r];
                    const cpx<T> zp = q == 0 ? (t != 0 ? v[8 + (7 - r)] : v[(8 - r) & 7])
                                             : (t != 0 ? v[7 - r] : v[8 + (7 - r)]);
                    const cpx<T> e = {A.re + zp.re, A.im - zp.im};
                    const cpx<T> o = {A.im + zp.im, zp.re - A.re};  // -i (A - conj zp)
                    const cpx<T> wk = mulw16(wb[q], r);
                    const cpx<T> x2 = cadd(e, cmul(wk, o));    // 2 X[k]
                    const int k = bq[q] + B * r;
                    if constexpr (OUT == kOutPower) {
                        a.out[w * M + k] = T(0.25) * (x2.re * x2.re + x2.im * x2.im);
                    } else {
                        v2 o2;
                        o2.x = T(0.5) * x2.re;
                        o2.y = T(0.5) * x2.im;
                        *reinterpret_cast<v2 *>(a.out + w * N + 2 * k) = o2;
                    }
                }
        }
    }
}

template <typename T> struct TwoPow;

template <typename T, int LOG2N, int DETREND, int OUT, bool VEC>
hipError_t launch_one(const SpectrumLaunch &L, hipStream_t stream) {
    using G = Geo<LOG2N>;
    SpecArgs<T> a;
    a.series = static_cast<const T *>(L.series);
    a.out = static_cast<T *>(L.out);
    a.win = static_cast<const T *>(L.window);
    a.tw = static_cast<const cpx<T> *>(L.twiddle);
    a.hop = L.hop;
    a.n_windows = L.n_windows;
    a.n_groups = (L.n_windows + G::WPB - 1) / G::WPB;
    a.alpha = L.iir_alpha;
    a.c = L.iir_c;
    for (int j = 0; j < 8; ++j) a.apow[j] = L.iir_apow[j];
    int64_t grid = L.grid > 0 ? L.grid : 256 * 16;
    if (grid > a.n_groups) grid = a.n_groups;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((spectrum_kernel<T, LOG2N, DETREND, OUT, VEC>), dim3((unsigned)grid), dim3(kBlock), 0, stream,
                       a);
    return hipGetLastError();
}

template <typename T, int LOG2N, int DETREND, int OUT>
hipError_t dispatch_vec(const SpectrumLaunch &L, hipStream_t s) {
    const bool vec = (L.hop % 2 == 0) && ((reinterpret_cast<uintptr_t>(L.series) % (2 * sizeof(T))) == 0);
    return vec ? launch_one<T, LOG2N, DETREND, OUT, true>(L, s) : launch_one<T, LOG2N, DETREND, OUT, false>(L, s);
}

template <typename T, int LOG2N, int DETREND>
hipError_t dispatch_out(const SpectrumLaunch &L, hipStream_t s) {
    return L.output == kOutPacked ? dispatch_vec<T, LOG2N, DETREND, kOutPacked>(L, s)
                                  : dispatch_vec<T, LOG2N, DETREND, kOutPower>(L, s);
}

template <typename T, int LOG2N> hipError_t dispatch_detrend(const SpectrumLaunch &L, hipStream_t s) {
    switch (L.detrend) {
    case kDetrendNone: return dispatch_out<T, LOG2N, kDetrendNone>(L, s);
    case kDetrendMean: return dispatch_out<T, LOG2N, kDetrendMean>(L, s);
    case kDetrendIir: return dispatch_out<T, LOG2N, kDetrendIir>(L, s);
    default: return hipErrorInvalidValue;
    }
}

template <typename T> hipError_t dispatch_n(const SpectrumLaunch &L, hipStream_t s) {
    switch (L.log2n) {
    case 5: return dispatch_detrend<T, 5>(L, s);
    case 6: return dispatch_detrend<T, 6>(L, s);
    case 7: return dispatch_detrend<T, 7>(L, s);
    case 8: return dispatch_detrend<T, 8>(L, s);
    case 9: return dispatch_detrend<T, 9>(L, s);
    case 10: return dispatch_detrend<T, 10>(L, s);
    case 11: return dispatch_detrend<T, 11>(L, s);
    case 12: return dispatch_detrend<T, 12>(L, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_spectrum(const SpectrumLaunch &L, hipStream_t stream) {
    if (L.n_windows <= 0) return hipSuccess;
    return L.f32 ? dispatch_n<float>(L, stream) : dispatch_n<double>(L, stream);
}

}  // namespace wsp
