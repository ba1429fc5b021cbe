// spectrum_core.h -- device code of the fused sliding-window power-spectrum
// kernel for gfx950 (MI355X, CDNA4).  Included by spectrum_kernels.hip (the
// library's dispatch) and by tools/kbench.hip (ablation variants).
//
// One launch = the whole hot path of WaveSpecZZ for a batch of windows:
//   gather (1.1.0:765-769) -> detrend (none 1.1.0:1239 / mean
//   L/WaveSpecZZ_gpu_wip.mq5:940-950 / IIR trend L/WaveSpecZZ_1.0.2.mq5:3040-3053)
//   -> window (L/WaveSpecZZ_1.0.2.mq5:884-935)
//   -> real FFT (replaces FourierTransformManual L/WaveSpecZZ_1.0.2.mq5:938-974
//      and the DLL's gpu_fft_real_forward, Include/imports.mqh:7)
//   -> |X_k|^2, k < N/2 (FftProcessor::Run 1.1.0:529-530) or the packed
//      out[2k]=Re, out[2k+1]=Im layout (1.1.0:522-528).
//
// Design (DESIGN.md "Kernel"):
//  * A window of N real samples is FFT'd as an M = N/2 point complex FFT of
//    z[n] = x[2n] + i x[2n+1] plus a real-to-complex post-twiddle; one 16-B
//    load of (x[2n], x[2n+1]) gives z[n].
//  * M/16 threads per window, 16 complex points per thread in registers;
//    Stockham autosort passes of radix 16/8/4/2 with a final radix-8 pass;
//    LDS only for the transposes between passes: complex AoS, one 16-B
//    element per ds_read_b128/ds_write_b128, +1 element pad per 16.
//  * The final pass gives thread t butterflies {t, B-t} (thread 0: {0, B/2}),
//    so Z[k] and Z[M-k] -- the pair the real post-processing needs -- sit in
//    the same thread: no extra LDS round trip for the R2C step.
//  * Each workgroup holds 2048 complex points (1 window at N=4096, 2048/M
//    windows at smaller N) and walks the batch with a grid-stride loop,
//    prefetching the next group's samples into registers while it
//    transforms the current one.
//  * Window coefficients a0 + a1 cos(th) + a2 cos(2 th), th = 2 pi i/(N-1),
//    come from a per-thread rotation recurrence (no table traffic).
//  * Detrend arithmetic is fp64 in both precisions (prices ~1.1 minus a trend
//    of the same size: fp32 would cancel catastrophically).
#pragma once
#include <type_traits>

#include "wsp_internal.h"

namespace wsp {
namespace core {

template <typename T> struct alignas(2 * sizeof(T)) cpx { T re, im; };
template <typename T> struct V2;
// clang ext vectors (not HIP's double2 struct): usable with the nontemporal builtins
typedef double d2v __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));
template <> struct V2<double> { using t = d2v; };
template <> struct V2<float> { using t = f2v; };

template <typename T> __device__ __forceinline__ cpx<T> cadd(cpx<T> a, cpx<T> b) { return {a.re + b.re, a.im + b.im}; }
template <typename T> __device__ __forceinline__ cpx<T> csub(cpx<T> a, cpx<T> b) { return {a.re - b.re, a.im - b.im}; }
template <typename T> __device__ __forceinline__ cpx<T> cmul(cpx<T> a, cpx<T> b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
template <typename T> __device__ __forceinline__ cpx<T> cconj(cpx<T> a) { return {a.re, -a.im}; }

// fp32: complex arithmetic on (re, im) register pairs as packed fp32 (v_pk_add / v_pk_mul / v_pk_fma_f32, the
// swaps and negations folded into op_sel / neg modifiers): one instruction per complex add and two per multiply
// instead of 2 and 4, and no v_mov to assemble the pairs the vectoriser otherwise forms ad hoc (the fp32 spectrum
// kernel is VALU-issue-bound: 0.97 of the issue slots, profiles/r04/sq/c3_sq_counters.csv)
__device__ __forceinline__ f2v pk(cpx<float> a) { return __builtin_bit_cast(f2v, a); }
__device__ __forceinline__ cpx<float> unpk(f2v a) { return __builtin_bit_cast(cpx<float>, a); }
template <> __device__ __forceinline__ cpx<float> cadd(cpx<float> a, cpx<float> b) { return unpk(pk(a) + pk(b)); }
template <> __device__ __forceinline__ cpx<float> csub(cpx<float> a, cpx<float> b) { return unpk(pk(a) - pk(b)); }
template <> __device__ __forceinline__ cpx<float> cmul(cpx<float> a, cpx<float> b) {
    const f2v A = pk(a), Bv = pk(b);
    return unpk(__builtin_elementwise_fma(A.yy, f2v{-Bv.y, Bv.x}, A.xx * Bv));
}

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
    if constexpr (std::is_same_v<T, float>) {  // packed: a c + (a.im, -a.re) s
        const f2v A = pk(a), J = f2v{A.y, -A.x};
        const float h = 0.70710678118654752440f;
        switch (k & 15) {
        case 0: return a;
        case 4: return unpk(J);
        case 8: return unpk(-A);
        case 12: return unpk(-J);
        case 2: return unpk((A + J) * h);
        case 6: return unpk((J - A) * h);
        case 10: return unpk((-A - J) * h);
        case 14: return unpk((A - J) * h);
        default: return unpk(__builtin_elementwise_fma(A, f2v{float(cos16(k)), float(cos16(k))}, J * float(sin16(k))));
        }
    }
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
    static constexpr int M = N / 2;           // complex points
    static constexpr int LOG2M = LOG2N - 1;
    static constexpr int TPW = M / 16;        // threads per window
    static constexpr int BLOCK = TPW > kBlock ? TPW : kBlock;  // threads per workgroup
    static constexpr int WPB = BLOCK / TPW;                    // windows per workgroup
    static constexpr int NWV = TPW >= 64 ? TPW / 64 : 1;       // waves per window
    static constexpr int SLOT = M + M / 16;   // padded complex slots per window
    static constexpr int Q = LOG2M - 3;
    static constexpr int N16 = Q / 4, REM = Q % 4;
    static constexpr int NPASS = N16 + (REM ? 1 : 0) + 1;
    static constexpr int B = M / 8;           // butterflies of the final radix-8 pass
    static constexpr int radix(int p) { return p < N16 ? 16 : ((REM && p == N16) ? (1 << REM) : 8); }
    static constexpr int ns(int p) {
        int s = 1;
        for (int i = 0; i < p; ++i) s *= radix(i);
        return s;
    }
    static constexpr int R0 = radix(0);
    static constexpr int BPT0 = 16 / R0;
    static_assert(TPW >= 1 && TPW <= 512, "window size out of range");
};

__device__ __forceinline__ int pad16(int i) { return i + (i >> 4); }
__device__ __forceinline__ int pad32(int i) { return i + (i >> 5); }
// One pad element per 2^PS: padS<4> = pad16.
template <int PS> __device__ __forceinline__ int padS(int i) { return i + (i >> PS); }
// padS(base + STRIDE*r) written so the per-r part is a compile-time constant
// (folds into the ds_read/ds_write immediate offset instead of one address
// VGPR per access): for STRIDE % 2^PS == 0, padS(x + STRIDE k) = padS(x) + (STRIDE + STRIDE/2^PS) k.
template <int STRIDE, int PS = 4> __device__ __forceinline__ int pad16_at(int pbase, int base, int r) {
    if constexpr (STRIDE % (1 << PS) == 0) return pbase + (STRIDE + (STRIDE >> PS)) * r;
    else return padS<PS>(base + STRIDE * r);
}
// Pad spacing of the exchange written by pass X.  The AoS exchange (16-B elements) and the first
// split exchange keep one pad per 16 (conflict-free 8-B writes of the radix-16 pass's lane-strided
// outputs; its reads of 32 consecutive elements then see one 2-way conflict, as the writes would
// under any other spacing).  The later split exchanges write runs of >= 16 consecutive elements:
// one pad per 64 / 128 at N = 2048 / 4096 makes both their 8-B writes and their 8-B reads
// conflict-free (exhaustive bank simulation of every widx/ridx pattern; at N = 1024 one pad per 32
// would too, but its mean-detrend instantiation then spills at 168 VGPRs).
template <int LOG2N, int X, bool SPLIT> constexpr int pad_shift() {
    return (SPLIT && X >= 1 && LOG2N >= 11 && LOG2N <= 12) ? LOG2N - 5 : 4;
}

// Window classes: none; a0 + a1 cos th + a2 cos 2th (Hann, Hamming, Blackman);
// Bartlett (evaluated exactly as L/WaveSpecZZ_1.0.2.mq5:918-922).
enum WClass : int { kWinNone = 0, kWinCos = 1, kWinBartlett = 2, kWinCos2 = 3 };  // kWinCos: a2 = 0
// Variant bits (tools/kbench.hip ablations; the library's defaults: default_var in spectrum_dispatch.h).
enum Var : int {
    kVarNoPrefetch = 1, kVarSkeleton = 2, kVarNtLoad = 4, kVarNtStore = 8, kVarBlocked = 16, kVarSkelWide = 32,
    kVarSplitLds = 64,  // real/imaginary halves exchanged separately: half the LDS, 3 waves/SIMD
    kVarOcc4 = 128,     // with kVarSplitLds: 4 waves/SIMD (8 workgroups/CU, <= 128 VGPRs)
    kVarTwTable = 256,  // twiddle powers loaded from the W_N^k table instead of product chains
    kVarWave1 = 512,    // single-wave workgroups when a window fits one wave (TPW <= 64): no s_barrier
    kVarDirectStore = 1024,  // power bins stored straight from registers (coalesced 8-B), no LDS staging
    kVarWinRec = 2048,  // Hann/Hamming values by a 3-term (Chebyshev) recurrence: 3 ops per sample, not 5
    kVarLdsB64 = 4096,  // with kVarSplitLds: exchange reads as single ds_read_b64 (no ds_read2_b64 pairing)
    kVarWinTab = 8192,  // window values (with the R2C factor 1/2) from an fp64 table a.win (L1/L2-resident)
    kVarVec = 16384,    // sample pairs known 2-element aligned: one 16-B (8-B) load per pair, no run-time test of a.vec
    kVarWtStore = 32768,  // power rows written through to memory (agent-scope sc1 buffer stores), no dirty L2 lines
};

// Workgroup shape of a variant: kVarWave1 shrinks the workgroup to one wave
// (64 / TPW windows) when a window needs at most 64 threads.
template <int LOG2N, int VAR> struct Blk {
    static constexpr int TPW = Geo<LOG2N>::TPW;
    static constexpr int BLOCK = ((VAR & kVarWave1) && TPW <= 64) ? 64 : Geo<LOG2N>::BLOCK;
    static constexpr int WPB = BLOCK / TPW;
};

template <typename T> struct SpecArgs {
    const T *__restrict__ series;
    T *__restrict__ out;
    const cpx<T> *__restrict__ tw;  // W_N^k, k < N
    int64_t hop, n_windows, n_groups;
    int vec;                         // 16-B (8-B for f32) pair loads are aligned
    int nt;                          // windows do not overlap: stream with non-temporal loads
    // window: a0 + a1 c + a2 (2c^2 - 1); rotation by step (cs, ss) per r and
    // by (co, so) from an even to the next odd sample
    double a0, a1, a2, cs, ss, co, so, inv_theta;  // inv_theta = 2 pi/(N-1)
    double inv_nm1;                  // 1/(N-1) for Bartlett
    const double *__restrict__ win;  // kVarWinTab: h(i)/2, i < N (cosine windows)
    int topk, kmin, kmax;            // kOutTopK(Phase): k slots over bins [kmin, kmax]
    double alpha, c;                 // IIR trend (L/WaveSpecZZ_1.0.2.mq5:3041-3043)
    double apow[8];                  // alpha^(32 * 2^j)
};

// LDS element index (padded) where pass PASS writes its element i = q*R + r.
template <int LOG2N, int PASS, int PS = 4> __device__ __forceinline__ int widx(int t, int i) {
    using G = Geo<LOG2N>;
    constexpr int R = G::radix(PASS), Ns = G::ns(PASS);
    const int q = i / R, r = i % R, b = t + G::TPW * q;
    if constexpr (PASS == 0) {
        // R consecutive elements: padS(b R + r) = padS(b R) + r (b R % 2^PS + r < 2^PS for R | 16 | 2^PS)
        return padS<PS>(b * R) + r;
    } else {
        const int base = (b / Ns) * Ns * R + (b % Ns);
        if constexpr (Ns < (1 << PS) && (Ns * R) % (1 << PS) == 0) {
            // base mod 2^PS = b mod Ns < Ns, and Ns | 2^PS: adding Ns r crosses a multiple of 2^PS exactly
            // at the compile-time r's where Ns r does, so the per-r part stays an immediate offset
            return padS<PS>(base) + Ns * r + ((Ns * r) >> PS);
        } else {
            return pad16_at<Ns, PS>(padS<PS>(base), base, r);
        }
    }
}

// LDS element index pass PASS reads its element i from (the final pass owns
// butterflies {t, B-t}, {0, B/2} for t = 0).
template <int LOG2N, int PASS, int PS = 4> __device__ __forceinline__ int ridx(int t, int i) {
    using G = Geo<LOG2N>;
    if constexpr (PASS == G::NPASS - 1) {
        const int q = i / 8, r = i % 8;
        const int b = q == 0 ? t : (t == 0 ? G::TPW : 2 * G::TPW - t);
        return pad16_at<G::B, PS>(padS<PS>(b), b, r);
    } else {
        constexpr int R = G::radix(PASS);
        const int q = i / R, r = i % R, b = t + G::TPW * q;
        return pad16_at<G::M / R, PS>(padS<PS>(b), b, r);
    }
}

// LDS transpose between passes: write v at widx<PASS>, read v at ridx<PASS+1>.
// AoS: one complex per ds_write_b128/ds_read_b128 (f64), 2 barriers.  SPLIT:
// real parts then imaginary parts through half the LDS, 4 barriers.
template <int SPLIT, typename T, int LOG2N, int PASS>
__device__ __forceinline__ void exchange(char *base, cpx<T> (&v)[16], int t) {
    if constexpr (!SPLIT) {
        cpx<T> *s = reinterpret_cast<cpx<T> *>(base);
        __syncthreads();  // every read of the previous contents is done
#pragma unroll
        for (int i = 0; i < 16; ++i) s[widx<LOG2N, PASS>(t, i)] = v[i];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = s[ridx<LOG2N, PASS + 1>(t, i)];
    } else {
        // SPLIT == 2: the reads go through a volatile view so that the compiler keeps them as
        // single ds_read_b64 (2 LDS cycles each) instead of pairing them into ds_read2_b64
        // (8 cycles for the same 16 bytes, MI355X_MICROARCH.md LDS table)
        T *s = reinterpret_cast<T *>(base);
        using RT = std::conditional_t<SPLIT == 2, const volatile __attribute__((address_space(3))) T,
                                      const __attribute__((address_space(3))) T>;
        RT *rs = (RT *)s;  // LDS address space: the volatile view must stay a ds_read, not a flat load
        constexpr int PS = sizeof(T) == 8 ? pad_shift<LOG2N, PASS, true>() : 4;  // 8-B elements (f64 halves)
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i) s[widx<LOG2N, PASS, PS>(t, i)] = v[i].re;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i].re = rs[ridx<LOG2N, PASS + 1, PS>(t, i)];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i) s[widx<LOG2N, PASS, PS>(t, i)] = v[i].im;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i].im = rs[ridx<LOG2N, PASS + 1, PS>(t, i)];
    }
}

// Stockham pass 0 < PASS < NPASS-1 on data already in its read layout:
// twiddle W^(r (b mod Ns)) then in-register radix-R DFTs, then the exchange.
// Multiplies v[r] (r = 1..R-1) by W_N^(r*k1): product chain of the base
// twiddle (VALU) or one table load per power (TABLE; |r*k1| < N).
template <bool TABLE, typename T, int R>
__device__ __forceinline__ void twiddle(cpx<T> *v, const cpx<T> *__restrict__ tw, int k1) {
    if constexpr (TABLE) {
#pragma unroll
        for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw[r * k1]);
    } else {
        const cpx<T> w = tw[k1];
        cpx<T> wr = w;
#pragma unroll
        for (int r = 1; r < R; ++r) {
            v[r] = cmul(v[r], wr);
            if (r + 1 < R) wr = cmul(wr, w);
        }
    }
}

template <int SPLIT, bool TABLE, typename T, int LOG2N, int PASS>
__device__ __forceinline__ void mid_passes(char *base, cpx<T> (&v)[16], const cpx<T> *__restrict__ tw, int t) {
    using G = Geo<LOG2N>;
    if constexpr (PASS < G::NPASS - 1) {
        constexpr int R = G::radix(PASS), Ns = G::ns(PASS), BPT = 16 / R;
        if constexpr (!TABLE && BPT > 1 && G::TPW % Ns == 0) {
            // every group q has b % Ns = t % Ns: one product chain of W^(r k1) serves all of them
            const cpx<T> w = tw[(t % Ns) * (G::N / (Ns * R))];
            cpx<T> wr = w;
#pragma unroll
            for (int r = 1; r < R; ++r) {
#pragma unroll
                for (int q = 0; q < BPT; ++q) v[q * R + r] = cmul(v[q * R + r], wr);
                if (r + 1 < R) wr = cmul(wr, w);
            }
#pragma unroll
            for (int q = 0; q < BPT; ++q) dft<T, R>(&v[q * R]);
        } else {
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                const int b = t + G::TPW * q;
                twiddle<TABLE, T, R>(&v[q * R], tw, (b % Ns) * (G::N / (Ns * R)));
                dft<T, R>(&v[q * R]);
            }
        }
        exchange<SPLIT, T, LOG2N, PASS>(base, v, t);
        mid_passes<SPLIT, TABLE, T, LOG2N, PASS + 1>(base, v, tw, t);
    }
}

// Lane exchanges that stay in the VALU: DPP row/quad permutations and the gfx950
// v_permlane16/32_swap (no LDS-crossbar round trip as with ds_bpermute).
template <int CTRL> __device__ __forceinline__ unsigned dpp_u32(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xf, 0xf, false);
}
template <typename T> struct Bits;
template <> struct Bits<double> {
    static constexpr int W = 2;
    __device__ static void split(double v, unsigned (&u)[2]) {
        const unsigned long long x = __builtin_bit_cast(unsigned long long, v);
        u[0] = (unsigned)x;
        u[1] = (unsigned)(x >> 32);
    }
    __device__ static double join(const unsigned (&u)[2]) {
        return __builtin_bit_cast(double, (unsigned long long)u[0] | ((unsigned long long)u[1] << 32));
    }
};
template <> struct Bits<float> {
    static constexpr int W = 1;
    __device__ static void split(float v, unsigned (&u)[1]) { u[0] = __builtin_bit_cast(unsigned, v); }
    __device__ static float join(const unsigned (&u)[1]) { return __builtin_bit_cast(float, u[0]); }
};

// Argmax of (p, b) under (p desc, b asc) over aligned segments of SW lanes (SW = 1..64, a power
// of two); every lane of a segment ends with the segment's winner.  The combine is idempotent,
// so the mirror steps and both halves of a permlane swap can be folded in unconditionally.
template <int SW, typename T> __device__ __forceinline__ void seg_argmax(T &p, int &b) {
    using BT = Bits<T>;
    auto comb = [&](T op, int ob) {
        if (op > p || (op == p && ob < b)) {
            p = op;
            b = ob;
        }
    };
    auto dpp_step = [&](auto ctrl) {
        constexpr int C = decltype(ctrl)::value;
        unsigned u[BT::W];
        BT::split(p, u);
#pragma unroll
        for (int i = 0; i < BT::W; ++i) u[i] = dpp_u32<C>(u[i]);
        comb(BT::join(u), (int)dpp_u32<C>((unsigned)b));
    };
    auto swap_step = [&](auto which) {
        unsigned u[BT::W], r0[BT::W], r1[BT::W];
        BT::split(p, u);
#pragma unroll
        for (int i = 0; i < BT::W; ++i) {
            const auto r = decltype(which)::value == 16 ? __builtin_amdgcn_permlane16_swap(u[i], u[i], false, false)
                                                         : __builtin_amdgcn_permlane32_swap(u[i], u[i], false, false);
            r0[i] = r[0];
            r1[i] = r[1];
        }
        const auto rb = decltype(which)::value == 16
                            ? __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false)
                            : __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
        comb(BT::join(r0), (int)rb[0]);
        comb(BT::join(r1), (int)rb[1]);
    };
    if constexpr (SW >= 2) dpp_step(std::integral_constant<int, 0xB1>{});   // quad_perm [1,0,3,2]
    if constexpr (SW >= 4) dpp_step(std::integral_constant<int, 0x4E>{});   // quad_perm [2,3,0,1]
    if constexpr (SW >= 8) dpp_step(std::integral_constant<int, 0x141>{});  // row_half_mirror
    if constexpr (SW >= 16) dpp_step(std::integral_constant<int, 0x140>{}); // row_mirror
    if constexpr (SW >= 32) swap_step(std::integral_constant<int, 16>{});   // rows 2i <-> 2i+1
    if constexpr (SW >= 64) swap_step(std::integral_constant<int, 32>{});   // lanes 0-31 <-> 32-63
}

// Same argmax as seg_argmax in two cheaper reductions: max of p (DPP-moved halves + v_max),
// then the minimum bin among the lanes whose own p equals that max.  Identical result for
// non-NaN p.
template <int SW, typename T> __device__ __forceinline__ void seg_argmax2(T p0, int b0, T &wp, int &wb) {
    using BT = Bits<T>;
    T m = p0;
    auto dpp_max = [&](auto ctrl) {
        constexpr int C = decltype(ctrl)::value;
        unsigned u[BT::W];
        BT::split(m, u);
#pragma unroll
        for (int i = 0; i < BT::W; ++i) u[i] = dpp_u32<C>(u[i]);
        m = fmax(m, BT::join(u));
    };
    auto swap_max = [&](auto which) {
        unsigned u[BT::W], r0[BT::W], r1[BT::W];
        BT::split(m, u);
#pragma unroll
        for (int i = 0; i < BT::W; ++i) {
            const auto r = decltype(which)::value == 16 ? __builtin_amdgcn_permlane16_swap(u[i], u[i], false, false)
                                                         : __builtin_amdgcn_permlane32_swap(u[i], u[i], false, false);
            r0[i] = r[0];
            r1[i] = r[1];
        }
        m = fmax(m, fmax(BT::join(r0), BT::join(r1)));
    };
    int b = p0 == m ? b0 : 0x7fffffff;  // placeholder: recomputed after the max is final
    if constexpr (SW >= 2) dpp_max(std::integral_constant<int, 0xB1>{});
    if constexpr (SW >= 4) dpp_max(std::integral_constant<int, 0x4E>{});
    if constexpr (SW >= 8) dpp_max(std::integral_constant<int, 0x141>{});
    if constexpr (SW >= 16) dpp_max(std::integral_constant<int, 0x140>{});
    if constexpr (SW >= 32) swap_max(std::integral_constant<int, 16>{});
    if constexpr (SW >= 64) swap_max(std::integral_constant<int, 32>{});
    b = p0 == m ? b0 : 0x7fffffff;
    auto dpp_min = [&](auto ctrl) { b = min(b, (int)dpp_u32<decltype(ctrl)::value>((unsigned)b)); };
    auto swap_min = [&](auto which) {
        const auto r = decltype(which)::value == 16 ? __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false)
                                                     : __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
        b = min(b, min((int)r[0], (int)r[1]));
    };
    if constexpr (SW >= 2) dpp_min(std::integral_constant<int, 0xB1>{});
    if constexpr (SW >= 4) dpp_min(std::integral_constant<int, 0x4E>{});
    if constexpr (SW >= 8) dpp_min(std::integral_constant<int, 0x141>{});
    if constexpr (SW >= 16) dpp_min(std::integral_constant<int, 0x140>{});
    if constexpr (SW >= 32) swap_min(std::integral_constant<int, 16>{});
    if constexpr (SW >= 64) swap_min(std::integral_constant<int, 32>{});
    wp = m;
    wb = b;
}

// Wave-wide (64-lane) max of a non-negative-or-sentinel T and min of an int: every lane ends with
// the result (DPP row steps, then the two permlane swaps).
template <typename T> __device__ __forceinline__ T wave_max64(T m) {
    using BT = Bits<T>;
    auto dpp_max = [&](auto ctrl) {
        constexpr int C = decltype(ctrl)::value;
        unsigned u[BT::W];
        BT::split(m, u);
#pragma unroll
        for (int i = 0; i < BT::W; ++i) u[i] = dpp_u32<C>(u[i]);
        m = fmax(m, BT::join(u));
    };
    auto swap_max = [&](auto which) {
        unsigned u[BT::W], r0[BT::W], r1[BT::W];
        BT::split(m, u);
#pragma unroll
        for (int i = 0; i < BT::W; ++i) {
            const auto r = decltype(which)::value == 16 ? __builtin_amdgcn_permlane16_swap(u[i], u[i], false, false)
                                                         : __builtin_amdgcn_permlane32_swap(u[i], u[i], false, false);
            r0[i] = r[0];
            r1[i] = r[1];
        }
        m = fmax(m, fmax(BT::join(r0), BT::join(r1)));
    };
    dpp_max(std::integral_constant<int, 0xB1>{});
    dpp_max(std::integral_constant<int, 0x4E>{});
    dpp_max(std::integral_constant<int, 0x141>{});
    dpp_max(std::integral_constant<int, 0x140>{});
    swap_max(std::integral_constant<int, 16>{});
    swap_max(std::integral_constant<int, 32>{});
    return m;
}
__device__ __forceinline__ int wave_min64(int b) {
    auto dpp_min = [&](auto ctrl) { b = min(b, (int)dpp_u32<decltype(ctrl)::value>((unsigned)b)); };
    auto swap_min = [&](auto which) {
        const auto r = decltype(which)::value == 16 ? __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false)
                                                     : __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
        b = min(b, min((int)r[0], (int)r[1]));
    };
    dpp_min(std::integral_constant<int, 0xB1>{});
    dpp_min(std::integral_constant<int, 0x4E>{});
    dpp_min(std::integral_constant<int, 0x141>{});
    dpp_min(std::integral_constant<int, 0x140>{});
    swap_min(std::integral_constant<int, 16>{});
    swap_min(std::integral_constant<int, 32>{});
    return b;
}

// Top-k of one window by ONE wave over the band staged at xb[j] = X[kmin + j], j < span (lane l
// holds j = l + 64 i, i < NB), in the reference's order (power desc, bin asc).  Per round: one
// wave-wide max of the lanes' best powers, then the winning lane from the ballot of lanes holding
// that max (scalar find-first, no second reduction chain); only a tie between lanes (equal powers)
// takes the min-over-bins reduction.  Lane r keeps round r's winner; lanes < k write the records
// at the end (one contiguous 4k-element row).
// RW: record width (4; 6 for kOutTopKPhase, whose fields 4-5 the caller adds); *slot_bin (optional): the bin of
// this lane's slot, -1 when empty.
template <int NB, typename T, int RW = 4>
__device__ __forceinline__ void topk_wave64(const cpx<T> *xb, int kmin, int span, int k, int lane, T *rec, bool active,
                                            int *winners = nullptr, int *slot_bin = nullptr) {
    // the lane's NB candidates sorted once (power desc, bin asc): its best is always p[0] and
    // retiring it is a shift, not a rescan
    T p[NB];
    int jj[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int j = lane + 64 * i;
        T v = T(-1);
        if (j < span) {
            const cpx<T> x = xb[j];
            v = x.re * x.re + x.im * x.im;
        }
        p[i] = v;
        jj[i] = j;
    }
    // insertion sort; ascending j within the lane, so strict '>' keeps the lower bin first on ties
#pragma unroll
    for (int i = 1; i < NB; ++i) {
#pragma unroll
        for (int q = i; q > 0; --q) {
            const bool sw = p[q] > p[q - 1];
            const T hi = sw ? p[q] : p[q - 1], lo = sw ? p[q - 1] : p[q];
            const int jh = sw ? jj[q] : jj[q - 1], jl = sw ? jj[q - 1] : jj[q];
            p[q - 1] = hi;
            p[q] = lo;
            jj[q - 1] = jh;
            jj[q] = jl;
        }
    }
    T my_p = T(-1);
    int my_j = -1;
    const int kk = k < 64 ? k : 64;
    using BT = Bits<T>;
    for (int r = 0; r < kk; ++r) {
        const T bp = p[0];
        if (__ballot(bp >= T(0)) == 0) break;  // nothing left in range (uniform)
        // the high word of a non-negative IEEE value orders like the value: max over it (integer DPP
        // steps), and usually one lane holds that word -> the winner without a second chain
        unsigned u[BT::W];
        BT::split(bp, u);
        const unsigned hi = bp >= T(0) ? u[BT::W - 1] : 0u;
        unsigned mh = hi;
        mh = max(mh, dpp_u32<0xB1>(mh));
        mh = max(mh, dpp_u32<0x4E>(mh));
        mh = max(mh, dpp_u32<0x141>(mh));
        mh = max(mh, dpp_u32<0x140>(mh));
        {
            const auto r16 = __builtin_amdgcn_permlane16_swap(mh, mh, false, false);
            mh = max(mh, max((unsigned)r16[0], (unsigned)r16[1]));
            const auto r32 = __builtin_amdgcn_permlane32_swap(mh, mh, false, false);
            mh = max(mh, max((unsigned)r32[0], (unsigned)r32[1]));
        }
        unsigned long long hold = __ballot(bp >= T(0) && hi == mh);
        int lw;
        if (__popcll(hold) == 1) {
            lw = __ffsll((long long)hold) - 1;
        } else {  // several lanes share the high word: exact max, then the lowest bin
            const T m = wave_max64(bp >= T(0) && hi == mh ? bp : T(-1));
            hold = __ballot(bp == m && bp >= T(0));
            if (__popcll(hold) == 1) {
                lw = __ffsll((long long)hold) - 1;
            } else {
                const int jm = wave_min64(bp == m ? jj[0] : 0x7fffffff);
                lw = __builtin_amdgcn_readfirstlane(jm) & 63;
            }
        }
        lw = __builtin_amdgcn_readfirstlane(lw);
        const int jw = __builtin_amdgcn_readlane(jj[0], lw);
        unsigned mu[BT::W];
#pragma unroll
        for (int i = 0; i < BT::W; ++i) mu[i] = (unsigned)__builtin_amdgcn_readlane((int)u[i], lw);
        if (lane == r) {
            my_p = BT::join(mu);
            my_j = jw;
        }
        if (lane == lw) {  // retire the winner: shift the lane's sorted candidates
#pragma unroll
            for (int i = 0; i + 1 < NB; ++i) {
                p[i] = p[i + 1];
                jj[i] = jj[i + 1];
            }
            p[NB - 1] = T(-1);
        }
    }
    if (winners && lane < k) winners[lane] = my_j;  // band index of slot `lane`, -1 when empty
    if (slot_bin) *slot_bin = my_j >= 0 ? kmin + my_j : -1;
    if (active && lane < k) {
        T *o = rec + RW * lane;
        if (my_j >= 0) {
            const cpx<T> x = xb[my_j];
            o[0] = T(kmin + my_j);
            o[1] = my_p;
            o[2] = x.re;
            o[3] = x.im;
        } else {  // empty slot
            o[0] = T(-1);
            o[1] = T(-1);
            o[2] = T(0);
            o[3] = T(0);
        }
    }
}

// k rounds of the top-k scan for one lane holding NB bins kmin + t + TPW i (i < NB).  Round r's
// winner (power desc, bin asc) goes to on_win(r, wp, wb, own); the owner retires its bin.
template <int NB, int SW, int TPW, typename T, typename XF, typename WF>
__device__ __forceinline__ void topk_rounds(int t, int kmin, int span, int k, XF power_of, WF on_win) {
    constexpr int kNone = 0x7fffffff;
    T p[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) p[i] = t + TPW * i < span ? power_of(kmin + t + TPW * i) : T(-1);
    T bp;
    int bi;
    auto lane_best = [&]() {  // ascending i = ascending bin: strict '>' keeps the lower bin
        bp = T(-1);
        bi = -1;
#pragma unroll
        for (int i = 0; i < NB; ++i)
            if (p[i] > bp) {
                bp = p[i];
                bi = i;
            }
    };
    lane_best();
    for (int r = 0; r < k; ++r) {
        const int mb = bi >= 0 ? kmin + t + TPW * bi : kNone;
        T wp;
        int wb;
        seg_argmax2<SW>(bp, mb, wp, wb);
        if (wp < T(0)) wb = kNone;  // nothing left in range
        const bool own = wb != kNone && wb == mb;
        if (own) {
#pragma unroll
            for (int i = 0; i < NB; ++i)
                if (i == bi) p[i] = T(-1);
            lane_best();
        }
        on_win(r, wp, wb, own);
    }
}

// atan2 with its polynomial coefficients in SGPRs (the split phase record, round 5): the operations of OCML's
// __ocml_atan2_f64 / __ocmlpriv_atanred_f64 (ROCm device library; min / max, one IEEE division, a degree-19 Horner
// polynomial in t^2 by fma, the same selects for the quadrants, +-0 and the non-finite cases), so the results are
// bit-identical to atan2() on the device; but the 20 coefficients are read from a constant table through a
// per-window pinned pointer -- scalar loads into SGPRs, one SGPR operand per v_fma_f64 -- instead of being
// materialised in 40 VGPRs and hoisted out of the window loop, which is what makes the inline atan2 spill (or, as
// a call, forces the caller-saved registers around 18 calls to scratch) at the 168-VGPR bound of 3 waves per SIMD.
__constant__ unsigned long long kAtanRed[20] = {
    0x3EEBA404B5E68A13ull, 0xBF23E260BD3237F4ull, 0x3F4B2BB069EFB384ull, 0xBF67952DAF56DE9Bull, 0x3F7D6D43A595C56Full,
    0xBF8C6EA4A57D9582ull, 0x3F967E295F08B19Full, 0xBF9E9AE6FC27006Aull, 0x3FA2C15B5711927Aull, 0xBFA59976E82D3FF0ull,
    0x3FA82D5D6EF28734ull, 0xBFAAE5CE6A214619ull, 0x3FAE1BB48427B883ull, 0xBFB110E48B207F05ull, 0x3FB3B13657B87036ull,
    0xBFB745D119378E4Full, 0x3FBC71C717E1913Cull, 0xBFC2492492376B7Dull, 0x3FC99999999952CCull, 0xBFD5555555555523ull};
__device__ __forceinline__ double atan2_sc(double y, double x, const unsigned long long *cf) {
    auto C = [&](int i) { return __builtin_bit_cast(double, cf[i]); };
    constexpr double kPiO2 = 1.5707963267948966, kPi = 3.1415926535897931, k3PiO4 = 2.3561944901923448,
                     kPiO4 = 0.78539816339744828;
    const double ay = fabs(y), ax = fabs(x);
    const double v = fmin(ax, ay) / fmax(ax, ay);
    const double v2 = v * v;
    double p = fma(v2, C(0), C(1));
#pragma unroll
    for (int i = 2; i < 20; ++i) p = fma(v2, p, C(i));
    const double r = fma(v, v2 * p, v);
    const bool xneg = __builtin_signbit(x);
    double a = ax < ay ? kPiO2 - r : r;
    a = xneg ? kPi - a : a;
    a = y == 0.0 ? (xneg ? kPi : 0.0) : a;
    if (ax == __builtin_inf() && ay == __builtin_inf()) a = xneg ? k3PiO4 : kPiO4;
    if (__builtin_isnan(x) || __builtin_isnan(y)) a = __builtin_nan("");
    return __builtin_copysign(a, y);
}

// atan2 as a call (the top-k + phase forms): inlined into the window loop, its ~19 fp64 polynomial coefficients are
// materialised in VGPRs once and hoisted out of the loop (38 VGPRs held across the FFT: 20-212 B/lane of spills in
// those forms); as a call they are rebuilt inside it, per call.  The full phase record (kOutPhase: 18 atan2 per
// lane, unspilled at N = 4096) keeps them inline for the interleaving of its independent atan2 chains.
__device__ __noinline__ double atan2_call(double y, double x) { return atan2(y, x); }

// Phase, unwrap and group delay of one window (CalculateFFTPhase, UnwrapPhase,
// CalculateGroupDelay: L/WaveSpecZZ_1.0.4-new.mq5:1040-1120, called at :3225-3227
// with n = N over the GPU unpack of :3183-3196, i.e. X_k for k < N/2 and zeros
// above).  X is staged in LDS at xrow[pad16(k)]; thread t owns bins
// [16t, 16t + 16) (TPW = M/16) and recomputes the phase of its two neighbour
// bins itself.  The reference's sequential unwrap u_i = u_(i-1) + diff + corr
// equals phi_i + 2 pi K_i with K_i the running count of +-1 corrections: K is
// an exact integer prefix scan and u is one fma, so only the rounding of the
// reference's running sum (not its decisions) differs.
// Lane l <- lane l - 1 (wave_shr:1) / lane l + 1 (wave_shl:1) across the whole wave, one 64-bit value as two DPP
// moves (gfx9 DPP; the lanes at the wave's ends read 0, and their callers do not use it).  tools/dpp_probe.hip
// checks the direction on the device.
__device__ __forceinline__ double dpp_from_prev_lane(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), 0x138, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double dpp_from_next_lane(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), 0x130, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

template <int LOG2N, int CH = 16, bool kCall = false, bool kDpp = false>
__device__ __forceinline__ void phase_chunk(const cpx<double> *xrow, int t, double *scanbuf, double (&pw)[CH],
                                            double (&u)[CH], double (&gd)[CH]) {
    // CH = bins per thread (16: the whole row; smaller for the top-k records, which only need the
    // bins up to the scan range: CH * TPW >= kmax + 2, chosen at run time by the caller)
    // kDpp (round 6, the full phase record): the two neighbour bins' phases are not recomputed -- they are the
    // adjacent lanes' own first / last phases, moved by DPP (16 atan2 per lane instead of 18).  Where the neighbour
    // lies in another wave of the window (N >= 4096: lane 0 of waves 1.., lane 63 of all but the last) the value
    // comes through LDS at the unwrap scan's barrier, and that wave boundary's correction is added to the counts
    // there.  The same atan2 values as recomputing them: bit-identical output.
    using G = Geo<LOG2N>;
    constexpr int M = G::M, TPW = G::TPW;
    constexpr double kPi = 3.14159265358979323846;  // M_PI
    constexpr double k2Pi = 2.0 * kPi;              // the reference's 2.0 * M_PI correction
    const int k0 = CH * t;
    constexpr int SW = TPW < 64 ? TPW : 64;
    const int lt = t & (SW - 1);
    double ph[CH + 2];  // bins k0 - 1 .. k0 + CH
    if constexpr (kDpp) {
        static_assert(CH == 16 && !kCall, "the DPP exchange serves the full phase record");
#pragma unroll
        for (int j = 1; j <= CH; ++j) {  // the thread's own bins, all < M
            const cpx<double> x = xrow[pad16(k0 - 1 + j)];
            ph[j] = atan2(x.im, x.re);
            pw[j - 1] = x.re * x.re + x.im * x.im;
        }
        const double prv = dpp_from_prev_lane(ph[CH]), nxt = dpp_from_next_lane(ph[1]);
        ph[0] = k0 == 0 ? 0.0 : prv;            // bin -1 does not exist (its correction is forced to 0)
        ph[CH + 1] = k0 + CH >= M ? 0.0 : nxt;  // bin M: the zeroed upper half, atan2(0, 0) = 0
    } else {
#pragma unroll
        for (int j = 0; j < CH + 2; ++j) {
            const int k = k0 - 1 + j;
            ph[j] = 0.0;  // bin M: the zeroed upper half, atan2(0, 0) = 0
            if (k >= 0 && k < M) {
                const cpx<double> x = xrow[pad16(k)];
                ph[j] = kCall ? atan2_call(x.im, x.re) : atan2(x.im, x.re);
                if (j >= 1 && j <= CH) pw[j - 1] = x.re * x.re + x.im * x.im;
            }
        }
    }
    // kDpp, several waves per window: lane 0 of waves 1.. and lane 63 of all waves but the last hold a neighbour
    // from another wave, fixed after the barrier below
    const bool wlead = kDpp && TPW >= 128 && lt == 0 && t > 0;
    const bool wtail = kDpp && TPW >= 128 && lt == 63 && k0 + CH < M;
    int cj[CH + 1];  // correction count of bins k0 .. k0 + CH (UnwrapPhase :1068-1077)
#pragma unroll
    for (int j = 0; j < CH + 1; ++j) {
        const double diff = ph[j + 1] - ph[j];
        cj[j] = (k0 + j == 0) ? 0 : diff > kPi ? -1 : diff < -kPi ? 1 : 0;
    }
    if (wlead) cj[0] = 0;  // the wave boundary's correction: added below
    int sum = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j) sum += cj[j];
    int incl = sum;
#pragma unroll
    for (int d = 1; d < SW; d <<= 1) {
        const int up = __shfl_up(incl, d, SW);
        if (lt >= d) incl += up;
    }
    int K = incl - sum;  // corrections of every bin < k0
    if constexpr (TPW >= 128) {  // add the totals of the window's earlier waves
        int *sb = reinterpret_cast<int *>(scanbuf + 8);
        double *bhi = scanbuf + 16, *blo = scanbuf + 16 + G::NWV;  // kDpp: each wave's last / first phase
        if (lt == 63) sb[t >> 6] = incl;
        if constexpr (kDpp) {
            if (lt == 63) bhi[t >> 6] = ph[CH];
            if (lt == 0) blo[t >> 6] = ph[1];
        }
        __syncthreads();
        const int wv = t >> 6;
        auto cw = [&](int i) {  // correction at wave i's first bin (i >= 1)
            const double diff = blo[i] - bhi[i - 1];
            return diff > kPi ? -1 : diff < -kPi ? 1 : 0;
        };
        for (int i = 0; i < wv; ++i) K += sb[i] + ((kDpp && i > 0) ? cw(i) : 0);
        if constexpr (kDpp) {
            if (wv > 0) {
                if (lt == 0) {
                    ph[0] = bhi[wv - 1];
                    cj[0] = cw(wv);
                } else {
                    K += cw(wv);
                }
            }
            if (wtail) {
                ph[CH + 1] = blo[wv + 1];
                const double diff = ph[CH + 1] - ph[CH];
                cj[CH] = diff > kPi ? -1 : diff < -kPi ? 1 : 0;
            }
        }
    }
    const double um1 = fma((double)K, k2Pi, ph[0]);  // u[k0 - 1]
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        K += cj[j];
        u[j] = fma((double)K, k2Pi, ph[j + 1]);
    }
    const double upc = fma((double)(K + cj[CH]), k2Pi, ph[CH + 1]);  // u[k0 + CH]
#pragma unroll
    for (int j = 0; j < CH; ++j) {  // :1102-1119 (n = N >= 32: every bin < M has two neighbours but bin 0)
        const double lo = j ? u[j - 1] : um1, hi = j < CH - 1 ? u[j + 1] : upc;
        double g = (k0 + j == 0) ? -(u[1] - u[0]) : -(hi - lo) / 2.0;
        if (g > 100.0) g = 100.0;
        if (g < -100.0) g = -100.0;
        gd[j] = g;
    }
}

// The unwrap's correction between consecutive bins (UnwrapPhase, L/WaveSpecZZ_1.0.4-new.mq5:1068-1077): -1 when
// atan2(B) - atan2(A) > pi, +1 when < -pi, else 0 -- decided from the half-planes and the cross product
// cross(A, B) = |A||B| sin(phi_B - phi_A) instead of two atan2: with both imaginary parts non-zero, a jump above
// pi needs phi_A < 0 < phi_B and sin < 0 (below -pi: phi_A > 0 > phi_B and sin > 0).  Where that test is not
// clear-cut -- an exactly zero imaginary part (the +-0 / +-pi conventions of atan2) or |sin| <= 1e-12, i.e.
// within 1e-12 rad of the tie, far beyond the few ulps by which the computed atan2 difference can be off --
// the decision is taken from the atan2 values themselves, so it is the one phase_chunk takes in every case.
__device__ __noinline__ int unwrap_corr_atan2(double ax, double ay, double bx, double by) {  // the rare path: a call
    constexpr double kPi = 3.14159265358979323846;
    const double diff = atan2(by, bx) - atan2(ay, ax);
    return diff > kPi ? -1 : diff < -kPi ? 1 : 0;
}
__device__ __forceinline__ int unwrap_corr(cpx<double> A, cpx<double> B) {
    const double ya = A.im, yb = B.im;
    if (ya != 0.0 && yb != 0.0) {
        if ((ya < 0.0) == (yb < 0.0)) return 0;  // same open half-plane: |diff| < pi
        const double cr = A.re * B.im - A.im * B.re;
        const double na = A.re * A.re + A.im * A.im, nb = B.re * B.re + B.im * B.im;
        if (cr * cr > 1e-24 * na * nb) return ya < 0.0 ? (cr < 0.0 ? -1 : 0) : (cr > 0.0 ? 1 : 0);
    }
    return unwrap_corr_atan2(A.re, A.im, B.re, B.im);
}

// [unwrapped phase, group delay] of the top-k winners by ONE wave (kOutTopKPhase on the split exchange), the values
// phase_chunk gives them: bins 0 .. kmax + 1 are staged at xrow[k] (bin M, the zeroed upper half, reads as 0).
// Lane l holds the corrections into bins [CH l, CH l + CH] as two bit masks (unwrap_corr: no atan2 but at near
// ties), the count before its chunk is an exact wave prefix sum, and atan2 runs only for each winner and its two
// neighbours (lane s: slot s, `bin` its bin or -1): u = phi + 2 pi K (the same fma), delay -(u[b+1] - u[b-1]) / 2
// (bin 0: -(u[1] - u[0])), clamped to +-100 (L/WaveSpecZZ_1.0.4-new.mq5:1102-1119).  64 CH >= kmax + 2.
template <int CH>
__device__ __forceinline__ void topk_phase_wave(const cpx<double> *xrow, int M, int kmax, int k, int lane_in, int bin,
                                                double *rec, bool active) {
    constexpr double k2Pi = 2.0 * 3.14159265358979323846;
    int lane = lane_in;
    asm volatile("" : "+v"(lane));  // per window: the lane's addresses are not hoisted out of the window loop
    static_assert(CH <= 16, "two 32-bit correction masks per lane");
    const int top = kmax + 1;  // highest bin any winner's unwrapped phase or delay reads
    auto X = [&](int kk) { return kk < M && kk <= top ? xrow[kk] : cpx<double>{0.0, 0.0}; };
    const int k0 = CH * lane;
    unsigned pos = 0u, neg = 0u;  // bit j: the correction into bin k0 + j is +1 / -1 (j = CH: the next chunk's first)
    cpx<double> prev = k0 > 0 ? X(k0 - 1) : cpx<double>{0.0, 0.0};
#pragma unroll 1
    for (int j = 0; j <= CH; ++j) {
        const int kk = k0 + j;
        if (kk > top) break;  // bins past kmax + 1 feed no winner
        const cpx<double> cur = X(kk);
        const int c = kk == 0 ? 0 : unwrap_corr(prev, cur);
        pos |= (c > 0 ? 1u : 0u) << j;
        neg |= (c < 0 ? 1u : 0u) << j;
        prev = cur;
    }
    const unsigned own = (1u << CH) - 1u;
    const int sum = __popc(pos & own) - __popc(neg & own);
    int incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int up = __shfl_up(incl, d, 64);
        if (lane >= d) incl += up;
    }
    const int K = incl - sum;  // corrections of every bin < k0
    // the 3k unwrapped phases u[b_s - 1], u[b_s], u[b_s + 1] of the k winners as items l = 3 s + i spread over the
    // lanes (one atan2 per lane and pass: a single pass for k <= 21), then gathered back to lane s
    double um = 0.0, u0 = 0.0, up = 0.0;
    const int passes = (3 * k + 63) / 64;
#pragma unroll 1
    for (int p = 0; p < passes; ++p) {
        const int l = 64 * p + lane, s = l / 3 < 64 ? l / 3 : 63, i = l - 3 * (l / 3);
        const int bs = __shfl(bin, s, 64);
        const int bb = (bs >= 0 ? bs : 0) - 1 + i < 0 ? 0 : (bs >= 0 ? bs : 0) - 1 + i;
        const int ob = bb / CH < 64 ? bb / CH : 63, jb = bb - CH * ob;
        const int Ko = __shfl(K, ob, 64);
        const unsigned po = (unsigned)__shfl((int)pos, ob, 64), no = (unsigned)__shfl((int)neg, ob, 64);
        const unsigned m = jb >= 31 ? 0xffffffffu : (2u << jb) - 1u;
        const int Kb = Ko + __popc(po & m) - __popc(no & m);
        const cpx<double> x = X(bb);
        const double uu = fma((double)Kb, k2Pi, bb < M ? atan2_call(x.im, x.re) : 0.0);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int src = 3 * lane + j;  // this lane's winner's item j
            const double v = __shfl(uu, src & 63, 64);
            if ((src >> 6) == p) {
                um = j == 0 ? v : um;
                u0 = j == 1 ? v : u0;
                up = j == 2 ? v : up;
            }
        }
    }
    const int b = bin >= 0 ? bin : 0;
    const double u3[3] = {um, u0, up};
    double g = b == 0 ? -(u3[2] - u3[1]) : -(u3[2] - u3[0]) / 2.0;
    if (g > 100.0) g = 100.0;
    if (g < -100.0) g = -100.0;
    if (active && lane < k) {
        rec[6 * lane + 4] = bin >= 0 ? u3[1] : 0.0;
        rec[6 * lane + 5] = bin >= 0 ? g : 0.0;
    }
}

// Loads the 16 sample pairs of this thread for group g (pass-0 layout,
// element (q, r) = z[(t + TPW q) + (M/R0) r]).  Inactive slots read window 0.
template <typename T, int LOG2N, int VAR = 0>
__device__ __forceinline__ void load_group(const SpecArgs<T> &a, int64_t g, int slot, int t,
                                           typename V2<T>::t (&raw)[16]) {
    using G = Geo<LOG2N>;
    using v2 = typename V2<T>::t;
    const int64_t w = g * Blk<LOG2N, VAR>::WPB + slot;
    const T *__restrict__ xw = a.series + (w < a.n_windows ? w : 0) * a.hop;
    if ((VAR & kVarVec) || a.vec) {
#pragma unroll
        for (int q = 0; q < G::BPT0; ++q)
#pragma unroll
            for (int r = 0; r < G::R0; ++r)
            {
                const v2 *p = reinterpret_cast<const v2 *>(xw + 2 * ((t + G::TPW * q) + (G::M / G::R0) * r));
                if ((VAR & kVarNtLoad) || a.nt) raw[q * G::R0 + r] = __builtin_nontemporal_load(p);
                else raw[q * G::R0 + r] = *p;
            }
    } else {
#pragma unroll
        for (int q = 0; q < G::BPT0; ++q)
#pragma unroll
            for (int r = 0; r < G::R0; ++r) {
                const int n = (t + G::TPW * q) + (G::M / G::R0) * r;
                raw[q * G::R0 + r].x = xw[2 * n];
                raw[q * G::R0 + r].y = xw[2 * n + 1];
            }
    }
}

// The same loads through a buffer descriptor based at the window (split top-k + phase form): one 32-bit lane offset
// and 16 scalar offsets instead of 16 64-bit addresses (32 VGPRs), which that form's 168-VGPR budget needs; the
// 16-B loads are element-aligned for odd hops (unaligned mode), so there is no two-scalar path either.
template <typename T, int LOG2N, int AUX>
__device__ __forceinline__ void load_group_buf_aux(__amdgpu_buffer_rsrc_t rs, int t, typename V2<T>::t (&raw)[16]) {
    using G = Geo<LOG2N>;
    using v2 = typename V2<T>::t;
#pragma unroll
    for (int q = 0; q < G::BPT0; ++q)
#pragma unroll
        for (int r = 0; r < G::R0; ++r) {
            const int voff = 2 * (t + G::TPW * q) * (int)sizeof(T), soff = 2 * (G::M / G::R0) * r * (int)sizeof(T);
            if constexpr (sizeof(T) == 8)
                raw[q * G::R0 + r] = __builtin_bit_cast(v2, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, AUX));
            else
                raw[q * G::R0 + r] = __builtin_bit_cast(v2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, AUX));
        }
}
// (a wave never straddles two windows here: TPW >= 64, so the window base is wave-uniform -- readfirstlane puts
// the descriptor in SGPRs)
template <typename T, int LOG2N>
__device__ __forceinline__ void load_group_buf(const SpecArgs<T> &a, int64_t w, int t, typename V2<T>::t (&raw)[16]) {
    using G = Geo<LOG2N>;
    static_assert(G::TPW >= 64, "one window per wave");
    const uint64_t base = reinterpret_cast<uint64_t>(a.series + (w < a.n_windows ? w : 0) * a.hop);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base), hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    T *xw = reinterpret_cast<T *>(((uint64_t)hi << 32) | lo);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(xw, (short)0, (int)(G::N * sizeof(T)), 0x00020000);
    if (a.nt) load_group_buf_aux<T, LOG2N, 2>(rs, t, raw);  // nt: streamed once when windows do not overlap
    else load_group_buf_aux<T, LOG2N, 0>(rs, t, raw);
}

template <typename T, int LOG2N, int DETREND, int OUT, int WCLASS, int VAR>
__global__ __launch_bounds__((Blk<LOG2N, VAR>::BLOCK),(VAR & kVarSplitLds) ? ((VAR & kVarOcc4) ? 4 : 3) : 2) void spectrum_kernel(SpecArgs<T> a) {
    using G = Geo<LOG2N>;
    using v2 = typename V2<T>::t;
    constexpr int N = G::N, M = G::M, TPW = G::TPW, WPB = Blk<LOG2N, VAR>::WPB, SLOT = G::SLOT, B = G::B, NWV = G::NWV;
    constexpr int R0 = G::R0, BPT0 = G::BPT0;
    constexpr bool kPrefetch = !(VAR & kVarNoPrefetch);
    constexpr int kSplit = (VAR & kVarSplitLds) ? ((VAR & kVarLdsB64) ? 2 : 1) : 0;
    // per-window LDS slot: the exchange's SLOT elements; the AoS phase record (round 6) stages two of its three rows
    // at once, 2 x (M + M/8) doubles, slightly more than the exchange's SLOT complex (occupancy unchanged: 4
    // workgroups per CU at N = 4096 either way)
    constexpr int kSlotB = (OUT == kOutPhase && !kSplit && 2 * (M + M / 8) * 8 > SLOT * (int)sizeof(cpx<T>))
                               ? 2 * (M + M / 8) * 8
                               : SLOT * (int)(kSplit ? sizeof(T) : sizeof(cpx<T>));
    constexpr int kCplx = WPB * kSlotB;
    constexpr int kRaw = DETREND == kDetrendIir ? WPB * (N + N / 32) * 8 : 0;
    constexpr int kMain = kCplx > kRaw ? kCplx : kRaw;
    constexpr bool kPhase = OUT == kOutPhase || OUT == kOutTopKPhase;
    // scan scratch: 16 doubles, + (top-k, two waves per window) two sorted lists and the merge
    // scan scratch: doubles [0, 8) wave totals of the mean / IIR reductions, [8, 16) the unwrap's
    // int wave totals; + (top-k with several waves per window) one sorted list per wave;
    // + (kOutTopKPhase) the winners of every window
    // + (kOutPhase, several waves per window) each wave's first and last phase (phase_chunk's DPP exchange)
    constexpr int kScan = 16 * 8 + ((OUT == kOutTopK || OUT == kOutTopKPhase) && TPW >= 128 ? NWV * 64 * (8 + 4) : 0) +
                          (OUT == kOutPhase && TPW >= 128 ? 2 * NWV * 8 : 0) +
                          (OUT == kOutTopKPhase ? WPB * (M < 64 ? M : 64) * 4 : 0);
    static_assert(!kPhase || sizeof(T) == 8, "phase outputs are fp64");
    constexpr bool kCosWin = WCLASS == kWinCos || WCLASS == kWinCos2;
    __shared__ __attribute__((aligned(16))) char smem[kMain + kScan];
    double *scanbuf = reinterpret_cast<double *>(smem + kMain);

    const int tid = threadIdx.x;
    const int slot = tid / TPW;
    int t = tid % TPW;  // re-pinned per window in the split top-k + phase form (below)
    char *lbase = smem + slot * kSlotB;  // this window's LDS slot

    // per-thread window rotation start: th_i at i = 2 (t + TPW q)
    double wc0[BPT0], ws0[BPT0];
    if constexpr (kCosWin) {
#pragma unroll
        for (int q = 0; q < BPT0; ++q) sincos(a.inv_theta * (double)(2 * (t + TPW * q)), &ws0[q], &wc0[q]);
    }

    // group sequence of this workgroup: cyclic (g = b + i*grid, the default:
    // the chip's in-flight windows stay one contiguous region) or blocked
    constexpr bool kBlocked = VAR & kVarBlocked;
    const int64_t per = kBlocked ? (a.n_groups + gridDim.x - 1) / gridDim.x : 0;
    const int64_t g_first = kBlocked ? (int64_t)blockIdx.x * per : (int64_t)blockIdx.x;
    const int64_t g_step = kBlocked ? 1 : (int64_t)gridDim.x;
    const int64_t g_end = kBlocked ? (g_first + per < a.n_groups ? g_first + per : a.n_groups) : a.n_groups;

    v2 raw[16];
    int64_t g = g_first;
    if (kPrefetch && g < g_end) load_group<T, LOG2N, VAR>(a, g, slot, t, raw);

    for (; g < g_end; g += g_step) {
        // split top-k + phase: every address and twiddle that depends on t is recomputed per window instead of being
        // hoisted out of the window loop -- the 168-VGPR budget of 3 waves per SIMD has no room for them
        if constexpr ((OUT == kOutTopKPhase || OUT == kOutPhase) && kSplit) asm volatile("" : "+v"(t));
        const int64_t w = g * WPB + slot;
        const bool active = w < a.n_windows;
        double xa[16], xb[16];
        if constexpr ((OUT == kOutTopKPhase || OUT == kOutPhase) && kSplit) {
            v2 rw[16];  // this window's samples only: nothing carried across windows
            load_group_buf<T, LOG2N>(a, w, t, rw);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                xa[i] = (double)rw[i].x;
                xb[i] = (double)rw[i].y;
            }
        } else {
            if (!kPrefetch) load_group<T, LOG2N, VAR>(a, g, slot, t, raw);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                xa[i] = (double)raw[i].x;
                xb[i] = (double)raw[i].y;
            }
        }
        if (kPrefetch && g + g_step < g_end) load_group<T, LOG2N, VAR>(a, g + g_step, slot, t, raw);

        // ---- detrend (fp64)
        if constexpr (DETREND == kDetrendMean) {
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < 16; ++i) s += xa[i] + xb[i];
            constexpr int SW = TPW < 64 ? TPW : 64;
#pragma unroll
            for (int off = SW / 2; off >= 1; off >>= 1) s += __shfl_xor(s, off, SW);
            if constexpr (TPW >= 128) {  // one window per workgroup: combine its waves
                __syncthreads();  // scanbuf reuse across groups
                if ((tid & 63) == 0) scanbuf[tid >> 6] = s;
                __syncthreads();
                s = 0.0;
#pragma unroll
                for (int i = 0; i < NWV; ++i) s += scanbuf[i];
            }
            const double mean = s / (double)N;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                xa[i] -= mean;
                xb[i] -= mean;
            }
        } else if constexpr (DETREND == kDetrendIir) {
            // t0 = c(x0+x0), tj = c(xj+x(j-1)) + alpha t(j-1), d = x - t.
            // Chunk of 32 samples per thread, affine carry scan across threads.
            double *rawl = reinterpret_cast<double *>(smem) + slot * (N + N / 32);
            __syncthreads();  // previous group's LDS reads are complete
#pragma unroll
            for (int q = 0; q < BPT0; ++q)
#pragma unroll
                for (int r = 0; r < R0; ++r) {
                    const int n = (t + TPW * q) + (M / R0) * r;
                    rawl[pad32(2 * n)] = xa[q * R0 + r];
                    rawl[pad32(2 * n + 1)] = xb[q * R0 + r];
                }
            __syncthreads();
            const double alpha = a.alpha, c = a.c;
            double xc[33];
            xc[0] = rawl[pad32(t == 0 ? 0 : 32 * t - 1)];
#pragma unroll
            for (int j = 0; j < 32; ++j) xc[j + 1] = rawl[pad32(32 * t + j)];
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
            if constexpr (TPW >= 128) {
                // state entering wave wv: G = sum_(i<wv) A^(wv-1-i) T_i over the earlier waves'
                // local totals T_i, A = alpha^(32*64) (one wave's 64 chunks)
                if (lt == 63) scanbuf[t >> 6] = v;
                __syncthreads();
                const int wv = t >> 6;
                if (wv > 0) {
                    double G = 0.0;
                    for (int i = 0; i < wv; ++i) G = a.apow[6] * G + scanbuf[i];
                    double p = 1.0;
                    const int m = lt + 1;
#pragma unroll
                    for (int j = 0; j < 7; ++j)
                        if ((m >> j) & 1) p *= a.apow[j];
                    v = p * G + v;
                    carry = __shfl_up(v, 1, SW);
                    if (lt == 0) carry = G;
                }
            }
            if (t == 0) carry = 0.0;
            tr = carry;
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                tr = c * (xc[j + 1] + xc[j]) + alpha * tr;
                rawl[pad32(32 * t + j)] = xc[j + 1] - tr;
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < BPT0; ++q)
#pragma unroll
                for (int r = 0; r < R0; ++r) {
                    const int n = (t + TPW * q) + (M / R0) * r;
                    xa[q * R0 + r] = rawl[pad32(2 * n)];
                    xb[q * R0 + r] = rawl[pad32(2 * n + 1)];
                }
        }

        // ---- window (fp64) + pass 0 (no twiddles: Ns = 1)
        cpx<T> v[16];
        constexpr bool kRec = (VAR & kVarWinRec) && WCLASS == kWinCos && R0 >= 8;
        if constexpr ((VAR & kVarWinTab) && kCosWin) {
#pragma unroll
            for (int q = 0; q < BPT0; ++q)
#pragma unroll
                for (int r = 0; r < R0; ++r) {
                    const d2v h = *reinterpret_cast<const d2v *>(a.win + 2 * ((t + TPW * q) + (M / R0) * r));
                    v[q * R0 + r] = {T(xa[q * R0 + r] * h.x), T(xb[q * R0 + r] * h.y)};
                }
        } else if constexpr (kRec) {
            // h(i) = a0 + a1 cos(th i) along the thread's even samples i = i0 + D r (D = 2M/R0) and
            // odd samples i0 + 1 + D r: h_(r+1) = 2C h_r - h_(r-1) + a0 (2 - 2C), C = cos(th D) = a.cs.
            // Seeds h_0, h_1 of both sequences from the per-thread rotation start; the recurrence
            // amplifies rounding by at most 1/sin(th D) (~2.6 at R0 = 16) over <= 15 steps.
            const double C2 = 2.0 * a.cs, K = a.a0 * (2.0 - C2);
#pragma unroll
            for (int q = 0; q < BPT0; ++q) {
                double c = wc0[q], s = ws0[q];
                asm volatile("" : "+v"(c), "+v"(s));  // recompute per window: no hoisted seeds
                const double c1 = c * a.cs - s * a.ss, s1 = s * a.cs + c * a.ss;
                double he0 = a.a0 + a.a1 * c, he1 = a.a0 + a.a1 * c1;
                double ho0 = a.a0 + a.a1 * (c * a.co - s * a.so), ho1 = a.a0 + a.a1 * (c1 * a.co - s1 * a.so);
#pragma unroll
                for (int r = 0; r < R0; ++r) {
                    v[q * R0 + r] = {T(xa[q * R0 + r] * he0), T(xb[q * R0 + r] * ho0)};
                    const double he2 = fma(C2, he1, K - he0), ho2 = fma(C2, ho1, K - ho0);
                    he0 = he1;
                    he1 = he2;
                    ho0 = ho1;
                    ho1 = ho2;
                }
            }
        } else {
#pragma unroll
        for (int q = 0; q < BPT0; ++q) {
            double c = 0.0, s = 0.0;
            if constexpr (kCosWin) {
                c = wc0[q];
                s = ws0[q];
                asm volatile("" : "+v"(c), "+v"(s));  // recompute per window: no 64-VGPR hoist
            }
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                double da = xa[q * R0 + r], db = xb[q * R0 + r];
                if constexpr (kCosWin) {
                    const double co = c * a.co - s * a.so;  // th_(i+1)
                    if constexpr (WCLASS == kWinCos2) {      // Blackman: + a2 cos 2th
                        da *= a.a0 + a.a1 * c + a.a2 * (2.0 * c * c - 1.0);
                        db *= a.a0 + a.a1 * co + a.a2 * (2.0 * co * co - 1.0);
                    } else {                                 // Hann 0.5(1 - cos), Hamming
                        da *= a.a0 + a.a1 * c;
                        db *= a.a0 + a.a1 * co;
                    }
                    const double cn = c * a.cs - s * a.ss;
                    s = s * a.cs + c * a.ss;
                    c = cn;
                } else if constexpr (WCLASS == kWinBartlett) {
                    int tq = t + TPW * q;
                    asm volatile("" : "+v"(tq));  // recompute per window: no hoisted 32-value table
                    const int i = 2 * (tq + (M / R0) * r);
                    da *= 1.0 - fabs((2.0 * i - N + 1) * a.inv_nm1);
                    db *= 1.0 - fabs((2.0 * (i + 1) - N + 1) * a.inv_nm1);
                }
                v[q * R0 + r] = {T(da), T(db)};
            }
        }
        }  // !kRec

        if constexpr (VAR & kVarSkelWide) {
            // memory-pattern ablation with 16-B contiguous stores
            if (active) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    v2 o;
                    o.x = v[2 * j].re + v[2 * j].im;
                    o.y = v[2 * j + 1].re + v[2 * j + 1].im;
                    *reinterpret_cast<v2 *>(a.out + w * M + 2 * (t + TPW * j)) = o;
                }
            }
            continue;
        }
        if constexpr (VAR & kVarSkeleton) {
            // memory-pattern ablation: same loads and stores, no transform
            if (active) {
#pragma unroll
                for (int q = 0; q < 2; ++q)
#pragma unroll
                    for (int r = 0; r < 8; ++r) {
                        const int k = (q == 0 ? t : (t == 0 ? TPW : 2 * TPW - t)) + B * r;
                        a.out[w * M + k] = v[q * 8 + r].re + v[q * 8 + r].im;
                    }
            }
            continue;
        }

#pragma unroll
        for (int q = 0; q < BPT0; ++q) dft<T, R0>(&v[q * R0]);
        exchange<kSplit, T, LOG2N, 0>(lbase, v, t);  // also orders the previous group's reads
        mid_passes<kSplit, (VAR & kVarTwTable) != 0, T, LOG2N, 1>(lbase, v, a.tw, t);

        // ---- final radix-8 pass: thread t owns butterflies {t, B-t} ({0, B/2} for t = 0)
        const int bq0 = t, bq1 = t == 0 ? TPW : 2 * TPW - t;
        cpx<T> u0[8], u1[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            u0[r] = v[r];
            u1[r] = v[8 + r];
        }
        if constexpr (G::NPASS > 1) {  // (b % Ns) * N/(Ns*8) = 2b with Ns = B
            twiddle<(VAR & kVarTwTable) != 0, T, 8>(u0, a.tw, 2 * bq0);
            twiddle<(VAR & kVarTwTable) != 0, T, 8>(u1, a.tw, 2 * bq1);
        }
        dft<T, 8>(u0);
        dft<T, 8>(u1);
        // u0[r] = Z[t + B r], u1[r] = Z[(B - t) + B r] = conj-partner of u0[7 - r].
        // Thread 0 holds Z[B r] and Z[B/2 + B r]; permute it into the same
        // slot pattern (slot s pairs u0[s] with u1[7-s], M - k_A = k_B).
        if (t == 0) {
            cpx<T> n0[8], n1[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                n0[r] = u1[r];           // k = B/2 + B r   <->  u1[7-r]
                n0[4 + r] = u0[r];       // k = B r  (slot 4: Z[0], special)
                n1[4 + r] = u1[4 + r];
            }
            n1[0] = u0[5];               // partner of u0[3]: B*5 = M - 3B
            n1[1] = u0[6];
            n1[2] = u0[7];
            n1[3] = u0[4];               // slot 4 partner: Z[M/2] (special)
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                u0[r] = n0[r];
                u1[r] = n1[r];
            }
        }

        // ---- real-to-complex post-processing + |X|^2, one slot per (k, M-k):
        // E = (Z[k] + conj Z[M-k])/2, O = -i (Z[k] - conj Z[M-k])/2,
        // X[k] = E + W_N^k O, X[M-k] = conj(E - W_N^k O).
        // the 1/2 of E, O (and 1/4 of |X|^2): folded into the window coefficients for the cosine
        // windows (make_args halves a0, a1, a2 -- an exact power-of-two scaling, bit-identical results)
        constexpr T kS1 = kCosWin ? T(1) : T(0.5), kS2 = kCosWin ? T(1) : T(0.25);
        T *prow = reinterpret_cast<T *>(lbase);  // power row staged in this window's LDS slot
        constexpr bool kDirect = OUT == kOutPower && (VAR & kVarDirectStore);
        if constexpr (OUT != kOutPacked && !kDirect) __syncthreads();  // every final-pass LDS read is done
        // bin indices and twiddle of the R2C slots; for the split top-k + phase form recomputed here (pinned after the
        // barrier), so that neither the twiddle load nor the 16 staging addresses and bound tests are issued at the
        // top of the window and held (spilled) across its FFT
        int tb0 = t;
        if constexpr ((OUT == kOutTopKPhase || OUT == kOutPhase) && kSplit) asm volatile("" : "+v"(tb0));
        constexpr bool kPhaseSplit = OUT == kOutPhase && kSplit != 0;
        double pim[kPhaseSplit ? 16 : 1];  // split phase record: Im X of the R2C slots, held until the slot is free
        const cpx<T> wt = a.tw[tb0];
        const cpx<T> wlo = tb0 == 0 ? cpx<T>{T(0.98078528040323044913), T(-0.19509032201612826785)} : wt;  // W_N^(B/2)
        const cpx<T> whi = tb0 == 0 ? cpx<T>{T(0), T(1)} : wt;  // W16^-4: slot s >= 4 of thread 0 -> W16^(s-4)
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const cpx<T> A = u0[s], Bv = u1[7 - s];
            const cpx<T> wk = mulw16(s < 4 ? wlo : whi, s);
            const cpx<T> e = {A.re + Bv.re, A.im - Bv.im};
            const cpx<T> o = {A.im + Bv.im, Bv.re - A.re};
            const cpx<T> wo = cmul(wk, o);
            cpx<T> xa = cadd(e, wo);                   // 2 X[k_A]
            cpx<T> xb = {e.re - wo.re, wo.im - e.im};  // 2 X[M - k_A]
            int ka = tb0 + B * s, kb = M - ka;
            if (tb0 == 0) {
                ka = s < 4 ? B / 2 + B * s : B * (s - 4);
                kb = s == 4 ? M / 2 : M - ka;
                if (s == 4) {  // self-paired bins: X[0] real, X[M/2] = conj Z[M/2]
                    xa = {T(2) * (A.re + A.im), T(0)};
                    xb = {T(2) * Bv.re, T(-2) * Bv.im};
                }
            }
            if constexpr (kDirect) {  // lanes t, t+1 -> bins ka, ka+1 (kb, kb-1): 512-B runs per wave store
                if (active) {
                    const T pa = kS2 * (xa.re * xa.re + xa.im * xa.im);
                    const T pb = kS2 * (xb.re * xb.re + xb.im * xb.im);
                    if constexpr (VAR & kVarNtStore) {
                        __builtin_nontemporal_store(pa, a.out + w * M + ka);
                        __builtin_nontemporal_store(pb, a.out + w * M + kb);
                    } else {
                        a.out[w * M + ka] = pa;
                        a.out[w * M + kb] = pb;
                    }
                }
            } else if constexpr (OUT == kOutPower) {
                prow[ka] = kS2 * (xa.re * xa.re + xa.im * xa.im);
                prow[kb] = kS2 * (xb.re * xb.re + xb.im * xb.im);
            } else if constexpr (OUT == kOutTopK) {  // stage the scan band X[kmin..kmax] only
                cpx<T> *xrow = reinterpret_cast<cpx<T> *>(lbase);
                if ((unsigned)(ka - a.kmin) <= (unsigned)(a.kmax - a.kmin)) xrow[ka - a.kmin] = {kS1 * xa.re, kS1 * xa.im};
                if ((unsigned)(kb - a.kmin) <= (unsigned)(a.kmax - a.kmin)) xrow[kb - a.kmin] = {kS1 * xb.re, kS1 * xb.im};
            } else if constexpr (OUT == kOutTopKPhase && kSplit) {  // stage X[0 .. kmax + 1] (split slot)
                cpx<T> *xrow = reinterpret_cast<cpx<T> *>(lbase);
                if ((unsigned)ka <= (unsigned)(a.kmax + 1)) xrow[ka] = {kS1 * xa.re, kS1 * xa.im};
                if ((unsigned)kb <= (unsigned)(a.kmax + 1)) xrow[kb] = {kS1 * xb.re, kS1 * xb.im};
            } else if constexpr (kPhaseSplit) {  // split phase record: Re X to the split slot, Im in registers
                double *srow = reinterpret_cast<double *>(lbase);
                srow[pad16(ka)] = kS1 * xa.re;
                srow[pad16(kb)] = kS1 * xb.re;
                pim[s] = kS1 * xa.im;
                pim[8 + s] = kS1 * xb.im;
            } else if constexpr (kPhase) {  // stage X for the phase / scan (AoS slot)
                cpx<T> *xrow = reinterpret_cast<cpx<T> *>(lbase);
                xrow[pad16(ka)] = {kS1 * xa.re, kS1 * xa.im};
                xrow[pad16(kb)] = {kS1 * xb.re, kS1 * xb.im};
            } else if (active) {  // packed: (Re, Im) of one bin is already one 16-B (8-B) store
                v2 oa, ob;
                oa.x = kS1 * xa.re;
                oa.y = kS1 * xa.im;
                ob.x = kS1 * xb.re;
                ob.y = kS1 * xb.im;
                *reinterpret_cast<v2 *>(a.out + w * N + 2 * ka) = oa;
                *reinterpret_cast<v2 *>(a.out + w * N + 2 * kb) = ob;
            }
        }
        // unwrapped phase / group delay of bins [16t, 16t + 16) (kept in registers
        // through the top-k scan for kOutTopKPhase)
        if constexpr (kPhaseSplit) {
            // Split phase record (round 5): the AoS form stages X as 16-B complex (35 KiB per window: two workgroups
            // per CU) and holds [P | phase | delay] for 16 bins at once (241 VGPRs: two waves per SIMD).  Here the
            // window's 17 KiB split slot takes Re X, each thread reads its 18 consecutive bins (16 + two neighbours),
            // then Im X the same way; the rows are computed and written one after another (P, then the unwrapped
            // phase, then the group delay), so at most one row of 16 values is live: 3 waves per SIMD.  Same
            // arithmetic as phase_chunk (the unwrap decisions from the atan2 values, K an exact integer prefix count,
            // u = phi + 2 pi K by one fma, CalculateGroupDelay's central difference clamped to +-100).
            constexpr double kPi = 3.14159265358979323846, k2Pi = 2.0 * kPi;
            double *srow = reinterpret_cast<double *>(lbase);
            const int k0 = 16 * t;
            double re[18], ph[18];
            __syncthreads();  // Re row complete
#pragma unroll
            for (int j = 0; j < 18; ++j) {
                const int k = k0 - 1 + j;
                re[j] = (k >= 0 && k < M) ? srow[pad16(k)] : 0.0;  // bin M: the zeroed upper half
            }
            __syncthreads();  // Re reads done: the slot takes Im
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                int ka = tb0 + B * s, kb = M - ka;
                if (tb0 == 0) {
                    ka = s < 4 ? B / 2 + B * s : B * (s - 4);
                    kb = s == 4 ? M / 2 : M - ka;
                }
                srow[pad16(ka)] = pim[s];
                srow[pad16(kb)] = pim[8 + s];
            }
            __syncthreads();
            double im[18], pwr[16];
#pragma unroll
            for (int j = 0; j < 18; ++j) {
                const int k = k0 - 1 + j;
                im[j] = (k >= 0 && k < M) ? srow[pad16(k)] : 0.0;
                if (j >= 1 && j <= 16) pwr[j - 1] = re[j] * re[j] + im[j] * im[j];
            }
            // [P | unwrapped phase | group delay] rows through the slot: pairs 16-B aligned (two pad doubles per 32
            // inside the SLOT doubles), written with contiguous 16-B NT stores (1 KiB per wave instruction)
            auto pidx2 = [](int k) { return k + 2 * (k >> 5); };
            auto put = [&](const double(&val)[16], int row) {
                __syncthreads();  // previous reads of the slot are done
#pragma unroll
                for (int j = 0; j < 16; j += 2)
                    *reinterpret_cast<v2 *>(srow + pidx2(16 * t + j)) = v2{val[j], val[j + 1]};
                __syncthreads();
                if (active) {
                    T *dst = a.out + w * (int64_t)(3 * M) + row * M;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int k = 2 * (t + TPW * j);
                        __builtin_nontemporal_store(*reinterpret_cast<const v2 *>(srow + pidx2(k)),
                                                    reinterpret_cast<v2 *>(dst + k));
                    }
                }
            };
            put(pwr, 0);  // the power row first: nothing but (re, im) is held across the 18 atan2
            const unsigned long long *cf = kAtanRed;
            asm volatile("" : "+s"(cf));  // per window: the coefficients' scalar loads stay inside the window loop
#pragma unroll
            for (int j = 0; j < 18; ++j) ph[j] = atan2_sc(im[j], re[j], cf);
            int cj[17];  // correction of bins k0 .. k0 + 16 (UnwrapPhase :1068-1077)
#pragma unroll
            for (int j = 0; j < 17; ++j) {
                const double diff = ph[j + 1] - ph[j];
                cj[j] = (k0 + j == 0) ? 0 : diff > kPi ? -1 : diff < -kPi ? 1 : 0;
            }
            int sum = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) sum += cj[j];
            constexpr int SW = TPW < 64 ? TPW : 64;
            const int lt = t & (SW - 1);
            int incl = sum;
#pragma unroll
            for (int d = 1; d < SW; d <<= 1) {
                const int up = __shfl_up(incl, d, SW);
                if (lt >= d) incl += up;
            }
            int K = incl - sum;  // corrections of every bin < k0
            if constexpr (TPW >= 128) {  // + the totals of the window's earlier waves
                int *sb = reinterpret_cast<int *>(scanbuf + 8);
                __syncthreads();  // the previous window's reads of sb are done
                if (lt == 63) sb[t >> 6] = incl;
                __syncthreads();
                for (int i = 0; i < (t >> 6); ++i) K += sb[i];
            }
            const double um1 = fma((double)K, k2Pi, ph[0]);  // u[k0 - 1]
            double uu[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                K += cj[j];
                uu[j] = fma((double)K, k2Pi, ph[j + 1]);
            }
            const double upc = fma((double)(K + cj[16]), k2Pi, ph[17]);  // u[k0 + 16]
            put(uu, 1);
            double gdd[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {  // :1102-1119
                const double lo = j ? uu[j - 1] : um1, hi = j < 15 ? uu[j + 1] : upc;
                double g = (k0 + j == 0) ? -(uu[1] - uu[0]) : -(hi - lo) / 2.0;
                if (g > 100.0) g = 100.0;
                if (g < -100.0) g = -100.0;
                gdd[j] = g;
            }
            put(gdd, 2);
        }
        double pw[OUT == kOutPhase ? 16 : 1], u[OUT == kOutPhase ? 16 : 1], gd[OUT == kOutPhase ? 16 : 1];
        if constexpr (OUT == kOutPhase && !kPhaseSplit) {
            const cpx<double> *xrow = reinterpret_cast<const cpx<double> *>(lbase);
            __syncthreads();  // X row complete
            phase_chunk<LOG2N, 16, false, true>(xrow, t, scanbuf, pw, u, gd);
            {
                // record [P | unwrapped phase | group delay]: each row staged through this window's
                // LDS slot (2 pad doubles per 16 keep pairs 16-B aligned and the lane-strided writes
                // conflict-free), then written with contiguous 16-B NT stores like the power row
                double *srow = reinterpret_cast<double *>(lbase);
                auto pidx = [](int k) { return k + 2 * (k >> 4); };
                auto put = [&](const double(&val)[16], int row) {
                    __syncthreads();  // previous reads of the slot are done
#pragma unroll
                    for (int j = 0; j < 16; j += 2)
                        *reinterpret_cast<v2 *>(srow + pidx(16 * t + j)) = v2{val[j], val[j + 1]};
                    __syncthreads();
                    if (active) {
                        T *dst = a.out + w * (int64_t)(3 * M) + row * M;
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const int k = 2 * (t + TPW * j);
                            __builtin_nontemporal_store(*reinterpret_cast<const v2 *>(srow + pidx(k)),
                                                        reinterpret_cast<v2 *>(dst + k));
                        }
                    }
                };
                // the power and phase rows staged together (round 6: one barrier pair fewer per window), then the
                // group delay
                {
                    constexpr int RW = M + M / 8;  // doubles per staged row (pidx(M))
                    __syncthreads();  // the X reads of phase_chunk are done
#pragma unroll
                    for (int j = 0; j < 16; j += 2) {
                        *reinterpret_cast<v2 *>(srow + pidx(16 * t + j)) = v2{pw[j], pw[j + 1]};
                        *reinterpret_cast<v2 *>(srow + RW + pidx(16 * t + j)) = v2{u[j], u[j + 1]};
                    }
                    __syncthreads();
                    if (active) {
                        T *dst = a.out + w * (int64_t)(3 * M);
#pragma unroll
                        for (int r = 0; r < 2; ++r)
#pragma unroll
                            for (int j = 0; j < 8; ++j) {
                                const int k = 2 * (t + TPW * j);
                                __builtin_nontemporal_store(*reinterpret_cast<const v2 *>(srow + r * RW + pidx(k)),
                                                            reinterpret_cast<v2 *>(dst + r * M + k));
                            }
                    }
                }
                put(gd, 2);
            }
        }
        if constexpr (OUT == kOutTopK || OUT == kOutTopKPhase) {
            // Top-k bin scan (L/WaveSpecZZ_1.0.3-pla-kalman-fast-gpuopt-nodetrend.mq5:536-554) in the
            // order (power desc, bin asc) that the reference's strict-'>' insertion in ascending bin
            // order produces.  Each lane keeps the powers of its bins kmin + t + TPW i in registers;
            // k rounds of a wave-wide argmax (xor shuffles, no barrier) pick the winners and the
            // owner retires its bin.  With two waves per window (N = 4096) each wave builds its own
            // sorted list and the two lists merge by rank counting behind one barrier.  The X row
            // is left intact: kOutTopKPhase computes the phases after the scan and the owners of
            // the winners' chunks add them to the records.
            const cpx<T> *xrow = reinterpret_cast<const cpx<T> *>(lbase);
            constexpr int SW = TPW < 64 ? TPW : 64;
            constexpr int kNone = 0x7fffffff;
            constexpr int RW = OUT == kOutTopKPhase ? 6 : 4;  // record width
            const int kmin0 = a.kmin;
            auto xi = [&](int k) { return kPhase ? pad16(k) : k - kmin0; };  // kOutTopK stages the band only
            __syncthreads();  // X row complete
            const int span = a.kmax - a.kmin + 1;
            T *recw = a.out + w * (int64_t)(RW * a.topk);
            if constexpr (OUT == kOutTopK && TPW >= 64) {
                // one wave scans the window's whole band (<= 512 bins, 8 per lane): no cross-wave merge.
                // The split-exchange instantiation carries only this path (the host sends wider bands to
                // the AoS one), which keeps it within the 168 VGPRs of 3 waves per SIMD.
                if ((VAR & kVarSplitLds) || span <= 64 * 8) {
                    if (t < 64) {
                        const cpx<T> *xb = xrow;
                        const int nb = (span + 63) / 64;
                        if (nb <= 1) topk_wave64<1, T>(xb, a.kmin, span, a.topk, t, recw, active);
                        else if (nb <= 2) topk_wave64<2, T>(xb, a.kmin, span, a.topk, t, recw, active);
                        else if (nb <= 4) topk_wave64<4, T>(xb, a.kmin, span, a.topk, t, recw, active);
                        else topk_wave64<8, T>(xb, a.kmin, span, a.topk, t, recw, active);
                    }
                    continue;  // next group (its first exchange barrier orders this scan's LDS reads)
                }
            }
            if constexpr (OUT == kOutTopKPhase && TPW >= 64 && (VAR & kVarSplitLds)) {
                // the split-exchange form (the host checks that bins 0 .. kmax + 1 fit the slot and the band holds
                // at most 8 bins per lane): one wave scans the band, then the same wave adds the winners' unwrapped
                // phase and group delay (topk_phase_wave) -- 3 waves per SIMD instead of the AoS form's 2
                if (t < 64) {
                    const cpx<T> *xb = xrow + a.kmin;
                    const int nb = (span + 63) / 64;
                    int bin = -1;
                    if (nb <= 1) topk_wave64<1, T, 6>(xb, a.kmin, span, a.topk, t, recw, active, nullptr, &bin);
                    else if (nb <= 2) topk_wave64<2, T, 6>(xb, a.kmin, span, a.topk, t, recw, active, nullptr, &bin);
                    else if (nb <= 4) topk_wave64<4, T, 6>(xb, a.kmin, span, a.topk, t, recw, active, nullptr, &bin);
                    else topk_wave64<8, T, 6>(xb, a.kmin, span, a.topk, t, recw, active, nullptr, &bin);
                    const int need = a.kmax + 2;
                    const cpx<double> *xd = reinterpret_cast<const cpx<double> *>(xrow);
                    double *rd = reinterpret_cast<double *>(recw);
                    if (need <= 128) topk_phase_wave<2>(xd, M, a.kmax, a.topk, t, bin, rd, active);
                    else if (need <= 256) topk_phase_wave<4>(xd, M, a.kmax, a.topk, t, bin, rd, active);
                    else if (need <= 512) topk_phase_wave<8>(xd, M, a.kmax, a.topk, t, bin, rd, active);
                    else topk_phase_wave<16>(xd, M, a.kmax, a.topk, t, bin, rd, active);
                }
                continue;  // next group (its first exchange barrier orders this wave's LDS reads)
            }
            if constexpr (!(OUT == kOutTopK && TPW >= 64 && (VAR & kVarSplitLds))) {
            auto write_x = [&](T *rec, int b, T pw_) {
                const cpx<T> x = xrow[xi(b)];
                rec[0] = T(b);
                rec[1] = pw_;
                rec[2] = x.re;
                rec[3] = x.im;
            };
            auto write_empty = [&](T *rec) {
                rec[0] = T(-1);
                rec[1] = T(-1);
#pragma unroll
                for (int j = 2; j < RW; ++j) rec[j] = T(0);
            };
            constexpr int KW = M < 64 ? M : 64;  // winners that can exist per window (k <= 64, span <= M)
            constexpr int LST = TPW >= 128 ? NWV * 64 : 0;  // list entries (several waves per window)
            int *win = reinterpret_cast<int *>(scanbuf + 16 + LST) + LST + slot * KW;  // kOutTopKPhase winners
            const int lt = t & (SW - 1);
            T cp = T(-1);  // TPW >= 128: this lane's entry of its wave's sorted list
            int cb = kNone;
            auto power_of = [&](int b) {
                const cpx<T> x = xrow[xi(b)];
                return x.re * x.re + x.im * x.im;
            };
            auto on_win = [&](int r, T wp, int wb, bool own) {
                if constexpr (TPW >= 128) {
                    if (lt == r) {
                        cp = wp;
                        cb = wb;
                    }
                } else {  // one wave segment per window: round r's winner is slot r
                    T *rec = recw + RW * r;
                    if (own && active) write_x(rec, wb, wp);
                    if (wb == kNone && t == 0 && active) write_empty(rec);
                    if constexpr (RW == 6) {
                        if (t == 0 && r < KW) win[r] = wb;
                    }
                }
            };
            // bins per lane: uniform branch to a register array of just that size
            const int nbl = span <= 0 ? 1 : (span + TPW - 1) / TPW;
            if (nbl <= 1) topk_rounds<1, SW, TPW, T>(t, a.kmin, span, a.topk, power_of, on_win);
            else if (nbl <= 2) topk_rounds<2, SW, TPW, T>(t, a.kmin, span, a.topk, power_of, on_win);
            else if (nbl <= 4) topk_rounds<4, SW, TPW, T>(t, a.kmin, span, a.topk, power_of, on_win);
            else if (nbl <= 8) topk_rounds<8, SW, TPW, T>(t, a.kmin, span, a.topk, power_of, on_win);
            else topk_rounds<16, SW, TPW, T>(t, a.kmin, span, a.topk, power_of, on_win);
            if constexpr (TPW >= 128) {
                double *lp = scanbuf + 16;                              // [NWV][64] powers
                int *lb = reinterpret_cast<int *>(scanbuf + 16 + LST);  // [NWV][64] bins
                const int wv = t >> 6;
                if (lt < a.topk) {
                    lp[64 * wv + lt] = (double)cp;
                    lb[64 * wv + lt] = cb;
                }
                __syncthreads();
                int rank = lt, nother = 0;  // rank among all lists (bins are distinct across lists)
                for (int v2 = 0; v2 < NWV; ++v2) {
                    if (v2 == wv) continue;
                    for (int j = 0; j < a.topk; ++j) {
                        const T op = (T)lp[64 * v2 + j];
                        const int ob = lb[64 * v2 + j];
                        nother += ob != kNone;
                        rank += ob != kNone && (op > cp || (op == cp && ob < cb));
                    }
                }
                const int nvalid = (int)__popcll(__ballot(lt < a.topk && cb != kNone)) + nother;
                const bool mine = lt < a.topk && cb != kNone && rank < a.topk;
                if (mine && active) write_x(recw + RW * rank, cb, cp);
                if (wv == 0 && lt >= nvalid && lt < a.topk && active) write_empty(recw + RW * lt);
                if constexpr (RW == 6) {
                    if (mine) win[rank] = cb;
                    if (wv == 0 && lt >= nvalid && lt < a.topk) win[lt] = kNone;
                }
            }
            if constexpr (RW == 6) {
                // phases of the (unmodified) X row, then the owner of each winner's chunk adds
                // [unwrapped phase, group delay] to that slot
                __syncthreads();  // winners list complete
                // only bins 0 .. kmax + 1 feed the winners' unwrapped phase and group delay: CH bins per
                // thread with CH * TPW >= kmax + 2 (wave-uniform choice) instead of the whole row
                auto add_phase = [&](auto chv) {
                    constexpr int CH = decltype(chv)::value;
                    double pwc[CH], uc[CH], gdc[CH];
                    phase_chunk<LOG2N, CH, true>(reinterpret_cast<const cpx<double> *>(lbase), t, scanbuf, pwc, uc, gdc);
                    const int nk = a.topk < KW ? a.topk : KW;
                    for (int s2 = 0; s2 < nk; ++s2) {
                        const int b = win[s2];
                        if (b != kNone && b / CH == t && active) {
                            double ub = 0.0, gb = 0.0;
#pragma unroll
                            for (int j = 0; j < CH; ++j)
                                if (b % CH == j) {
                                    ub = uc[j];
                                    gb = gdc[j];
                                }
                            T *rec = recw + RW * s2;
                            rec[4] = ub;
                            rec[5] = gb;
                        }
                    }
                };
                const int need = a.kmax + 2;  // bins 0 .. kmax + 1
                if (need <= 2 * TPW) add_phase(std::integral_constant<int, 2>{});
                else if (need <= 4 * TPW) add_phase(std::integral_constant<int, 4>{});
                else if (need <= 8 * TPW) add_phase(std::integral_constant<int, 8>{});
                else add_phase(std::integral_constant<int, 16>{});
            }
            }  // !(split one-wave top-k)
        }
        if constexpr (OUT == kOutPower && !kDirect) {
            // write the row back with contiguous 16-B stores (1 KiB per wave instruction)
            constexpr int VE = 16 / (int)sizeof(T);
            typedef T vst __attribute__((ext_vector_type(16 / sizeof(T))));
            __syncthreads();
            if (active) {
#pragma unroll
                for (int j = 0; j < 16 / VE; ++j) {
                    const int k = VE * (t + TPW * j);
                    const vst val = *reinterpret_cast<const vst *>(prow + k);
                    if constexpr (VAR & kVarWtStore) {  // descriptor at the group's first row: uniform, small offsets
                        const __amdgpu_buffer_rsrc_t orc =
                            __builtin_amdgcn_make_buffer_rsrc(a.out + g * WPB * (int64_t)M, (short)0, 0x7fffffff, 0x00020000);
                        typedef unsigned u4 __attribute__((ext_vector_type(4)));
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, val), orc,
                                                               (int)((slot * M + k) * (int)sizeof(T)), 0, 16);
                    } else if constexpr (VAR & kVarNtStore) {
                        __builtin_nontemporal_store(val, reinterpret_cast<vst *>(a.out + w * M + k));
                    } else {
                        *reinterpret_cast<vst *>(a.out + w * M + k) = val;
                    }
                }
            }
        }
    }
}

// Host-side argument setup shared by the library and the tools.
template <typename T> SpecArgs<T> make_args(const SpectrumLaunch &L, int wpb);

}  // namespace core
}  // namespace wsp
