// transform_kernels.hip -- the other transforms of the spectrum machinery:
//
//  * inverse real FFT of packed spectra (gpu_fft_real_inverse, declared at
//    L/WaveSpecZZ_1.0.4-core.mq5:65 and called at :426 on what
//    gpu_fft_real_forward produced at :344, after the spectral stages);
//  * phase / unwrap / group delay of one packed spectrum
//    (gpu_spectral_phase_unwrap, L/WaveSpecZZ_1.0.4-core.mq5:72,416), with the
//    arithmetic of CalculateFFTPhase / UnwrapPhase / CalculateGroupDelay
//    (L/WaveSpecZZ_1.0.4-new.mq5:1040-1120).
//
// The inverse reuses the forward kernel's Stockham passes (spectrum_core.h):
// x = IDFT_N(X) is computed as the M = N/2 point complex transform
// z = conj(DFT_M(conj Z)) / M of Z_k = E_k + i O_k, where
//   E_k = (X_k + conj X_(M-k)) / 2,  O_k = W_N^-k (X_k - conj X_(M-k)) / 2,
// and x[2n] = Re z_n, x[2n+1] = Im z_n (the forward R2C step run backwards).
// The packed layout carries X_k for k < N/2 only: X_(N/2) is taken as 0 and
// in[1] (Im X_0 of a real signal, 0) is ignored -- inverse(forward(x)) = x
// for every x without a Nyquist component.
#include "spectrum_core.h"

namespace wsp {
namespace core {

template <int LOG2N>
__global__ __launch_bounds__(Geo<LOG2N>::BLOCK, 2) void inverse_kernel(const double *__restrict__ in, double *__restrict__ out,
                                                           const cpx<double> *__restrict__ tw, int64_t n_windows,
                                                           int64_t n_groups) {
    using G = Geo<LOG2N>;
    using T = double;
    using v2 = V2<double>::t;
    constexpr int N = G::N, M = G::M, TPW = G::TPW, WPB = G::WPB, SLOT = G::SLOT, B = G::B;
    constexpr int R0 = G::R0, BPT0 = G::BPT0;
    __shared__ __attribute__((aligned(16))) char smem[WPB * SLOT * sizeof(cpx<T>)];
    const int tid = threadIdx.x;
    const int slot = tid / TPW;
    const int t = tid % TPW;
    char *lbase = smem + slot * SLOT * (int)sizeof(cpx<T>);
    cpx<T> *zrow = reinterpret_cast<cpx<T> *>(lbase);

    for (int64_t g = blockIdx.x; g < n_groups; g += gridDim.x) {
        const int64_t w = g * WPB + slot;
        const bool active = w < n_windows;
        const T *xin = in + (active ? w : 0) * N;

        // ---- C2R pre-step: thread t forms Z_k and Z_(M-k) for k = t + TPW j, j < 8 (k < M/2),
        // stored conjugated in natural order; thread 0 also forms Z_(M/2) = conj X_(M/2).
        __syncthreads();  // the previous group's final-pass reads of this slot are done
        const int pa0 = pad16(t), pb0 = pad16(M - t);
        // unroll 2: fully unrolled, the scheduler hoists all 16 sample loads and spills (up to
        // 324 B/lane at N = 16384); pairs of iterations keep it at zero scratch for every N
#pragma unroll 2
        for (int j = 0; j < 8; ++j) {
            const int k = t + TPW * j;
            // pad16(t + TPW j), pad16(M - t - TPW j) with the j part folded into the ds offset
            const int ia = pad16_at<TPW>(pa0, t, j);
            const int ib = TPW % 16 == 0 ? pb0 - (TPW / 16) * 17 * j : pad16(M - k);
            const v2 pa = __builtin_nontemporal_load(reinterpret_cast<const v2 *>(xin + 2 * k));
            cpx<T> xa = {pa.x, pa.y}, xb = {T(0), T(0)};
            if (k == 0) {
                xa.im = T(0);  // real DC; X_M = 0
            } else {
                const v2 pb = __builtin_nontemporal_load(reinterpret_cast<const v2 *>(xin + 2 * (M - k)));
                xb = {pb.x, pb.y};
            }
            const cpx<T> e = {T(0.5) * (xa.re + xb.re), T(0.5) * (xa.im - xb.im)};
            const cpx<T> d = {T(0.5) * (xa.re - xb.re), T(0.5) * (xa.im + xb.im)};
            const cpx<T> o = cmul(cconj(tw[k]), d);
            // conj Z_k = conj(E + iO); conj Z_(M-k) = conj(conj E + i conj O) = E - i O
            zrow[ia] = {e.re - o.im, -(e.im + o.re)};
            if (k != 0) zrow[ib] = {e.re + o.im, e.im - o.re};
        }
        if (t == 0) {
            const v2 ph = __builtin_nontemporal_load(reinterpret_cast<const v2 *>(xin + M));  // X_(M/2)
            zrow[pad16(M / 2)] = {ph.x, ph.y};                                                  // conj(conj X)
        }
        __syncthreads();

        // ---- forward Stockham transform of conj Z (pass-0 read layout of spectrum_kernel)
        cpx<T> v[16];
#pragma unroll
        for (int q = 0; q < BPT0; ++q)
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                const int b = t + TPW * q;
                v[q * R0 + r] = zrow[pad16_at<M / R0>(pad16(b), b, r)];
            }
#pragma unroll
        for (int q = 0; q < BPT0; ++q) dft<T, R0>(&v[q * R0]);
        exchange<false, T, LOG2N, 0>(lbase, v, t);
        mid_passes<false, false, T, LOG2N, 1>(lbase, v, tw, t);
        const int bq0 = t, bq1 = t == 0 ? TPW : 2 * TPW - t;
        cpx<T> u0[8], u1[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            u0[r] = v[r];
            u1[r] = v[8 + r];
        }
        if constexpr (G::NPASS > 1) {
            twiddle<false, T, 8>(u0, tw, 2 * bq0);
            twiddle<false, T, 8>(u1, tw, 2 * bq1);
        }
        dft<T, 8>(u0);
        dft<T, 8>(u1);

        // ---- z_n = conj(Y_n) / M -> x[2n] = Re z_n, x[2n+1] = Im z_n; u0[r] = Y[t + B r],
        // u1[r] = Y[bq1 + B r]: consecutive lanes store consecutive 16-B pairs
        if (active) {
            constexpr T kScale = T(1) / T(M);
            T *xo = out + w * N;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                __builtin_nontemporal_store(v2{u0[r].re * kScale, -u0[r].im * kScale},
                                            reinterpret_cast<v2 *>(xo + 2 * (bq0 + B * r)));
                __builtin_nontemporal_store(v2{u1[r].re * kScale, -u1[r].im * kScale},
                                            reinterpret_cast<v2 *>(xo + 2 * (bq1 + B * r)));
            }
        }
    }
}

// The same inverse with the C2R pre-step in registers (round 4): thread t forms the elements of its pass-0
// layout, conj Z_k for k = (t + TPW q) + (M/R0) r, straight from X_k and X_(M-k) (two 16-B loads; each X is read
// by two threads, the second time from L2), instead of staging all of conj Z through LDS and reading it back
// -- one LDS round trip and one barrier fewer -- and, with SPLIT, the real/imaginary split exchanges of the
// forward kernel (half the LDS, 3 waves per SIMD).  Z_(M/2) = conj X_(M/2) and the DC term as above.
// PAIRED (round 5, the default): the 16 elements are loaded in the order r = 0, 15, 1, 14, ... -- element k's mirror
// M - k is element 15 - r of the partner thread TPW - t (the other wave of the window), so the two reads of every
// X_k (once as k, once as the partner's mirror) fall one load step apart instead of up to 15, and the second one
// hits the line the first brought into L2 (in natural order 0.3 of the second reads went to HBM: PMC 2.79 GB of
// reads per step against 2.15 GB algorithmic, profiles/r04/inverse_*); variant 3 keeps the natural order.
// NTS: non-temporal sample stores (the default); variant 4 = plain stores (a pure write stream ran 5.75 TB/s with
// plain 16-B stores against 5.5 with non-temporal ones, profiles/r02/slide/write_probe.log).
template <int LOG2N, int SPLIT, bool PAIRED = true, bool NTS = true>
__global__ __launch_bounds__(Geo<LOG2N>::BLOCK, SPLIT ? 3 : 2) void inverse_direct_kernel(
    const double *__restrict__ in, double *__restrict__ out, const cpx<double> *__restrict__ tw, int64_t n_windows,
    int64_t n_groups) {
    using G = Geo<LOG2N>;
    using T = double;
    using v2 = V2<double>::t;
    constexpr int N = G::N, M = G::M, TPW = G::TPW, WPB = G::WPB, SLOT = G::SLOT, B = G::B;
    constexpr int R0 = G::R0, BPT0 = G::BPT0;
    constexpr int ES = SPLIT ? (int)sizeof(T) : (int)sizeof(cpx<T>);
    __shared__ __attribute__((aligned(16))) char smem[WPB * SLOT * ES];
    const int tid = threadIdx.x;
    const int slot = tid / TPW;
    const int t0 = tid % TPW;
    char *lbase = smem + slot * SLOT * ES;
    for (int64_t g = blockIdx.x; g < n_groups; g += gridDim.x) {
        // per window: the thread's twiddles and addresses are not hoisted out of the window loop (and spilled)
        int t = t0;
        asm volatile("" : "+v"(t));
        const int64_t w = g * WPB + slot;
        const bool active = w < n_windows;
        const T *xin = in + (active ? w : 0) * N;
        cpx<T> v[16];
#pragma unroll
        for (int q = 0; q < BPT0; ++q)
#pragma unroll
            for (int i = 0; i < R0; ++i) {
                const int r = PAIRED ? ((i & 1) ? R0 - 1 - (i >> 1) : (i >> 1)) : i;
                const int k = (t + TPW * q) + (M / R0) * r;
                const v2 pa = *reinterpret_cast<const v2 *>(xin + 2 * k);
                const v2 pb = *reinterpret_cast<const v2 *>(xin + 2 * ((M - k) & (M - 1)));
                // k = 0 only for t = 0 at (q, r) = (0, 0): real DC, X_M = 0 (branch-free selects)
                const bool dc = (q == 0 && r == 0) && k == 0;
                const cpx<T> xa = {pa.x, dc ? T(0) : pa.y};
                const cpx<T> xb = {dc ? T(0) : pb.x, dc ? T(0) : pb.y};
                const cpx<T> e = {T(0.5) * (xa.re + xb.re), T(0.5) * (xa.im - xb.im)};
                const cpx<T> d = {T(0.5) * (xa.re - xb.re), T(0.5) * (xa.im + xb.im)};
                const cpx<T> o = cmul(cconj(tw[k]), d);
                const cpx<T> z = {e.re - o.im, -(e.im + o.re)};  // conj Z_k
                v[q * R0 + r] = k == M / 2 ? cpx<T>{pa.x, pa.y} : z;  // conj(conj X_(M/2))
                // at most 4 elements' loads in flight: hoisting all 32 sample and 16 twiddle loads spills
                if ((i & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
        for (int q = 0; q < BPT0; ++q) dft<T, R0>(&v[q * R0]);
        exchange<SPLIT, T, LOG2N, 0>(lbase, v, t);  // also orders the previous group's reads
        mid_passes<SPLIT, false, T, LOG2N, 1>(lbase, v, tw, t);
        const int bq0 = t, bq1 = t == 0 ? TPW : 2 * TPW - t;
        cpx<T> u0[8], u1[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            u0[r] = v[r];
            u1[r] = v[8 + r];
        }
        if constexpr (G::NPASS > 1) {
            twiddle<false, T, 8>(u0, tw, 2 * bq0);
            twiddle<false, T, 8>(u1, tw, 2 * bq1);
        }
        dft<T, 8>(u0);
        dft<T, 8>(u1);
        if (active) {
            constexpr T kScale = T(1) / T(M);
            T *xo = out + w * N;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const v2 a = {u0[r].re * kScale, -u0[r].im * kScale}, b = {u1[r].re * kScale, -u1[r].im * kScale};
                v2 *pa = reinterpret_cast<v2 *>(xo + 2 * (bq0 + B * r)), *pb = reinterpret_cast<v2 *>(xo + 2 * (bq1 + B * r));
                if constexpr (NTS) {
                    __builtin_nontemporal_store(a, pa);
                    __builtin_nontemporal_store(b, pb);
                } else {
                    *pa = a;
                    *pb = b;
                }
            }
        }
    }
}

// One packed spectrum of nb bins; bins >= nb are the zeroed upper half of the
// reference's arrays (phase 0).  256 threads, contiguous chunks, two passes:
// correction counts -> block scan -> outputs.  Same unwrap formulation as
// phase_chunk (spectrum_core.h).
constexpr int kRowThreads = 256;
__global__ __launch_bounds__(kRowThreads) void phase_row_kernel(const double *__restrict__ spec, int nb, int method,
                                                                 double *__restrict__ out) {
    constexpr double kPi = 3.14159265358979323846, k2Pi = 2.0 * kPi;
    __shared__ int part[kRowThreads];
    const int t = threadIdx.x;
    const int chunk = (nb + kRowThreads - 1) / kRowThreads;
    const int k0 = min(t * chunk, nb), k1 = min(k0 + chunk, nb);
    auto phase = [&](int k) { return k < nb ? atan2(spec[2 * k + 1], spec[2 * k]) : 0.0; };
    auto corr = [&](double cur, double prev) { const double d = cur - prev; return d > kPi ? -1 : d < -kPi ? 1 : 0; };
    int sum = 0;
    double prev = k0 > 0 ? phase(k0 - 1) : 0.0;
    for (int k = k0; k < k1; ++k) {
        const double p = phase(k);
        if (k > 0) sum += corr(p, prev);
        prev = p;
    }
    part[t] = sum;
    __syncthreads();
    for (int d = 1; d < kRowThreads; d <<= 1) {  // Hillis-Steele inclusive scan
        const int add = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += add;
        __syncthreads();
    }
    int K = part[t] - sum;  // corrections of every bin < k0
    if (k0 >= k1) return;
    const int n = 2 * nb;   // length of the reference's arrays
    double pm = k0 > 0 ? phase(k0 - 1) : 0.0;
    const double um1 = fma((double)K, k2Pi, pm);
    double pc = phase(k0);
    if (k0 > 0) K += corr(pc, pm);
    double uc = fma((double)K, k2Pi, pc), ul = k0 > 0 ? um1 : 0.0;
    for (int k = k0; k < k1; ++k) {
        const double pn = phase(k + 1);  // k + 1 <= nb: bin nb is phase 0
        const int Kn = K + corr(pn, pc);
        const double un = fma((double)Kn, k2Pi, pn);
        double val;
        if (method == 1) {
            val = pc;
        } else if (method == 0) {
            val = uc;
        } else {  // CalculateGroupDelay :1092-1119
            double g;
            if (n < 3) g = 0.0;
            else if (k == 0) g = -(un - uc);
            else g = -(un - ul) / 2.0;
            val = g > 100.0 ? 100.0 : g < -100.0 ? -100.0 : g;
        }
        out[k] = val;
        ul = uc;
        uc = un;
        pc = pn;
        K = Kn;
    }
}

}  // namespace core

hipError_t launch_inverse(const InverseLaunch &L, hipStream_t stream) {
    using namespace core;
    if (L.n_windows <= 0) return hipSuccess;
    const auto *tw = static_cast<const cpx<double> *>(L.twiddle);
    // the C2R pre-step in registers with the split exchange at N = 2048 .. 8192 (inverse_direct_kernel); variant 1
    // = the LDS pre-step kernel (round 1-3 form), variant 2 = the register pre-step with the AoS exchange, variant 3 =
    // the element loads in natural order (round 4; the default pairs each element's two reads in time), variant 4 = plain
    // sample stores
#define INV_CASE(LG)                                                                                          \
    case LG: {                                                                                                \
        const int64_t groups = (L.n_windows + Geo<LG>::WPB - 1) / Geo<LG>::WPB;                               \
        int64_t grid = L.grid > 0 ? L.grid : 32768;                                                           \
        if (grid > groups) grid = groups;                                                                     \
        if (L.variant == 1 || LG < 11 || LG > 13)                                                             \
            hipLaunchKernelGGL(inverse_kernel<LG>, dim3((unsigned)grid), dim3(Geo<LG>::BLOCK), 0, stream, L.in, L.out, tw, \
                               L.n_windows, groups);                                                          \
        else if (L.variant == 2)                                                                              \
            hipLaunchKernelGGL((inverse_direct_kernel<LG, 0>), dim3((unsigned)grid), dim3(Geo<LG>::BLOCK), 0, stream, L.in, \
                               L.out, tw, L.n_windows, groups);                                               \
        else if (L.variant == 3)                                                                              \
            hipLaunchKernelGGL((inverse_direct_kernel<LG, 2, false>), dim3((unsigned)grid), dim3(Geo<LG>::BLOCK), 0, stream, \
                               L.in, L.out, tw, L.n_windows, groups);                                         \
        else if (L.variant == 4)                                                                              \
            hipLaunchKernelGGL((inverse_direct_kernel<LG, 2, true, false>), dim3((unsigned)grid), dim3(Geo<LG>::BLOCK), 0, \
                               stream, L.in, L.out, tw, L.n_windows, groups);                                 \
        else                                                                                                  \
            hipLaunchKernelGGL((inverse_direct_kernel<LG, 2>), dim3((unsigned)grid), dim3(Geo<LG>::BLOCK), 0, stream, L.in, \
                               L.out, tw, L.n_windows, groups);                                               \
        return hipGetLastError();                                                                             \
    }
    switch (L.log2n) {
        INV_CASE(5)
        INV_CASE(6)
        INV_CASE(7)
        INV_CASE(8)
        INV_CASE(9)
        INV_CASE(10)
        INV_CASE(11)
        INV_CASE(12)
        INV_CASE(13)
        INV_CASE(14)
    default: return hipErrorInvalidValue;
    }
#undef INV_CASE
}

hipError_t launch_phase_row(const double *spec, int n_bins, int method, double *out, hipStream_t stream) {
    if (n_bins <= 0) return hipSuccess;
    hipLaunchKernelGGL(core::phase_row_kernel, dim3(1), dim3(core::kRowThreads), 0, stream, spec, n_bins, method, out);
    return hipGetLastError();
}

}  // namespace wsp
