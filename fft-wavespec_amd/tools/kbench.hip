// kbench.hip -- ablation micro-benchmark for the spectrum kernel (not part
// of the library).  One process, interleaved rounds (cdna_hip_programming.md
// sec. 5.4 rule 24): variants of the same kernel, a 2:1 read/write copy
// kernel as the practical HBM ceiling for this traffic shape, grid sweeps.
//
//   kbench [log2n=12] [windows=65536] [reps=20] [rounds=3]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../csrc/spectrum_dispatch.h"

using namespace wsp;
using namespace wsp::core;

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

__global__ void fill_walk(double *x, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 32;
        x[i] = 1.1 + 1e-3 * ((double)(h >> 11) * (1.0 / 9007199254740992.0) - 0.5) + 0.002 * sin(0.1256 * (double)i);
    }
}

// 1:1 float4 copy (calibration against MI355X_MICROARCH.md: 6.29 TB/s)
__global__ __launch_bounds__(256) void copy11(const double2 *__restrict__ in, double2 *__restrict__ out, int64_t n) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
        out[j] = in[j];
}

// 1:1 copy, 4 float4 in flight per thread
__global__ __launch_bounds__(256) void copy11x4(const double2 *__restrict__ in, double2 *__restrict__ out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j + 3 * stride < n; j += 4 * stride) {
        const double2 a = in[j], b = in[j + stride], c = in[j + 2 * stride], d = in[j + 3 * stride];
        out[j] = a;
        out[j + stride] = b;
        out[j + 2 * stride] = c;
        out[j + 3 * stride] = d;
    }
}

// 1:1 copy, 4 x 16 B in flight per thread, non-temporal loads and stores (the inverse's store form)
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy11nt(const double2 *__restrict__ in, double2 *__restrict__ out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += 4 * stride) {
        d2v v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t k = j + u * stride;
            if (k < n) v[u] = NTL ? __builtin_nontemporal_load(reinterpret_cast<const d2v *>(in + k))
                                  : *reinterpret_cast<const d2v *>(in + k);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t k = j + u * stride;
            if (k < n) {
                if (NTS) __builtin_nontemporal_store(v[u], reinterpret_cast<d2v *>(out + k));
                else *reinterpret_cast<d2v *>(out + k) = v[u];
            }
        }
    }
}

// kbench copy [reps=20] [rounds=3]: the inverse's traffic as a pure 1:1 stream -- 65536 x 4096 fp64 read (2.147 GB)
// and the same written, 16-B accesses, grid sweep; whole-GPU grids are multiples of 256 CUs.
int copy_main(int reps, int rounds) {
    const int64_t n2 = (int64_t)65536 * 4096 / 2;  // double2 elements
    double2 *in, *out;
    CK(hipMalloc(&in, n2 * 16));
    CK(hipMalloc(&out, n2 * 16));
    hipLaunchKernelGGL(fill_walk, dim3(4096), dim3(256), 0, 0, (double *)in, n2 * 2);
    CK(hipMemset(out, 0, n2 * 16));
    CK(hipDeviceSynchronize());
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)n2 * 32;
    printf("# 1:1 copy of %.3f GB read + %.3f GB written (the inverse plan's 65536 x 4096 fp64 in and out)\n", bytes / 2e9,
           bytes / 2e9);
    const char *nm[] = {"copy11", "copy11x4", "copy11-ntl", "copy11-nts", "copy11-nt2"};
    for (int round = 0; round < rounds; ++round)
        for (int kind = 0; kind < 5; ++kind)
            for (int g : {1024, 2048, 4096, 8192, 16384, 32768}) {
                auto go = [&] {
                    if (kind == 0) hipLaunchKernelGGL(copy11, dim3(g), dim3(256), 0, s, in, out, n2);
                    else if (kind == 1) hipLaunchKernelGGL((copy11nt<false, false>), dim3(g), dim3(256), 0, s, in, out, n2);
                    else if (kind == 2) hipLaunchKernelGGL((copy11nt<true, false>), dim3(g), dim3(256), 0, s, in, out, n2);
                    else if (kind == 3) hipLaunchKernelGGL((copy11nt<false, true>), dim3(g), dim3(256), 0, s, in, out, n2);
                    else hipLaunchKernelGGL((copy11nt<true, true>), dim3(g), dim3(256), 0, s, in, out, n2);
                };
                go();
                CK(hipEventRecord(e0, s));
                for (int i = 0; i < reps; ++i) go();
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double us = ms * 1000.0 / reps;
                printf("round %d %-11s grid=%6d  %8.1f us  %7.1f GB/s  %.3f of 8 TB/s\n", round, nm[kind], g, us,
                       bytes / us / 1e3, bytes / us / 1e3 / 8000.0);
                fflush(stdout);
            }
    return 0;
}

// 2:1 with 4 independent loads in flight per thread, optional nt stores
template <bool NT>
__global__ __launch_bounds__(256) void copy21u(const double2 *__restrict__ in, double2 *__restrict__ out, int64_t n_out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n_out; j += 2 * stride) {
        const bool two = j + stride < n_out;
        const double2 a = in[2 * j], b = in[2 * j + 1];
        double2 c = a, d = b;
        if (two) { c = in[2 * (j + stride)]; d = in[2 * (j + stride) + 1]; }
        const double2 o0 = make_double2(a.x + b.x, a.y + b.y), o1 = make_double2(c.x + d.x, c.y + d.y);
        if (NT) {
            __builtin_nontemporal_store(d2v{o0.x, o0.y}, reinterpret_cast<d2v *>(out + j));
            if (two) __builtin_nontemporal_store(d2v{o1.x, o1.y}, reinterpret_cast<d2v *>(out + j + stride));
        }
        else { out[j] = o0; if (two) out[j + stride] = o1; }
    }
}

// 2:1 read:write streaming kernel (the spectrum's traffic shape, no compute)
__global__ __launch_bounds__(256) void copy21(const double2 *__restrict__ in, double2 *__restrict__ out, int64_t n_out) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n_out; j += (int64_t)gridDim.x * blockDim.x) {
        const double2 a = in[2 * j], b = in[2 * j + 1];
        out[j] = make_double2(a.x + b.x, a.y + b.y);
    }
}

template <int VAR>
float time_variant(const SpectrumLaunch &L, hipStream_t s, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 2; ++i) CK((launch_one<double, 12, kDetrendNone, kOutPower, kWinCos, VAR>(L, s)));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) CK((launch_one<double, 12, kDetrendNone, kOutPower, kWinCos, VAR>(L, s)));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms * 1000.f / reps;
}

template <int OUT, int VAR>
float time_out(const SpectrumLaunch &L, hipStream_t s, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 2; ++i) CK((launch_one<double, 12, kDetrendNone, OUT, kWinCos, VAR>(L, s)));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) CK((launch_one<double, 12, kDetrendNone, OUT, kWinCos, VAR>(L, s)));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.f / reps;
}

// Output-mode ablation at the north-star shape: where the top-k / phase time goes.
int out_main(int reps) {
    const int64_t W = 65536;
    const int n = 4096;
    double *x, *out, *tw;
    CK(hipMalloc(&x, W * n * 8));
    CK(hipMalloc(&out, W * n * 3 / 2 * 8));
    CK(hipMalloc(&tw, n * 16));
    std::vector<double> h(2 * n);
    for (int k = 0; k < n; ++k) {
        long double a = -2.0L * 3.14159265358979323846264338327950288L * k / n;
        h[2 * k] = (double)cosl(a);
        h[2 * k + 1] = (double)sinl(a);
    }
    CK(hipMemcpy(tw, h.data(), n * 16, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(fill_walk, dim3(4096), dim3(256), 0, 0, x, W * n);
    CK(hipDeviceSynchronize());
    hipStream_t s;
    CK(hipStreamCreate(&s));
    SpectrumLaunch L{};
    L.series = x; L.out = out; L.twiddle = tw; L.window = 1; L.hop = n; L.n_windows = W; L.log2n = 12;
    L.kmin = 21; L.kmax = 227;  // periods [18, 200]
    constexpr int AOS = kVarNoPrefetch | kVarNtStore;
    for (int round = 0; round < 2; ++round) {
        L.topk = 8;
        const float pa = time_out<kOutPower, AOS>(L, s, reps);
        const float ps = time_out<kOutPower, AOS | kVarSplitLds>(L, s, reps);
        const float pk = time_out<kOutPacked, AOS>(L, s, reps);
        L.topk = 0;
        const float t0 = time_out<kOutTopK, AOS>(L, s, reps);
        L.topk = 1;
        const float t1 = time_out<kOutTopK, AOS>(L, s, reps);
        L.topk = 8;
        const float t8 = time_out<kOutTopK, AOS>(L, s, reps);
        L.kmax = 22;
        const float t8n = time_out<kOutTopK, AOS>(L, s, reps);
        L.kmax = 227;
        const float ph = time_out<kOutPhase, AOS>(L, s, reps);
        const float tp = time_out<kOutTopKPhase, AOS>(L, s, reps);
        // library defaults: power and top-k (band-staged, one-wave scan) on the split exchange
        const float pd = time_out<kOutPower, kDefaultVar>(L, s, reps);
        const float td = time_out<kOutTopK, kDefaultVar>(L, s, reps);
        L.topk = 0;
        const float td0 = time_out<kOutTopK, kDefaultVar>(L, s, reps);
        L.topk = 8;
        const float tc = time_out<kOutTopK, kCommonVar>(L, s, reps);
        printf("round %d  power-aos %.1f  power-split %.1f  packed %.1f | topk k=0 %.1f  k=1 %.1f  k=8 %.1f  "
               "k=8/2 bins %.1f | phase %.1f  topk-phase %.1f us | library: power %.1f  topk k=8 %.1f (k=0 %.1f, "
               "AoS slot %.1f)\n", round, pa, ps, pk, t0, t1, t8, t8n, ph, tp, pd, td, td0, tc);
        fflush(stdout);
    }
    return 0;
}

static const double *g_win = nullptr;  // window table of the hop1 mode (kVarWinTab variants)

// launch_one with the window table patched into the arguments
template <int LOG2N, int VAR> hipError_t launch_h1(const SpectrumLaunch &L, hipStream_t s) {
    if constexpr (!(VAR & kVarWinTab)) {
        return launch_one<double, LOG2N, kDetrendNone, kOutPower, kWinCos, VAR>(L, s);
    } else {
        using G = Blk<LOG2N, VAR>;
        SpecArgs<double> a = make_args<double>(L, G::WPB);
        a.win = g_win;
        int64_t grid = L.grid > 0 ? L.grid : kDefaultGrid;
        if (grid > a.n_groups) grid = a.n_groups;
        hipLaunchKernelGGL((spectrum_kernel<double, LOG2N, kDetrendNone, kOutPower, kWinCos, VAR>), dim3((unsigned)grid),
                           dim3(G::BLOCK), 0, s, a);
        return hipGetLastError();
    }
}

template <int LOG2N, int VAR>
float time_h1(const SpectrumLaunch &L, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK((launch_h1<LOG2N, VAR>(L, 0)));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) CK((launch_h1<LOG2N, VAR>(L, 0)));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms * 1000.f / reps;
}

// per-window max |P - P_ref| / max P_ref of one launch of a variant against `ref`
template <int LOG2N, int VAR>
double check_h1(const SpectrumLaunch &L, const std::vector<double> &ref) {
    std::vector<double> got(ref.size());
    CK(hipMemset(L.out, 0, got.size() * 8));
    CK((launch_h1<LOG2N, VAR>(L, 0)));
    CK(hipMemcpy(got.data(), L.out, got.size() * 8, hipMemcpyDeviceToHost));
    const size_t m = size_t(1) << (LOG2N - 1);
    double worst = 0;
    for (size_t w = 0; w * m < ref.size(); ++w) {
        double mx = 0, d = 0;
        for (size_t k = 0; k < m; ++k) {
            mx = std::max(mx, std::fabs(ref[w * m + k]));
            d = std::max(d, std::fabs(got[w * m + k] - ref[w * m + k]));
        }
        worst = std::max(worst, mx > 0 ? d / mx : d);
    }
    return worst;
}

template <int LOG2N> struct H1Var {
    const char *name;
    float (*time)(const SpectrumLaunch &, int);
    double (*check)(const SpectrumLaunch &, const std::vector<double> &);
};
#define H1V(NAME, V) H1Var<LOG2N>{NAME, &time_h1<LOG2N, (V)>, &check_h1<LOG2N, (V)>}

// hop = 1 shapes (C4: 1M windows x 2048; the C5 lengths): VALU/LDS-bound, so the
// variants trade instructions, barriers and LDS round trips
template <int LOG2N>
int hop1_main(int64_t W, int reps) {
    const int n = 1 << LOG2N;
    double *x, *out, *tw;
    CK(hipMalloc(&x, (W + n) * 8));
    CK(hipMalloc(&out, W * (n / 2) * 8));
    CK(hipMalloc(&tw, n * 16));
    std::vector<double> h(2 * n);
    for (int k = 0; k < n; ++k) {
        long double ang = -2.0L * 3.14159265358979323846264338327950288L * k / n;
        h[2 * k] = (double)cosl(ang);
        h[2 * k + 1] = (double)sinl(ang);
    }
    CK(hipMemcpy(tw, h.data(), n * 16, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(fill_walk, dim3(1024), dim3(256), 0, 0, x, W + n);
    CK(hipDeviceSynchronize());
    std::vector<double> hw(n);  // Hann/2 (the R2C factor folded in, as make_args does for the coefficients)
    for (int i = 0; i < n; ++i)
        hw[i] = (double)(0.25L - 0.25L * cosl(6.283185307179586476925286766559005768L * i / (long double)(n - 1)));
    double *win;
    CK(hipMalloc(&win, n * 8));
    CK(hipMemcpy(win, hw.data(), n * 8, hipMemcpyHostToDevice));
    g_win = win;
    SpectrumLaunch L{};
    L.series = x; L.out = out; L.twiddle = tw; L.window = 1; L.hop = 1; L.n_windows = W; L.log2n = LOG2N;
    const double bytes = (W + n) * 8.0 + W * (n / 2) * 8.0;
    printf("# hop=1 W=%lld N=%d algorithmic bytes=%.3f GB, roofline %.1f us\n", (long long)W, n, bytes / 1e9,
           bytes / 8e6);
    constexpr int S = kVarSplitLds | kVarNoPrefetch | kVarNtStore, A = kVarNoPrefetch | kVarNtStore;
    const H1Var<LOG2N> vars[] = {
        H1V("split", S),
        H1V("split+w1", S | kVarWave1),
        H1V("split+direct", S | kVarDirectStore),
        H1V("split+rec", S | kVarWinRec),
        H1V("split+b64", S | kVarLdsB64),
        H1V("split+w1+rec", S | kVarWave1 | kVarWinRec),
        H1V("split+w1+rec+b64", S | kVarWave1 | kVarWinRec | kVarLdsB64),
        H1V("split+rec+b64", S | kVarWinRec | kVarLdsB64),
        H1V("aos+w1+rec", A | kVarWave1 | kVarWinRec),
        H1V("split+w1+tab+b64", S | kVarWave1 | kVarWinTab | kVarLdsB64),
    };
    {  // every variant against the previous library default on the first 4096 windows
        std::vector<double> ref((size_t)4096 * (n / 2));
        SpectrumLaunch R = L;
        R.n_windows = 4096;
        CK((launch_one<double, LOG2N, kDetrendNone, kOutPower, kWinCos, S>(R, 0)));
        CK(hipMemcpy(ref.data(), out, ref.size() * 8, hipMemcpyDeviceToHost));
        for (const auto &v : vars) printf("check %-28s max rel err vs split %.3e\n", v.name, v.check(R, ref));
        fflush(stdout);
    }
    for (int round = 0; round < 2; ++round)
        for (int g : {32768, 65536, 131072}) {
            L.grid = g;
            for (const auto &v : vars) {
                const float us = v.time(L, reps);
                printf("round %d grid=%6d %-28s %8.1f us  %7.1f GB/s  %.3f of 8 TB/s\n", round, g, v.name, us,
                       bytes / us / 1e3, bytes / us / 1e3 / 8000.0);
            }
            fflush(stdout);
        }
    return 0;
}


int main(int argc, char **argv) {
    if (argc > 1 && std::string(argv[1]) == "hop1") {  // kbench hop1 [log2n=11] [windows=1M] [reps=5]
        const int lg = argc > 2 ? atoi(argv[2]) : 11;
        const int64_t W = argc > 3 ? atoll(argv[3]) : (1 << 20);
        const int reps = argc > 4 ? atoi(argv[4]) : 5;
        switch (lg) {
        case 9: return hop1_main<9>(W, reps);
        case 10: return hop1_main<10>(W, reps);
        case 11: return hop1_main<11>(W, reps);
        case 12: return hop1_main<12>(W, reps);
        default: return 1;
        }
    }
    if (argc > 1 && std::string(argv[1]) == "out") return out_main(argc > 2 ? atoi(argv[2]) : 20);
    if (argc > 1 && std::string(argv[1]) == "copy") return copy_main(argc > 2 ? atoi(argv[2]) : 20, argc > 3 ? atoi(argv[3]) : 3);
    if (argc > 1 && std::string(argv[1]) == "store") {  // kbench store [reps=20] [rounds=4]: NT vs plain power-row stores
        const int reps = argc > 2 ? atoi(argv[2]) : 20, rounds = argc > 3 ? atoi(argv[3]) : 4;
        const int64_t W = 65536;
        const int n = 4096;
        double *x, *out, *tw;
        CK(hipMalloc(&x, W * n * 8));
        CK(hipMalloc(&out, W * n / 2 * 8));
        CK(hipMalloc(&tw, n * 16));
        std::vector<double> h(2 * n);
        for (int k = 0; k < n; ++k) {
            long double a = -2.0L * 3.14159265358979323846264338327950288L * k / n;
            h[2 * k] = (double)cosl(a), h[2 * k + 1] = (double)sinl(a);
        }
        CK(hipMemcpy(tw, h.data(), n * 16, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(fill_walk, dim3(4096), dim3(256), 0, 0, x, W * n);
        hipStream_t s;
        CK(hipStreamCreate(&s));
        SpectrumLaunch L{};
        L.series = x, L.out = out, L.twiddle = tw, L.window = 1, L.hop = n, L.n_windows = W, L.log2n = 12;
        L.nt_mode = 1, L.grid = kDefaultGrid;
        const double bytes = (double)W * n * 8 * 1.5;
        for (int round = 0; round < rounds; ++round) {
            const float a = time_variant<kDefaultVar | kVarNtLoad>(L, s, reps);
            const float b = time_variant<(kDefaultVar & ~kVarNtStore) | kVarNtLoad>(L, s, reps);
            const float c = time_variant<(kDefaultVar & ~kVarNtStore)>(L, s, reps);
            L.nt_mode = 2;  // nt loads chosen at run time (a.nt, hop >= N): the round-2 library before ct_nt_variant
            const float d = time_variant<kDefaultVar>(L, s, reps);
            L.nt_mode = 1;
            const float e = time_variant<kDefaultVar | kVarNtLoad | kVarVec>(L, s, reps);
            const float f = time_variant<kDefaultVar | kVarNtLoad | kVarWtStore>(L, s, reps);
            const float g = time_variant<kDefaultVar | kVarNtLoad | kVarVec | kVarWtStore>(L, s, reps);
            printf("round %d  nt-store %7.1f us %6.0f GB/s | plain-store %7.1f us %6.0f GB/s | plain-store, cached loads %7.1f us %6.0f GB/s | run-time nt loads %7.1f us %6.0f GB/s | nt + compile-time pair loads %7.1f us %6.0f GB/s | write-through store %7.1f us %6.0f GB/s | wt + pair loads %7.1f us %6.0f GB/s\n",
                   round, a, bytes / a / 1e3, b, bytes / b / 1e3, c, bytes / c / 1e3, d, bytes / d / 1e3, e, bytes / e / 1e3,
                   f, bytes / f / 1e3, g, bytes / g / 1e3);
            fflush(stdout);
        }
        return 0;
    }
    const int64_t W = argc > 1 ? atoll(argv[1]) : 65536;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const int n = 4096;
    const int64_t len = W * n;
    double *x, *out, *tw;
    CK(hipMalloc(&x, len * 8));
    CK(hipMalloc(&out, W * n / 2 * 8));
    CK(hipMalloc(&tw, n * 16));
    std::vector<double> h(2 * n);
    for (int k = 0; k < n; ++k) {
        long double a = -2.0L * 3.14159265358979323846264338327950288L * k / n;
        h[2 * k] = (double)cosl(a);
        h[2 * k + 1] = (double)sinl(a);
    }
    CK(hipMemcpy(tw, h.data(), n * 16, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(fill_walk, dim3(4096), dim3(256), 0, 0, x, len);
    CK(hipDeviceSynchronize());
    hipStream_t s;
    CK(hipStreamCreate(&s));

    SpectrumLaunch L{};
    L.series = x;
    L.out = out;
    L.twiddle = tw;
    L.window = 1;
    L.hop = n;
    L.n_windows = W;
    L.log2n = 12;
    L.output = 0;
    L.nt_mode = 1;  // variants choose nt loads via VAR (kVarNtLoad)
    const double bytes = (double)len * 8 + (double)W * n / 2 * 8;
    printf("# W=%lld N=%d algorithmic bytes=%.3f GB, roofline(8 TB/s)=%.1f us\n", (long long)W, n, bytes / 1e9,
           bytes / 8e12 * 1e6);

    // fixed sizes and whole rounds of resident workgroups (6 per CU x 256 CUs = 1536 at 3 waves/SIMD)
    const int grids[] = {1536, 3072, 6144, 12288, 21846, 32768, 65536};
    for (int round = 0; round < rounds; ++round) {
        // copy ceiling
        if (getenv("KBENCH_COPIES")) {
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            for (int kind = 0; kind < 5; ++kind)
                for (int g : {1024, 2048, 8192}) {
                    auto go = [&] {
                        if (kind == 0)  // 1:1 copy of out-sized region x2 (same bytes: read 2/3, write... see below)
                            hipLaunchKernelGGL(copy11, dim3(g), dim3(256), 0, s, (const double2 *)x, (double2 *)out, len / 4);
                        else if (kind == 1)
                            hipLaunchKernelGGL(copy21, dim3(g), dim3(256), 0, s, (const double2 *)x, (double2 *)out, len / 4);
                        else if (kind == 2)
                            hipLaunchKernelGGL(copy21u<false>, dim3(g), dim3(256), 0, s, (const double2 *)x, (double2 *)out, len / 4);
                        else if (kind == 3)
                            hipLaunchKernelGGL(copy21u<true>, dim3(g), dim3(256), 0, s, (const double2 *)x, (double2 *)out, len / 4);
                        else
                            hipLaunchKernelGGL(copy11x4, dim3(g), dim3(256), 0, s, (const double2 *)x, (double2 *)out, len / 4);
                    };
                    go();
                    CK(hipEventRecord(e0, s));
                    for (int i = 0; i < reps; ++i) go();
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    const double us = ms * 1000.0 / reps;
                    const double b = (kind == 0 || kind == 4) ? (double)len / 4 * 32 : bytes;  // copy11: 16 B in + 16 B out
                    const char *nm[] = {"copy11", "copy21", "copy21u", "copy21u-nt", "copy11x4"};
                    printf("round %d %-11s grid=%6d  %8.1f us  %7.1f GB/s\n", round, nm[kind], g, us, b / us / 1e3);
                }
        }
        for (int g : grids) {
            L.grid = g;
            struct {
                const char *name;
                float us;
            } r[5] = {{"library", time_variant<kDefaultVar | kVarNtLoad>(L, s, reps)},
                      {"split+nt2", time_variant<kVarSplitLds | kVarNoPrefetch | kVarNtLoad | kVarNtStore>(L, s, reps)},
                      {"split+nt2+rec+b64", time_variant<kVarSplitLds | kVarNoPrefetch | kVarNtLoad | kVarNtStore |
                                                         kVarWinRec | kVarLdsB64>(L, s, reps)},
                      {"split+nt2+twtab", time_variant<kVarSplitLds | kVarNoPrefetch | kVarNtLoad | kVarNtStore | kVarTwTable>(L, s, reps)},
                      {"skelwide", time_variant<kVarSkelWide | kVarNoPrefetch | kVarNtLoad>(L, s, reps)}};
            for (auto &v : r)
                printf("round %d %-11s grid=%6d  %8.1f us  %7.1f GB/s  %.3f of 8TB/s\n", round, v.name, g, v.us,
                       bytes / v.us / 1e3, bytes / v.us / 1e3 / 8000.0);
        }
        fflush(stdout);
    }
    return 0;
}
