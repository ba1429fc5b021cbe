// unaligned_probe.hip -- checks that 16-B loads at 8-B-aligned addresses return
// the right data on this GPU (ROCm unaligned-access mode), and times hop=1
// spectra with scalar vs vector pair loads.  Experiment tool, not in the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../csrc/spectrum_dispatch.h"
using namespace wsp;
using namespace wsp::core;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));
__global__ void probe(const double *x, double *out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { d2 v = *reinterpret_cast<const d2 *>(x + 2 * i + 1); out[2 * i] = v.x; out[2 * i + 1] = v.y; }
}
int main() {
    const int n = 1 << 20;
    std::vector<double> h(2 * n + 2);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (double)i * 0.5 + 1.0;
    double *x, *o;
    CK(hipMalloc(&x, h.size() * 8)); CK(hipMalloc(&o, 2 * n * 8));
    CK(hipMemcpy(x, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(probe, dim3(n / 256), dim3(256), 0, 0, x, o, n);
    CK(hipDeviceSynchronize());
    std::vector<double> r(2 * n);
    CK(hipMemcpy(r.data(), o, 2 * n * 8, hipMemcpyDeviceToHost));
    long bad = 0;
    for (int i = 0; i < 2 * n; ++i) bad += r[i] != h[i + 1];
    printf("unaligned 16-B loads: %ld mismatches of %d\n", bad, 2 * n);
    if (bad) return 2;
    // hop = 1 spectra (C4 shape): 1M windows x 2048, scalar vs vector pair loads
    const int64_t W = 1 << 20; const int N = 2048;
    double *s, *out, *tw;
    CK(hipMalloc(&s, (W + N) * 8)); CK(hipMalloc(&out, W * N / 2 * 8)); CK(hipMalloc(&tw, N * 8));
    std::vector<double> t(N);
    for (int k = 0; k < N / 2; ++k) { long double a = -2.0L * 3.14159265358979323846L * k / N; t[2*k] = (double)cosl(a); t[2*k+1] = (double)sinl(a); }
    CK(hipMemcpy(tw, t.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(s, h.data(), 1024 * 8, hipMemcpyHostToDevice));
    SpectrumLaunch L{}; L.series = s; L.out = out; L.twiddle = tw; L.window = 1; L.hop = 1; L.n_windows = W; L.log2n = 11;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int round = 0; round < 2; ++round)
        for (int vm : {1, 2}) for (int g : {8192, 16384, 65536}) {
            L.vec_mode = vm; L.grid = g;
            CK((launch_one<double, 11, kDetrendNone, kOutPower, kWinCos>(L, 0)));
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < 5; ++i) CK((launch_one<double, 11, kDetrendNone, kOutPower, kWinCos>(L, 0)));
            CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            const double bytes = (W + N) * 8.0 + W * (N / 2) * 8.0;
            printf("round %d hop1 %s grid=%6d %8.1f us  %7.1f GB/s\n", round, vm == 1 ? "scalar" : "vector", g, ms * 200, bytes / (ms * 200) / 1e3);
        }
    return 0;
}
