// regfft_check.hip -- diagnostic: slide_mixed.hip's register-pass seed FFT (fft_reg_sub) against its LDS form
// (fft_lds_sub) and an fp64 host DFT, one workgroup per geometry the mixed launch uses (N, NT).
//   bin/regfft_check
#include <cmath>
#include <complex>
#include <cstdio>
#include <vector>

#include "../csrc/slide_mixed.hip"

namespace wsp {
namespace {
template <int LOG2N, int NT> __global__ void check_kernel(const d2 *x, const d2 *tw4096, d2 *out_reg, d2 *out_lds) {
    constexpr int N = 1 << LOG2N, R = N / NT;
    __shared__ d2 buf[N];
    __shared__ d2 twq[1024];
    const int t = threadIdx.x;
    for (int i = t; i < 1024; i += NT) twq[i] = tw4096[i];
    __syncthreads();
    d2 a[R];
#pragma unroll
    for (int r = 0; r < R; ++r) a[r] = x[t + NT * r];
    fft_reg_sub<LOG2N, NT>(a, buf, twq, t);
    for (int i = t; i < N; i += NT) out_reg[i] = buf[i];
    __syncthreads();
    for (int i = t; i < N; i += NT) buf[i] = x[i];
    __syncthreads();
    fft_lds_sub<LOG2N, NT>(buf, twq, t);
    for (int i = t; i < N; i += NT) out_lds[i] = buf[i];
}
template <int LOG2N, int NT> int run(const d2 *dx, const d2 *dtw, const std::vector<d2> &hx) {
    constexpr int N = 1 << LOG2N;
    d2 *dr, *dl;
    if (hipMalloc(&dr, N * sizeof(d2)) != hipSuccess || hipMalloc(&dl, N * sizeof(d2)) != hipSuccess) return 1;
    hipLaunchKernelGGL((check_kernel<LOG2N, NT>), dim3(1), dim3(NT), 0, 0, dx, dtw, dr, dl);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    std::vector<d2> r(N), l(N);
    (void)hipMemcpy(r.data(), dr, N * sizeof(d2), hipMemcpyDeviceToHost);
    (void)hipMemcpy(l.data(), dl, N * sizeof(d2), hipMemcpyDeviceToHost);
    double er = 0, el = 0, mx = 0;
    for (int k = 0; k < N; ++k) {
        std::complex<long double> s = 0;
        for (int i = 0; i < N; ++i)
            s += std::complex<long double>(hx[i].x, hx[i].y) * std::polar(1.0L, -2.0L * 3.14159265358979323846264L * (long double)((long)k * i % N) / N);
        const std::complex<double> sd((double)s.real(), (double)s.imag());
        er = std::max(er, std::abs(sd - std::complex<double>(r[k].x, r[k].y)));
        el = std::max(el, std::abs(sd - std::complex<double>(l[k].x, l[k].y)));
        mx = std::max(mx, std::abs(sd));
    }
    printf("N=%5d NT=%4d  register passes rel err %.3e   LDS passes rel err %.3e  %s\n", N, NT, er / mx, el / mx,
           er / mx < 1e-13 ? "ok" : "FAIL");
    (void)hipFree(dr);
    (void)hipFree(dl);
    return er / mx < 1e-13 ? 0 : 2;
}
}  // namespace
}  // namespace wsp

int main() {
    using namespace wsp;
    std::vector<d2> hx(4096), htw(1024);
    for (int i = 0; i < 4096; ++i) hx[i] = d2{std::sin(0.37 * i) + 1e-3 * i, std::cos(0.11 * i)};
    for (int k = 0; k < 1024; ++k) htw[k] = d2{std::cos(-2 * M_PI * k / 4096), std::sin(-2 * M_PI * k / 4096)};
    d2 *dx, *dtw;
    if (hipMalloc(&dx, 4096 * sizeof(d2)) != hipSuccess || hipMalloc(&dtw, 1024 * sizeof(d2)) != hipSuccess) return 1;
    (void)hipMemcpy(dx, hx.data(), 4096 * sizeof(d2), hipMemcpyHostToDevice);
    (void)hipMemcpy(dtw, htw.data(), 1024 * sizeof(d2), hipMemcpyHostToDevice);
    int bad = 0;
    bad |= run<12, 512>(dx, dtw, hx);
    bad |= run<11, 256>(dx, dtw, hx);
    bad |= run<10, 256>(dx, dtw, hx);
    bad |= run<9, 128>(dx, dtw, hx);
    bad |= run<10, 128>(dx, dtw, hx);
    bad |= run<9, 64>(dx, dtw, hx);
    return bad;
}
