// dpp_probe.hip -- checks the DPP wave_shr:1 / wave_shl:1 lane semantics the phase record relies on
// (spectrum_core.h phase_chunk<..., kDpp>): lane l reads lane l - 1 / l + 1.  Not part of the library.
#include <hip/hip_runtime.h>
__device__ __forceinline__ double dshr(double v) {
    const unsigned long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), 0x138, 0xf, 0xf, false);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double dshl(double v) {
    const unsigned long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), 0x130, 0xf, 0xf, false);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__global__ void k(const double *in, double *a, double *b) {
    double v = in[threadIdx.x];
    a[threadIdx.x] = dshr(v);
    b[threadIdx.x] = dshl(v);
}
int main() {  // wave_shr:1 / wave_shl:1 semantics on gfx950 (tools only)
    double *in, *a, *b; (void)hipMalloc(&in, 64*8); (void)hipMalloc(&a, 64*8); (void)hipMalloc(&b, 64*8);
    double h[64]; for (int i = 0; i < 64; ++i) h[i] = i + 0.5;
    (void)hipMemcpy(in, h, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, in, a, b);
    double ha[64], hb[64]; (void)hipMemcpy(ha, a, 512, hipMemcpyDeviceToHost); (void)hipMemcpy(hb, b, 512, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 64; ++i) {
        if (i > 0 && ha[i] != h[i-1]) bad++;
        if (i < 63 && hb[i] != h[i+1]) bad++;
    }
    printf("shr: lane0=%g lane1=%g lane63=%g | shl: lane0=%g lane62=%g lane63=%g | bad=%d\n", ha[0], ha[1], ha[63], hb[0], hb[62], hb[63], bad);
    return bad != 0;
}
