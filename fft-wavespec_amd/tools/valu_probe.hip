// valu_probe.hip -- issue cost of fp32 VALU forms for one or two waves per SIMD (tools only).
// Every SIMD of the chip gets exactly WPS waves (workgroups of 4*WPS waves with an LDS reservation
// admitting one workgroup per CU); each wave runs ILP independent dependency chains of one
// instruction form; cycles per instruction per wave from s_memtime.
//   valu_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 512;

template <int MODE, int ILP>
__global__ void probe(float *out, long long *cyc, float s) {
    f2 a[ILP];
#pragma unroll
    for (int i = 0; i < ILP; ++i) a[i] = f2{s * (threadIdx.x + i), s + i};
    const f2 b = {s, 0.5f * s}, c = {0.25f * s, s};
    __builtin_amdgcn_s_barrier();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < ILP; ++i) {
            if constexpr (MODE == 0) {  // v_fma_f32 on one half
                float x = a[i].x;
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(b.x), "v"(c.x));
                a[i].x = x;
            } else if constexpr (MODE == 1) {
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            } else if constexpr (MODE == 2) {
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            } else if constexpr (MODE == 3) {
                float x = a[i].x;
                asm volatile("v_rsq_f32 %0, %0" : "+v"(x));
                a[i].x = x;
            } else {
                float x = a[i].x;
                asm volatile("v_max_f32 %0, %0, %1" : "+v"(x) : "v"(b.x));
                a[i].x = x;
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float r = 0;
#pragma unroll
    for (int i = 0; i < ILP; ++i) r += a[i].x + a[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE, int ILP> void run(const char *name, int wps, int cus, float *out, long long *cyc) {
    const int threads = 256 * wps, blocks = cus;
    const size_t reserve = 84 * 1024;  // one workgroup per CU
    hipLaunchKernelGGL((probe<MODE, ILP>), dim3(blocks), dim3(threads), reserve, 0, out, cyc, 1.0001f);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((probe<MODE, ILP>), dim3(blocks), dim3(threads), reserve, 0, out, cyc, 1.0001f);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<long long> h((size_t)blocks * threads / 64);
    CK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
    double avg = 0;
    for (long long v : h) avg += (double)v;
    avg /= h.size();
    const double per = avg / ((double)kIters * ILP);
    printf("%-14s ILP %d  %d wave/SIMD: %6.2f memtime ticks per instr per wave; wall %.4f ms = %.2f cyc (2.4 GHz) per instr per SIMD\n",
           name, ILP, wps, per, ms, ms * 1e-3 * 2.4e9 / ((double)kIters * ILP * wps));
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    float *out;
    long long *cyc;
    CK(hipMalloc(&out, (size_t)cus * 1024 * 4));
    CK(hipMalloc(&cyc, (size_t)cus * 16 * 8));
    for (int wps = 1; wps <= 2; ++wps) {
        run<0, 1>("v_fma_f32", wps, cus, out, cyc);
        run<0, 8>("v_fma_f32", wps, cus, out, cyc);
        run<1, 1>("v_pk_fma_f32", wps, cus, out, cyc);
        run<1, 2>("v_pk_fma_f32", wps, cus, out, cyc);
        run<1, 8>("v_pk_fma_f32", wps, cus, out, cyc);
        run<2, 8>("v_pk_add_f32", wps, cus, out, cyc);
        run<3, 1>("v_rsq_f32", wps, cus, out, cyc);
        run<3, 8>("v_rsq_f32", wps, cus, out, cyc);
        run<4, 8>("v_max_f32", wps, cus, out, cyc);
    }
    return 0;
}
