// mall_probe.hip -- tools only.  Does a per-workgroup recycled scratch slot (the column results of a
// large-N window, 512 KiB at N = 65536 fp64) cost HBM bandwidth, or does the Infinity Cache absorb
// it?  Per window (one 1024-thread workgroup per window, grid-stride over 4096 windows):
//   stream : read the window (512 KiB), write half of it (256 KiB)            -- the algorithmic bytes
//   slot   : + write the window to the workgroup's slot, barrier, read it back transposed
//   slotnt : the same with non-temporal slot stores / loads
// Reports microseconds per launch and the effective bandwidth of the algorithmic bytes.
//   mall_probe [grid_per_cu=1]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));
constexpr int N = 65536, M = N / 2, T = 1024, PER = M / T;  // 32 complex per thread

template <int MODE>
__global__ __launch_bounds__(1024) void probe(const d2 *__restrict__ in, double *__restrict__ out, d2 *__restrict__ slots,
                                              int nwin) {
    d2 *slot = slots + (size_t)blockIdx.x * M;
    for (int w = blockIdx.x; w < nwin; w += gridDim.x) {
        const d2 *x = in + (size_t)w * M;
        double *o = out + (size_t)w * M;
        if constexpr (MODE == 0) {
#pragma unroll 8
            for (int r = 0; r < PER; ++r) {
                const d2 v = __builtin_nontemporal_load(x + threadIdx.x + T * r);
                __builtin_nontemporal_store(v.x + v.y, o + threadIdx.x + T * r);
            }
        } else {
#pragma unroll 8
            for (int r = 0; r < PER; ++r) {
                const d2 v = __builtin_nontemporal_load(x + threadIdx.x + T * r);
                if constexpr (MODE == 2) __builtin_nontemporal_store(v, slot + threadIdx.x + T * r);
                else slot[threadIdx.x + T * r] = v;
            }
            __syncthreads();
            // read back in another thread mapping, as the large-N column pass does: 16 lanes take 256 B
            // of one row, the wave's four 16-lane groups four rows 8 KiB apart
#pragma unroll 8
            for (int r = 0; r < PER; ++r) {
                const int i = (threadIdx.x % 16) + 16 * ((threadIdx.x / 16) * PER + r);
                const d2 v = MODE == 2 ? __builtin_nontemporal_load(slot + i) : slot[i];
                __builtin_nontemporal_store(v.x + v.y, o + threadIdx.x + T * r);
            }
            __syncthreads();
        }
    }
}

template <int MODE> float run(const d2 *in, double *out, d2 *slots, int nwin, int grid, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(probe<MODE>, dim3(grid), dim3(T), 0, 0, in, out, slots, nwin);
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(probe<MODE>, dim3(grid), dim3(T), 0, 0, in, out, slots, nwin);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3f / reps;
}

int main(int argc, char **argv) {
    const int per_cu = argc > 1 ? atoi(argv[1]) : 1;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int nwin = 4096, grid = cus * per_cu;
    d2 *in, *slots;
    double *out;
    CK(hipMalloc(&in, (size_t)nwin * M * sizeof(d2)));
    CK(hipMalloc(&out, (size_t)nwin * M * sizeof(double)));
    CK(hipMalloc(&slots, (size_t)grid * M * sizeof(d2)));
    CK(hipMemset(in, 0, (size_t)nwin * M * sizeof(d2)));
    const double alg = (double)nwin * (N * 8.0 + M * 8.0);  // read 512 KiB + write 256 KiB per window
    for (int round = 0; round < 2; ++round) {
        const float t0 = run<0>(in, out, slots, nwin, grid, 10), t1 = run<1>(in, out, slots, nwin, grid, 10),
                    t2 = run<2>(in, out, slots, nwin, grid, 10);
        printf("grid %d (%d/CU): stream %.1f us (%.2f TB/s)  slot %.1f us (%.2f TB/s)  slot-nt %.1f us (%.2f TB/s)  "
               "slot bytes %.2f GB per launch\n",
               grid, per_cu, t0, alg / t0 * 1e-6, t1, alg / t1 * 1e-6, t2, alg / t2 * 1e-6, 2.0 * nwin * M * 16.0 / 1e9);
    }
    return 0;
}
