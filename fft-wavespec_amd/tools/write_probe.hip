// write_probe.hip -- HBM write ceiling for the sliding-DFT output stream (C4: 8.6 GB of power rows).
// Variants: non-temporal vs plain stores, 8-B vs 16-B per lane; contiguous 1 KiB-per-wave-instruction
// pieces walked by each workgroup in row order (the slide kernel's pattern) or grid-strided.
// Usage: write_probe [GiB] [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double d2 __attribute__((ext_vector_type(2)));

template <bool NT, bool WIDE, bool ROWS>
__global__ __launch_bounds__(256) void wr(double *out, long n, long rows_per_wg, int row) {
    const int t = threadIdx.x;
    if (ROWS) {  // workgroup b writes rows [b*rows_per_wg, ...) of `row` doubles, like a slide segment
        long r0 = (long)blockIdx.x * rows_per_wg;
        for (long r = r0; r < r0 + rows_per_wg; ++r) {
            double *o = out + r * row;
            if (r * row >= n) return;
            for (int k = (WIDE ? 2 : 1) * t; k < row; k += (WIDE ? 2 : 1) * 256) {
                if (WIDE) {
                    d2 v = {(double)r, (double)k};
                    if (NT) __builtin_nontemporal_store(v, reinterpret_cast<d2 *>(o + k));
                    else *reinterpret_cast<d2 *>(o + k) = v;
                } else {
                    if (NT) __builtin_nontemporal_store((double)k, o + k);
                    else o[k] = (double)k;
                }
            }
        }
    } else {
        long stride = (long)gridDim.x * 256 * (WIDE ? 2 : 1);
        for (long i = ((long)blockIdx.x * 256 + t) * (WIDE ? 2 : 1); i < n; i += stride) {
            if (WIDE) {
                d2 v = {(double)i, 1.0};
                if (NT) __builtin_nontemporal_store(v, reinterpret_cast<d2 *>(out + i));
                else *reinterpret_cast<d2 *>(out + i) = v;
            } else {
                if (NT) __builtin_nontemporal_store((double)i, out + i);
                else out[i] = (double)i;
            }
        }
    }
}

template <bool NT, bool WIDE, bool ROWS> void run(const char *name, double *d, long n, int reps) {
    const int row = 1024;
    const long rows = n / row;
    const int grid = ROWS ? 4096 : 8192;
    const long rpw = (rows + grid - 1) / grid;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((wr<NT, WIDE, ROWS>), dim3(grid), dim3(256), 0, 0, d, n, rpw, row);
    (void)hipEventRecord(a);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((wr<NT, WIDE, ROWS>), dim3(grid), dim3(256), 0, 0, d, n, rpw, row);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    printf("%-28s %8.3f ms  %7.0f GB/s\n", name, ms, n * 8.0 / ms / 1e6);
}

int main(int argc, char **argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 8.0;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const long n = (long)(gib * (1l << 30) / 8);
    double *d;
    if (hipMalloc(&d, n * 8) != hipSuccess) return 1;
    for (int round = 0; round < 2; ++round) {
        run<true, false, true>("rows nt 8B", d, n, reps);
        run<true, true, true>("rows nt 16B", d, n, reps);
        run<false, false, true>("rows plain 8B", d, n, reps);
        run<false, true, true>("rows plain 16B", d, n, reps);
        run<true, true, false>("gridstride nt 16B", d, n, reps);
        run<false, true, false>("gridstride plain 16B", d, n, reps);
    }
    (void)hipFree(d);
    return 0;
}
