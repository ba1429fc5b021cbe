// kstep_probe.hip -- cycles per Kalman step of one wave per SIMD, without IO (tools only).
// Every SIMD runs exactly one wave (4-wave workgroups + an LDS reservation admitting one per CU);
// each lane steps CH independent packed two-segment states (kalman_core.h KState2) over a
// register-generated measurement stream, so the probe separates the step's issue cost from its
// dependency-chain latency: CH = 1 is the library's form, CH = 2 the same work with two chains
// interleaved (independent instruction streams the scheduler can fill each other's waits with).
//   kstep_probe [steps=4096]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../csrc/kalman_core.h"

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

using namespace wsp;
using kcore::kf2;

static const double kDefaults[16] = {1.0, 0.01, 0.003, 0.0008, 0.0002, 0.8, 1.0, 16.0, 9.0, 4.0, 1.0, 0.0, 0.0, 0.0, 6.0, 0.0};

// MODE 0: kstep_pk2 (original basis, floors); 1: kstep_nb2 (Newton basis, guard)
template <int MODE, int CH>
__global__ __launch_bounds__(256) void probe(float *out, long long *cyc, kcore::KP kp, int steps) {
    const kcore::KConst<float> kc = kcore::kconst<float, kcore::kKfAdapt | kcore::kKfClip>(kp);
    const kcore::KNb kn = kcore::knb_const(kp);
    kcore::KState2 st[CH];
    for (int c = 0; c < CH; ++c) {
        kcore::knb_reset(st[c], kp);
        if (MODE == 0) st[c].p11 = st[c].p22 = st[c].p33 = st[c].p00, st[c].p12 = st[c].p13 = st[c].p23 = kf2{0.f, 0.f};
    }
    // measurement stream: a rotating phasor (independent of the filter's chain), per lane and chain
    const float th = 0.05f + 1e-4f * (threadIdx.x % 64);
    kf2 cs = {1.f, 0.f};
    const kf2 rot = {cosf(th), sinf(th)};
    kf2 acc = {0.f, 0.f}, emin = {1e30f, 1e30f};
    __builtin_amdgcn_s_barrier();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int t = 0; t < steps; ++t) {
        cs = kf2{cs.x * rot.x - cs.y * rot.y, cs.x * rot.y + cs.y * rot.x};
        const kf2 z = 1e-3f * cs;
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const kf2 zc = c ? kf2{z.y, z.x} : z;
            if constexpr (MODE == 0) {
                acc += kcore::kstep_pk2(st[c], kc, zc);
            } else {
                kf2 e;
                acc += kcore::kstep_nb2(st[c], kn, zc, e);
                emin.x = fminf(emin.x, e.x);
                emin.y = fminf(emin.y, e.y);
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x + acc.y + emin.x + emin.y;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int MODE, int CH> void run(const char *name, int cus, int steps, float *out, long long *cyc) {
    kcore::KP kp;
    memcpy(&kp, kDefaults, sizeof(kp));
    const size_t reserve = 84 * 1024;
    for (int rep = 0; rep < 2; ++rep) {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((probe<MODE, CH>), dim3(cus), dim3(256), reserve, 0, out, cyc, kp, steps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<long long> h((size_t)cus * 4);
        CK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
        double avg = 0;
        for (long long v : h) avg += (double)v;
        avg /= h.size();
        if (rep)
            printf("%-34s chains %d: %7.1f memtime ticks per step of one chain (two segments); wall %.3f ms for %d steps x %d chains\n",
                   name, CH, avg / ((double)steps * CH), ms, steps, CH);
    }
}

int main(int argc, char **argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 4096;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    float *out;
    long long *cyc;
    CK(hipMalloc(&out, (size_t)cus * 256 * 4));
    CK(hipMalloc(&cyc, (size_t)cus * 4 * 8));
    for (int r = 0; r < 2; ++r) {
        run<0, 1>("kstep_pk2 (original basis)", cus, steps, out, cyc);
        run<0, 2>("kstep_pk2 (original basis)", cus, steps, out, cyc);
        run<1, 1>("kstep_nb2 (Newton basis)", cus, steps, out, cyc);
        run<1, 2>("kstep_nb2 (Newton basis)", cus, steps, out, cyc);
        run<1, 3>("kstep_nb2 (Newton basis)", cus, steps, out, cyc);
    }
    return 0;
}
