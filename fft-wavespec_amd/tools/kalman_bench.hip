// kalman_bench.hip -- ablation and correctness probe of the Kalman detrend
// pre-pass (not part of the library).  Built with -fno-slp-vectorize like
// csrc/kalman_kernels.hip, so the timed code is the library's code.
//
//   kalman_bench time  [reps=10]   variants at C3 (65536 x 4096, f32), back to back
//                                  and alternating with a 1.5 GB streaming kernel
//                                  (the C3 step's spectrum launch in between)
//   kalman_bench check [n=256]     variants vs a host restatement of the reference step
//   kalman_bench ab    [reps=10]   the two-segment filter, original against Newton basis, alternating
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../csrc/kalman_core.h"

using namespace wsp;

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t err_ = (x);                                                                \
        if (err_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(err_), __FILE__, __LINE__); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

static const double kDefaults[16] = {1.0, 0.01, 0.003, 0.0008, 0.0002, 0.8, 1.0, 16.0, 9.0, 4.0, 1.0, 0.0, 0.0, 0.0, 6.0, 0.0};

static unsigned *g_fallbacks = nullptr;  // waves that re-ran their second segments (SEG = 2)
static double *g_dbg = nullptr;
static void dump_dbg(const char *name, int64_t W);          // SEG = 2: per window [exact state (14) | warm-up state (14)]

// launch one variant: WAVES = 4 adds the one-workgroup-per-CU LDS reservation (two per CU for SEG = 2)
template <typename T, int J, int FL, bool TWO, int WAVES, bool PK = false, int SEG = 1, int WU = kcore::kSegWarm>
void launch(const T *x, T *d, int64_t hop, int64_t W, int n, const kcore::KP &kp, hipStream_t s) {
    constexpr int WPW = SEG == 2 ? 32 : 64;
    const size_t stat = 4 * 64 * (J + 1) * sizeof(T);
    const size_t reserve = WAVES == 4 ? (SEG == 2 ? 78 : 84) * 1024 - stat : 0;
    hipLaunchKernelGGL((kcore::kalman_detrend_kernel<T, T, J, WPW, J, FL, TWO, WAVES, PK, SEG, WU>),
                       dim3((W + WPW * WAVES - 1) / (WPW * WAVES)), dim3(64 * WAVES), reserve, s, x, d, hop, W, n, kp,
                       g_fallbacks, g_dbg);
}

__global__ __launch_bounds__(256) void stream_copy(const double2 *__restrict__ in, double2 *__restrict__ out, int64_t n) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
        out[j] = in[j];
}

// the packed two-segment kernel (fp32, default flags)
template <int WAVES, int WU, bool ROT = true, int NB = 0>
void launch_pk2(const float *x, float *d, int64_t hop, int64_t W, int n, const kcore::KP &kp, hipStream_t s) {
    const size_t stat = (size_t)WAVES * 64 * 34 * 8;
    const size_t reserve = WAVES == 4 ? 84 * 1024 - stat : 0;
    hipLaunchKernelGGL((kcore::kalman_pk2_kernel<32, WAVES, WU, ROT, 0, NB>), dim3((W + 64 * WAVES - 1) / (64 * WAVES)),
                       dim3(64 * WAVES), reserve, s, x, d, hop, W, n, kp, g_fallbacks);
}

template <int WU>
void launch_pk4(const float *x, float *d, int64_t hop, int64_t W, int n, const kcore::KP &kp, hipStream_t s) {
    hipLaunchKernelGGL((kcore::kalman_pk4_kernel<16, WU>), dim3((W + 31) / 32), dim3(64), 0, s, x, d, hop, W, n, kp, g_fallbacks);
}

template <int FL, bool TWO, int WAVES, bool PK = false, int SEG = 1, int WU = kcore::kSegWarm>
void time_variant(const char *name, const float *x, float *d, const double2 *ci, double2 *co, int64_t cn, int64_t W, int n,
                  int reps, hipStream_t s) {
    kcore::KP kp;
    memcpy(&kp, kDefaults, sizeof(kp));
    hipEvent_t a, b, c;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventCreate(&c));
    launch<float, 32, FL, TWO, WAVES, PK, SEG, WU>(x, d, n, W, n, kp, s);
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) launch<float, 32, FL, TWO, WAVES, PK, SEG, WU>(x, d, n, W, n, kp, s);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float back, alt = 0;
    CK(hipEventElapsedTime(&back, a, b));
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(stream_copy, dim3(8192), dim3(256), 0, s, ci, co, cn);
        CK(hipEventRecord(a, s));
        launch<float, 32, FL, TWO, WAVES, PK, SEG, WU>(x, d, n, W, n, kp, s);
        CK(hipEventRecord(c, s));
        CK(hipEventSynchronize(c));
        float t;
        CK(hipEventElapsedTime(&t, a, c));
        alt += t;
    }
    printf("%-44s back-to-back %8.1f us   after a streaming kernel %8.1f us\n", name, back * 1e3f / reps, alt * 1e3f / reps);
    fflush(stdout);
}

// SEGS = 5: the two-segment kernel in the Newton basis (kstep_nb2)
template <int WAVES, int WU, int SEGS = 2, bool ROT = true>
void time_pk2(const char *name, const float *x, float *d, const double2 *ci, double2 *co, int64_t cn, int64_t W, int n, int reps,
              hipStream_t s) {
    kcore::KP kp;
    memcpy(&kp, kDefaults, sizeof(kp));
    hipEvent_t a, b, c;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventCreate(&c));
    CK(hipMemset(g_fallbacks, 0, 4));
    auto go = [&]() {
        if constexpr (SEGS == 4) launch_pk4<WU>(x, d, n, W, n, kp, s);
        else if constexpr (SEGS == 5) launch_pk2<WAVES, WU, ROT, 1>(x, d, n, W, n, kp, s);
        else if constexpr (SEGS == 6) launch_pk2<WAVES, WU, ROT, 3>(x, d, n, W, n, kp, s);
        else launch_pk2<WAVES, WU, ROT>(x, d, n, W, n, kp, s);
    };
    go();
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) go();
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float back, alt = 0;
    CK(hipEventElapsedTime(&back, a, b));
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(stream_copy, dim3(8192), dim3(256), 0, s, ci, co, cn);
        CK(hipEventRecord(a, s));
        go();
        CK(hipEventRecord(c, s));
        CK(hipEventSynchronize(c));
        float t;
        CK(hipEventElapsedTime(&t, a, c));
        alt += t;
    }
    unsigned fb = 0;
    CK(hipMemcpy(&fb, g_fallbacks, 4, hipMemcpyDeviceToHost));
    printf("%-44s back-to-back %8.1f us   after a streaming kernel %8.1f us   fallback waves %u (+ %u guard) of %lld x %d\n",
           name, back * 1e3f / reps, alt * 1e3f / reps, fb & 0xffffu, fb >> 16, (long long)(W / 64), 1 + 2 * reps);
    fflush(stdout);
}

// one or two waves per SIMD?  pk2 and pk4 at half the C3 batch (pk4: one wave per SIMD) and the full one
int occ_main(int reps) {
    const int n = 4096;
    const int64_t W = 65536;
    float *x, *d;
    CK(hipMalloc(&x, W * n * 4));
    CK(hipMalloc(&d, W * n * 4));
    std::vector<float> h(W * n);
    std::mt19937_64 rng(11);
    std::normal_distribution<double> nd;
    double v = 1.1;
    for (int64_t i = 0; i < W * n; ++i) {
        v += 1e-4 * nd(rng);
        h[i] = (float)(v + 0.002 * sin(2 * M_PI * (double)i / 50));
    }
    CK(hipMemcpy(x, h.data(), W * n * 4, hipMemcpyHostToDevice));
    kcore::KP kp;
    memcpy(&kp, kDefaults, sizeof(kp));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int round = 0; round < 2; ++round)
        for (int64_t w : {(int64_t)4096, (int64_t)8192, (int64_t)16384, (int64_t)32768, (int64_t)65536}) {
            for (int k = 0; k < 2; ++k) {
                auto go = [&]() {
                    if (k) launch_pk4<kcore::kPk2Warm>(x, d, n, w, n, kp, 0);
                    else launch_pk2<1, kcore::kPk2Warm>(x, d, n, w, n, kp, 0);
                };
                go();
                CK(hipEventRecord(a, 0));
                for (int r = 0; r < reps; ++r) go();
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                printf("%s windows %6lld: %8.1f us\n", k ? "pk4" : "pk2", (long long)w, ms * 1e3f / reps);
            }
        }
    return 0;
}

int time_main(int reps, bool nb_only) {
    const int64_t W = 65536;
    const int n = 4096;
    float *x, *d;
    CK(hipMalloc(&x, W * n * 4));
    CK(hipMalloc(&d, W * n * 4));
    std::vector<float> h(W * n);
    std::mt19937_64 rng(11);
    std::normal_distribution<double> nd;
    double v = 1.1;
    for (int64_t i = 0; i < W * n; ++i) {  // synth.random_walk: 1.1 + cumsum(1e-4 N(0,1)) + 0.002 sin(2 pi t/50)
        v += 1e-4 * nd(rng);
        h[i] = (float)(v + 0.002 * sin(2 * M_PI * (double)i / 50));
    }
    CK(hipMemcpy(x, h.data(), W * n * 4, hipMemcpyHostToDevice));
    const int64_t cn = (int64_t)768 << 20 >> 4;  // 768 MiB in, 768 MiB out
    double2 *ci, *co;
    CK(hipMalloc(&ci, cn * 16));
    CK(hipMalloc(&co, cn * 16));
    CK(hipMemset(ci, 0, cn * 16));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    if (nb_only) {  // the round-6 A/B: original basis against the Newton basis, alternating
        for (int round = 0; round < 4; ++round) {
            time_pk2<1, 256>("packed 2 segments WU=256, original basis", x, d, ci, co, cn, W, n, reps, s);
            time_pk2<1, 256, 5>("packed 2 segments WU=256, Newton basis", x, d, ci, co, cn, W, n, reps, s);
            time_pk2<1, 256, 6>("packed 2 segments WU=256, tile IO only", x, d, ci, co, cn, W, n, reps, s);
        }
        return 0;
    }
    for (int round = 0; round < 2; ++round) {
        printf("round %d\n", round);
        time_variant<kcore::kKfRuntime, true, 1>("1-wave WG, runtime flags, two-stage", x, d, ci, co, cn, W, n, reps, s);
        time_variant<3, false, 1>("1-wave WG, static flags, expanded", x, d, ci, co, cn, W, n, reps, s);
        time_variant<3, true, 1>("1-wave WG, static flags, two-stage", x, d, ci, co, cn, W, n, reps, s);
        time_variant<3, true, 4>("4-wave WG + 1 WG/CU, static, two-stage", x, d, ci, co, cn, W, n, reps, s);
        time_variant<kcore::kKfRuntime, true, 4>("4-wave WG + 1 WG/CU, runtime, two-stage", x, d, ci, co, cn, W, n, reps, s);
        time_variant<3, true, 4, true>("4-wave WG + 1 WG/CU, static, packed update", x, d, ci, co, cn, W, n, reps, s);
        time_pk2<4, 128>("packed 2 segments WU=128, 4-wave WG", x, d, ci, co, cn, W, n, reps, s);
        time_pk2<4, 256>("packed 2 segments WU=256, 4-wave WG", x, d, ci, co, cn, W, n, reps, s);
        time_pk2<4, 512>("packed 2 segments WU=512, 4-wave WG", x, d, ci, co, cn, W, n, reps, s);
        time_pk2<1, 256, 2, false>("packed 2 segments WU=256, 1-wave WG, unrotated", x, d, ci, co, cn, W, n, reps, s);
        time_pk2<1, 256>("packed 2 segments WU=256, 1-wave WG", x, d, ci, co, cn, W, n, reps, s);
        time_pk2<1, 256, 5>("packed 2 segments WU=256, Newton basis", x, d, ci, co, cn, W, n, reps, s);
        time_pk2<1, 256, 4>("packed 4 segments WU=256, lane pairs", x, d, ci, co, cn, W, n, reps, s);
        time_pk2<1, 512, 4>("packed 4 segments WU=512, lane pairs", x, d, ci, co, cn, W, n, reps, s);
        if (round > 0) continue;
        auto seg = [&](auto wu) {
            constexpr int WU = decltype(wu)::value;
            CK(hipMemset(g_fallbacks, 0, 4));
            char nm[96];
            snprintf(nm, sizeof nm, "2 segments WU=%d, 4-wave WG + 2 WG/CU", WU);
            time_variant<3, true, 4, true, 2, WU>(nm, x, d, ci, co, cn, W, n, reps, s);
            unsigned fb = 0;
            CK(hipMemcpy(&fb, g_fallbacks, 4, hipMemcpyDeviceToHost));
            printf("    fallbacks: %u waves of %lld over %d launches\n", fb, (long long)(W / 32), 1 + 2 * reps);
            dump_dbg(nm, W);
        };
        seg(std::integral_constant<int, 256>{});
        seg(std::integral_constant<int, 512>{});
        seg(std::integral_constant<int, 768>{});
        seg(std::integral_constant<int, 1024>{});
    }
    return 0;
}

// host restatement of ResetKalmanState / StepKalman4D
// (L/WaveSpecZZ_1.0.3-pla-kalman-fast.mq5:2015-2125), full 4x4 covariance
static void host_kalman(const double *x, int n, const double *kp, double *d) {
    const double q = fmax(0.05, kp[0]);
    const double Qp = fmax(1e-9, kp[1] * q), Qv = fmax(1e-9, kp[2] * q), Qa = fmax(1e-9, kp[3] * q),
                 Qj = fmax(1e-9, kp[4] * q), R = fmax(1e-9, kp[6]);
    double pos = x[0], vel = kp[11], acc = kp[12], jerk = kp[13];
    double P[4][4] = {{fmax(1e-9, kp[7]), 0, 0, 0}, {0, fmax(1e-9, kp[8]), 0, 0}, {0, 0, fmax(1e-9, kp[9]), 0},
                      {0, 0, 0, fmax(1e-9, kp[10])}};
    const double F[4][4] = {{1, 1, 0.5, 1.0 / 6.0}, {0, 1, 1, 0.5}, {0, 0, 1, 1}, {0, 0, 0, 1}};
    double ema = 0;
    bool ema_ready = false;
    for (int j = 0; j < n; ++j) {
        double x0p = pos + vel + 0.5 * acc + jerk / 6.0, x1p = vel + acc + 0.5 * jerk, x2p = acc + jerk, x3p = jerk;
        double A[4][4] = {}, Pp[4][4] = {};
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b)
                for (int k = 0; k < 4; ++k) A[a][b] += F[a][k] * P[k][b];
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b)
                for (int k = 0; k < 4; ++k) Pp[a][b] += A[a][k] * F[b][k];
        Pp[1][1] += P[1][2] + P[2][2] + 0.5 * (P[1][3] + P[2][3]);  // the reference's P11 (:2052)
        Pp[0][0] += Qp; Pp[1][1] += Qv; Pp[2][2] += Qa; Pp[3][3] += Qj;
        double y = x[j] - x0p, S = Pp[0][0] + R;
        if (kp[5] > 0) {
            double k = fmin(5.0, fabs(y) / sqrt(S)) * kp[5];
            Pp[0][0] += k * Qp; Pp[1][1] += k * Qv; Pp[2][2] += k * Qa; Pp[3][3] += k * Qj;
            S = Pp[0][0] + R;
        }
        if (kp[14] > 0) { double lim = kp[14] * sqrt(S); y = fmin(fmax(y, -lim), lim); }
        double K[4];
        for (int a = 0; a < 4; ++a) K[a] = Pp[a][0] / S;
        pos = x0p + K[0] * y; vel = x1p + K[1] * y; acc = x2p + K[2] * y; jerk = x3p + K[3] * y;
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b) P[a][b] = Pp[a][b] - K[a] * Pp[0][b];
        for (int a = 0; a < 4; ++a) P[a][a] = fmax(1e-12, P[a][a]);
        double trend = pos;
        if (kp[15] > 0) {
            const double al = 2.0 / (kp[15] + 1.0);
            if (!ema_ready) { ema = trend; ema_ready = true; }
            ema = al * trend + (1.0 - al) * ema;
            trend = ema;
        }
        d[j] = x[j] - trend;
    }
}

template <int FL, bool TWO, int WAVES, int SEG = 1>
void check_one(const char *name, const double *dx, double *dd, const std::vector<double> &ref, int64_t W, int64_t hop, int n,
               const double *kpa) {
    kcore::KP kp;
    memcpy(&kp, kpa, sizeof(kp));
    CK(hipMemset(dd, 0xff, (W + 300) * n * 8));  // NaN canary past the batch end as well
    launch<double, 16, FL, TWO, WAVES, false, SEG>(dx, dd, hop, W, n, kp, 0);
    CK(hipDeviceSynchronize());
    std::vector<double> h((W + 300) * n);
    CK(hipMemcpy(h.data(), dd, h.size() * 8, hipMemcpyDeviceToHost));
    double worst = 0;
    int64_t at = -1;
    for (int64_t i = 0; i < W * n; ++i) {
        const double e = fabs(h[i] - ref[i]);
        if (!(e <= worst)) { worst = e; at = i; }
    }
    int64_t touched = 0;  // stores past the batch end must be dropped
    for (int64_t i = W * n; i < (int64_t)h.size(); ++i) touched += h[i] == h[i];
    printf("%-40s max|d-ref| %.3e (window %lld step %lld)  writes past end: %lld\n", name, worst, (long long)(at / n),
           (long long)(at % n), (long long)touched);
}

// fp32 filter (and the packed update) against the same host restatement: relative to the residual scale
template <bool PK, int SEG = 1>
void check_f32(const char *name, const std::vector<double> &x, const std::vector<double> &ref, int64_t W, int64_t hop, int n) {
    kcore::KP kp;
    memcpy(&kp, kDefaults, sizeof(kp));
    std::vector<float> xf(x.begin(), x.end());
    float *dx, *dd;
    CK(hipMalloc(&dx, xf.size() * 4));
    CK(hipMalloc(&dd, W * n * 4));
    CK(hipMemcpy(dx, xf.data(), xf.size() * 4, hipMemcpyHostToDevice));
    launch<float, 32, 3, true, 4, PK, SEG>(dx, dd, hop, W, n, kp, 0);
    CK(hipDeviceSynchronize());
    std::vector<float> h(W * n);
    CK(hipMemcpy(h.data(), dd, W * n * 4, hipMemcpyDeviceToHost));
    double worst = 0, scale = 0;
    for (int64_t i = 0; i < W * n; ++i) {
        worst = fmax(worst, fabs((double)h[i] - ref[i]));
        scale = fmax(scale, fabs(ref[i]));
    }
    printf("%-40s max|d-ref| / max|ref| %.3e\n", name, worst / scale);
    CK(hipFree(dx));
    CK(hipFree(dd));
}

// per state component: max |exact - warm| and max |exact| over the windows of the last SEG = 2 launch
static void dump_dbg(const char *name, int64_t W) {
    std::vector<double> h(W * 28);
    CK(hipMemcpy(h.data(), g_dbg, h.size() * 8, hipMemcpyDeviceToHost));
    static const char *nm[14] = {"pos", "vel", "acc", "jerk", "p00", "p01", "p02", "p03", "p11", "p12", "p13", "p22", "p23", "p33"};
    int64_t same = 0;
    for (int64_t w = 0; w < W; ++w) {
        bool eq = true;
        for (int k = 0; k < 14; ++k) eq = eq && h[w * 28 + k] == h[w * 28 + 14 + k];
        same += eq;
    }
    printf("    %s: %lld of %lld windows bit-identical after the warm-up\n", name, (long long)same, (long long)W);
    printf("    %s state |exact - warm| / |exact|:", name);
    for (int k = 0; k < 14; ++k) {
        double md = 0, mv = 0;
        for (int64_t w = 0; w < W; ++w) {
            md = fmax(md, fabs(h[w * 28 + k] - h[w * 28 + 14 + k]));
            mv = fmax(mv, fabs(h[w * 28 + k]));
        }
        printf(" %s %.2e/%.2e", nm[k], md, mv);
    }
    printf("\n");
}

int check_main(int n) {
    const int64_t W = 100, hop = 37;
    const int64_t len = (W - 1) * hop + n;
    std::vector<double> x(len);
    double v = 1.1;
    for (int64_t i = 0; i < len; ++i) {
        v += 1e-4 * (((i * 2654435761u) % 1000) / 500.0 - 1.0);
        x[i] = v + 0.002 * sin(0.1256 * (double)i);
    }
    double *dx, *dd;
    CK(hipMalloc(&dx, len * 8));
    CK(hipMalloc(&dd, (W + 300) * n * 8));
    CK(hipMemcpy(dx, x.data(), len * 8, hipMemcpyHostToDevice));
    std::vector<double> ref(W * n);
    for (int64_t w = 0; w < W; ++w) host_kalman(&x[w * hop], n, kDefaults, &ref[w * n]);
    check_one<kcore::kKfRuntime, false, 1>("1-wave runtime expanded", dx, dd, ref, W, hop, n, kDefaults);
    check_one<kcore::kKfRuntime, true, 1>("1-wave runtime two-stage", dx, dd, ref, W, hop, n, kDefaults);
    check_one<3, true, 1>("1-wave static two-stage", dx, dd, ref, W, hop, n, kDefaults);
    check_one<3, true, 4>("4-wave static two-stage", dx, dd, ref, W, hop, n, kDefaults);
    if (n >= 1024) {
        CK(hipMemset(g_fallbacks, 0, 4));
        check_one<3, true, 4, 2>("2 segments static two-stage", dx, dd, ref, W, hop, n, kDefaults);
        unsigned fb = 0;
        CK(hipMemcpy(&fb, g_fallbacks, 4, hipMemcpyDeviceToHost));
        printf("    2-segment fallbacks (f64): %u of %lld waves\n", fb, (long long)((W + 31) / 32));
        dump_dbg("f64", W);
    }
    double ema[16];
    memcpy(ema, kDefaults, sizeof(ema));
    ema[15] = 12.0;
    for (int64_t w = 0; w < W; ++w) host_kalman(&x[w * hop], n, ema, &ref[w * n]);
    check_one<kcore::kKfRuntime, true, 4>("4-wave runtime two-stage, EMA 12", dx, dd, ref, W, hop, n, ema);
    std::vector<double> xr(x.size());  // float-rounded prices for the fp32 filters
    for (size_t i = 0; i < x.size(); ++i) xr[i] = (double)(float)x[i];
    for (int64_t w = 0; w < W; ++w) host_kalman(&xr[w * hop], n, kDefaults, &ref[w * n]);
    check_f32<false>("f32 4-wave static two-stage", xr, ref, W, hop, n);
    check_f32<true>("f32 4-wave static packed update", xr, ref, W, hop, n);
    if (kcore::pk2_fits(n)) {  // packed segments, against the fp64 host filter and the sequential fp32 kernel
        kcore::KP kp;
        memcpy(&kp, kDefaults, sizeof(kp));
        float *dx32, *dd32, *dq32;
        CK(hipMalloc(&dx32, xr.size() * 4));
        CK(hipMalloc(&dd32, W * n * 4));
        CK(hipMalloc(&dq32, W * n * 4));
        // spikes: a value of 1000 added on the cold-start sample of the given segment starts (every third window)
        auto check_pk = [&](const char *name, int segs, std::vector<int> spikes) {
            std::vector<double> xs(xr);
            for (int64_t w = 0; w < W; w += 3)
                for (int at : spikes) xs[w * hop + at] += 1000.0;
            for (auto &v : xs) v = (double)(float)v;
            std::vector<double> refs(W * n);
            for (int64_t w = 0; w < W; ++w) host_kalman(&xs[w * hop], n, kDefaults, &refs[w * n]);
            std::vector<float> xsf(xs.begin(), xs.end());
            CK(hipMemcpy(dx32, xsf.data(), xsf.size() * 4, hipMemcpyHostToDevice));
            CK(hipMemset(g_fallbacks, 0, 4));
            if (segs == 4) launch_pk4<kcore::kPk2Warm>(dx32, dd32, hop, W, n, kp, 0);
            else if (segs == 5) launch_pk2<1, kcore::kPk2Warm, true, 1>(dx32, dd32, hop, W, n, kp, 0);
            else if (segs == 6) launch_pk2<1, kcore::kPk2Warm, true, 2>(dx32, dd32, hop, W, n, kp, 0);
            else if (segs == 3) launch_pk2<4, kcore::kPk2Warm, false>(dx32, dd32, hop, W, n, kp, 0);
            else launch_pk2<1, kcore::kPk2Warm>(dx32, dd32, hop, W, n, kp, 0);
            unsigned fb = 0;
            if (segs == 6) {  // the forced guard re-runs in the original basis: bit-identical to that kernel?
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(&fb, g_fallbacks, 4, hipMemcpyDeviceToHost));
                launch_pk2<1, kcore::kPk2Warm>(dx32, dq32, hop, W, n, kp, 0);
                CK(hipDeviceSynchronize());
                std::vector<float> a(W * n), b(W * n);
                CK(hipMemcpy(a.data(), dd32, W * n * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(b.data(), dq32, W * n * 4, hipMemcpyDeviceToHost));
                printf("%-36s bit-identical to the original-basis kernel: %s\n", name,
                       memcmp(a.data(), b.data(), a.size() * 4) == 0 ? "yes" : "NO");
            }
            launch<float, 32, 3, true, 4, true>(dx32, dq32, hop, W, n, kp, 0);
            CK(hipDeviceSynchronize());
            std::vector<float> h(W * n), q(W * n);
            CK(hipMemcpy(h.data(), dd32, W * n * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(q.data(), dq32, W * n * 4, hipMemcpyDeviceToHost));
            if (segs != 6) CK(hipMemcpy(&fb, g_fallbacks, 4, hipMemcpyDeviceToHost));
            double worst = 0, scale = 0, wseq = 0, wseqv = 0;
            int64_t same = 0;
            for (int64_t i = 0; i < W * n; ++i) {
                worst = fmax(worst, fabs((double)h[i] - refs[i]));
                scale = fmax(scale, fabs(refs[i]));
                wseq = fmax(wseq, fabs((double)h[i] - (double)q[i]));
                wseqv = fmax(wseqv, fabs((double)q[i] - refs[i]));
                same += h[i] == q[i];
            }
            printf("%-36s max|d-ref|/max|ref| %.3e (sequential fp32 %.3e)  vs sequential: %.3e, %lld of %lld identical; fallback re-runs %u (+ %u guard)\n",
                   name, worst / scale, wseqv / scale, wseq / scale, (long long)same, (long long)(W * n), fb & 0xffffu, fb >> 16);
        };
        const int L0 = (n + kcore::kPk2Warm) / 2, WU = kcore::kPk2Warm;
        check_pk("f32 packed 2 segments", 2, {});
        check_pk("f32 packed 2 segments, spikes", 2, {L0 - WU});
        check_pk("f32 packed 2 segments, Newton basis", 5, {});
        check_pk("f32 packed 2 segments, Newton basis, spikes", 5, {L0 - WU});
        check_pk("f32 packed 2 segments, Newton basis, guard forced", 6, {});
        check_pk("f32 packed 2 segments, Newton basis, guard forced, spikes", 6, {L0 - WU});
        check_pk("f32 packed 2 segments unrotated", 3, {});
        check_pk("f32 packed 2 segments unrotated, spikes", 3, {L0 - WU});
        if (kcore::pk4_fits(n)) {
            const int S = (n + 3 * WU) / 4 - WU;
            check_pk("f32 packed 4 segments", 4, {});
            check_pk("f32 packed 4 segments, spikes at 1", 4, {S});
            check_pk("f32 packed 4 segments, spikes at 2", 4, {2 * S});
            check_pk("f32 packed 4 segments, spikes at 3", 4, {3 * S});
            check_pk("f32 packed 4 segments, spikes at 1,2,3", 4, {S, 2 * S, 3 * S});
        }
        CK(hipFree(dx32));
        CK(hipFree(dd32));
        CK(hipFree(dq32));
    }
    if (n >= 1024) {
        CK(hipMemset(g_fallbacks, 0, 4));
        check_f32<true, 2>("f32 2 segments packed update", xr, ref, W, hop, n);
        unsigned fb = 0;
        CK(hipMemcpy(&fb, g_fallbacks, 4, hipMemcpyDeviceToHost));
        printf("    2-segment fallbacks (f32): %u of %lld waves\n", fb, (long long)((W + 31) / 32));
        dump_dbg("f32", W);
    }
    return 0;
}

int main(int argc, char **argv) {
    const std::string mode = argc > 1 ? argv[1] : "time";
    CK(hipMalloc(&g_fallbacks, 4));
    CK(hipMemset(g_fallbacks, 0, 4));
    CK(hipMalloc(&g_dbg, 65536 * 28 * 8));
    if (mode == "check") return check_main(argc > 2 ? atoi(argv[2]) : 256);
    if (mode == "occ") return occ_main(argc > 2 ? atoi(argv[2]) : 10);
    if (mode == "ab") return time_main(argc > 2 ? atoi(argv[2]) : 10, true);
    return time_main(argc > 2 ? atoi(argv[2]) : 10, false);
}
