// mtbridge.cpp -- C ABI of libmtbridge.so (include/mtbridge.h): the Linux /
// MI355X drop-in for `mt-bridge.dll` (reference Include/imports.mqh:4-20).
//
// Layers:
//   * thread-local last error          (gpu_get_last_error_w, 1.1.0:742-745)
//   * caching device / pinned-host allocator (per device, size buckets)
//   * per-device twiddle + window tables (built once, fp64 exact on host)
//   * enqueue(): the device hot path = [Kalman pre-pass] + spectrum kernel
//   * Batch: H2D from pinned staging -> enqueue -> D2H, one part per GPU
//     (windows sharded in contiguous ranges, no collective: SURVEY 8e)
//   * session (gpu_init/gpu_shutdown), job table (submit/try_get/free),
//     device-resident plans (wsp_plan_*).
// Every entry point is thread-safe; the product path has no CPU fallback
// (CHANGELOG.md:5,15 "sem fallback CPU"): without a GPU it fails with
// MTB_BACKEND_UNAVAILABLE.
#include "../../include/mtbridge.h"
#include "wsp_internal.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

using namespace wsp;

// ------------------------------------------------------------- last error
// initial-exec: the 32-B string sits in the static TLS surplus even when the library is dlopen()ed, so no
// __tls_get_addr allocation runs on a caller's first error (ThreadSanitizer's interceptor of that path
// intermittently aborted the tests/hostsan stress driver with "unable to unmap")
thread_local std::string t_last_error __attribute__((tls_model("initial-exec")));

void set_error(const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    t_last_error = buf;
}

#define HIP_OR(expr, code)                                                                          \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess) {                                                                     \
            set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
            return (code);                                                                          \
        }                                                                                           \
    } while (0)

int device_count() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// ------------------------------------------------------ caching allocator
// Size-bucketed free lists (power-of-two buckets >= 64 KiB).  Device
// buffers per device; pinned host buffers shared.  Keeps hipMalloc /
// hipHostMalloc out of the per-bar path (gpu_fft_real_forward runs every
// bar, 1.1.0:1249).
size_t bucket_bytes(size_t n) {
    size_t b = 64 * 1024;
    while (b < n) b <<= 1;
    return b;
}

struct Pool {
    std::mutex mu;
    std::map<std::pair<int, size_t>, std::vector<void *>> free_dev;  // (device, bytes)
    std::map<size_t, std::vector<void *>> free_host;
    std::map<int, std::vector<hipEvent_t>> free_events;              // per device, timing disabled
};
Pool &pool() {
    static Pool *p = new Pool();  // intentionally leaked: no teardown after the HIP runtime
    return *p;
}

void *dev_alloc(int dev, size_t bytes) {
    const size_t b = bucket_bytes(bytes);
    {
        std::lock_guard<std::mutex> lk(pool().mu);
        auto &v = pool().free_dev[{dev, b}];
        if (!v.empty()) {
            void *p = v.back();
            v.pop_back();
            return p;
        }
    }
    void *p = nullptr;
    if (hipSetDevice(dev) != hipSuccess || hipMalloc(&p, b) != hipSuccess) {
        set_error("hipMalloc(%zu bytes) failed on device %d", b, dev);
        return nullptr;
    }
    return p;
}
void dev_free(int dev, void *p, size_t bytes) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(pool().mu);
    pool().free_dev[{dev, bucket_bytes(bytes)}].push_back(p);
}
void *host_alloc(size_t bytes) {
    const size_t b = bucket_bytes(bytes);
    {
        std::lock_guard<std::mutex> lk(pool().mu);
        auto &v = pool().free_host[b];
        if (!v.empty()) {
            void *p = v.back();
            v.pop_back();
            return p;
        }
    }
    void *p = nullptr;
    if (hipHostMalloc(&p, b, hipHostMallocDefault) != hipSuccess) {
        set_error("hipHostMalloc(%zu bytes) failed", b);
        return nullptr;
    }
    return p;
}
void host_free(void *p, size_t bytes) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(pool().mu);
    pool().free_host[bucket_bytes(bytes)].push_back(p);
}
// Completion events of batch parts: recycled, so that a per-bar call creates
// none (hipEventCreate costs a driver round trip).
hipEvent_t event_alloc(int dev) {
    {
        std::lock_guard<std::mutex> lk(pool().mu);
        auto &v = pool().free_events[dev];
        if (!v.empty()) {
            hipEvent_t e = v.back();
            v.pop_back();
            return e;
        }
    }
    hipEvent_t e = nullptr;
    if (hipSetDevice(dev) != hipSuccess || hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
        set_error("hipEventCreateWithFlags failed on device %d", dev);
        return nullptr;
    }
    return e;
}
void event_free(int dev, hipEvent_t e) {
    if (!e) return;
    std::lock_guard<std::mutex> lk(pool().mu);
    pool().free_events[dev].push_back(e);
}
void pool_release_all() {
    std::lock_guard<std::mutex> lk(pool().mu);
    for (auto &kv : pool().free_dev) {
        (void)hipSetDevice(kv.first.first);
        for (void *p : kv.second) (void)hipFree(p);
    }
    pool().free_dev.clear();
    for (auto &kv : pool().free_host)
        for (void *p : kv.second) (void)hipHostFree(p);
    pool().free_host.clear();
    for (auto &kv : pool().free_events) {
        (void)hipSetDevice(kv.first);
        for (hipEvent_t e : kv.second) (void)hipEventDestroy(e);
    }
    pool().free_events.clear();
}

// ----------------------------------------------------------------- tables
// W_N^k = exp(-2 pi i k/N), k < N, rounded once from long double.  (Window
// coefficients are generated in the kernel by a rotation recurrence.)
struct Tables {
    void *tw = nullptr;
};
std::mutex g_tables_mu;
std::map<std::tuple<int, int, bool>, Tables> *g_tables = new std::map<std::tuple<int, int, bool>, Tables>();

int get_tables(int dev, int log2n, bool f32, Tables *out) {
    std::lock_guard<std::mutex> lk(g_tables_mu);
    auto key = std::make_tuple(dev, log2n, f32);
    auto it = g_tables->find(key);
    if (it != g_tables->end()) {
        *out = it->second;
        return MTB_OK;
    }
    const int n = 1 << log2n;
    const size_t es = f32 ? sizeof(float) : sizeof(double);
    std::vector<char> tw((size_t)n * 2 * es);
    for (int k = 0; k < n; ++k) {  // full period: table-loaded twiddle powers index up to N-1
        const long double ang = -2.0L * 3.141592653589793238462643383279502884L * (long double)k / (long double)n;
        const long double c = cosl(ang), s = sinl(ang);
        if (f32) {
            ((float *)tw.data())[2 * k] = (float)c;
            ((float *)tw.data())[2 * k + 1] = (float)s;
        } else {
            ((double *)tw.data())[2 * k] = (double)c;
            ((double *)tw.data())[2 * k + 1] = (double)s;
        }
    }
    Tables t;
    HIP_OR(hipSetDevice(dev), MTB_BACKEND_UNAVAILABLE);
    HIP_OR(hipMalloc(&t.tw, tw.size()), MTB_NO_MEM);
    HIP_OR(hipMemcpy(t.tw, tw.data(), tw.size(), hipMemcpyHostToDevice), MTB_INTERNAL_ERROR);
    (*g_tables)[key] = t;
    *out = t;
    return MTB_OK;
}

// Window pairs of the fp32 two-segment Kalman filter per (device, N, window) (kalman_folds_window): float pairs
// {h(j), h(j + seg_off)}, j < L0, of the reference's symmetric windows (L/WaveSpecZZ_1.0.2.mq5:884-914, denominator
// N - 1), each value from long double rounded once.
std::mutex g_wpairs_mu;
std::map<std::tuple<int, int, int>, void *> *g_wpairs = new std::map<std::tuple<int, int, int>, void *>();

long double window_value_ld(int window, int i, int n) {
    const long double pi = 3.141592653589793238462643383279502884L, th = 2.0L * pi * (long double)i / (long double)(n - 1);
    switch (window) {
    case MTB_WINDOW_HANN: return 0.5L * (1.0L - cosl(th));
    case MTB_WINDOW_HAMMING: return 0.54L - 0.46L * cosl(th);
    case MTB_WINDOW_BLACKMAN: return 0.42L - 0.5L * cosl(th) + 0.08L * cosl(2.0L * th);
    case MTB_WINDOW_BARTLETT: return 1.0L - fabsl((2.0L * (long double)i - (long double)n + 1.0L) / (long double)(n - 1));
    default: return 1.0L;
    }
}

int get_window_pairs(int dev, int n, int window, const float **out) {
    *out = nullptr;
    if (window == MTB_WINDOW_NONE) return MTB_OK;
    std::lock_guard<std::mutex> lk(g_wpairs_mu);
    auto key = std::make_tuple(dev, n, window);
    auto it = g_wpairs->find(key);
    if (it != g_wpairs->end()) {
        *out = static_cast<const float *>(it->second);
        return MTB_OK;
    }
    int l0 = 0, seg_off = 0;
    kalman_pair_geometry(n, &l0, &seg_off);
    std::vector<float> h((size_t)l0 * 2);
    for (int j = 0; j < l0; ++j) {
        h[2 * j] = (float)window_value_ld(window, j, n);
        h[2 * j + 1] = j + seg_off < n ? (float)window_value_ld(window, j + seg_off, n) : 0.0f;
    }
    void *d = nullptr;
    HIP_OR(hipSetDevice(dev), MTB_BACKEND_UNAVAILABLE);
    HIP_OR(hipMalloc(&d, h.size() * sizeof(float)), MTB_NO_MEM);
    HIP_OR(hipMemcpy(d, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice), MTB_INTERNAL_ERROR);
    (*g_wpairs)[key] = d;
    *out = static_cast<const float *>(d);
    return MTB_OK;
}

// Sliding-DFT tables per (device, N, window) (sliding_dft.hip), double complex, long double
// arithmetic rounded once: [nf][N/2] omega_f(k) = e^{2 pi j (k/N + m_f/(N-1))}, m_f = 0, +1, -1, +2, -2;
// [N/2] H_k = DFT_k of the window; [(nf-1)/2][N] e^{-j m th i}, th = 2 pi/(N-1).
struct WinCoef {
    double a0 = 1.0, a1 = 0.0, a2 = 0.0;
    int nf = 1;  // complex exponentials in the window (0 = not a cosine sum: Bartlett)
};
// L/WaveSpecZZ_1.0.2.mq5:884-922 as a0 + a1 cos(th i) + a2 cos(2 th i)
WinCoef window_coef(int window) {
    WinCoef w;
    switch (window) {
    case MTB_WINDOW_HANN: w.a0 = 0.5, w.a1 = -0.5, w.nf = 3; break;
    case MTB_WINDOW_HAMMING: w.a0 = 0.54, w.a1 = -0.46, w.nf = 3; break;
    case MTB_WINDOW_BLACKMAN: w.a0 = 0.42, w.a1 = -0.5, w.a2 = 0.08, w.nf = 5; break;
    case MTB_WINDOW_BARTLETT: w.nf = 0; break;
    default: break;
    }
    return w;
}
std::mutex g_slide_mu;
std::map<std::tuple<int, int, int>, void *> *g_slide_tables = new std::map<std::tuple<int, int, int>, void *>();

int get_slide_table(int dev, int log2n, int window, void **out) {
    std::lock_guard<std::mutex> lk(g_slide_mu);
    auto key = std::make_tuple(dev, log2n, window);
    auto it = g_slide_tables->find(key);
    if (it != g_slide_tables->end()) {
        *out = it->second;
        return MTB_OK;
    }
    typedef long double ld;
    const ld pi = 3.141592653589793238462643383279502884L;
    const WinCoef wc = window_coef(window);
    const int n = 1 << log2n, m2 = n / 2, nf = wc.nf, nm = (nf - 1) / 2;
    const int mf[5] = {0, 1, -1, 2, -2};
    const ld sc[5] = {(ld)wc.a0, (ld)wc.a1 / 2, (ld)wc.a1 / 2, (ld)wc.a2 / 2, (ld)wc.a2 / 2};
    std::vector<double> tab((size_t)2 * ((size_t)(nf + 1) * m2 + (size_t)nm * n));
    double *om = tab.data(), *hw = om + (size_t)2 * nf * m2, *md = hw + (size_t)2 * m2;
    for (int f = 0; f < nf; ++f)
        for (int k = 0; k < m2; ++k) {
            const ld ang = 2 * pi * ((ld)k / n + (ld)mf[f] / (n - 1));
            om[2 * ((size_t)f * m2 + k)] = (double)cosl(ang);
            om[2 * ((size_t)f * m2 + k) + 1] = (double)sinl(ang);
        }
    // H_k = sum_f s_f G(k/N + m_f/(N-1)), G(g) = sum_{i<N} e^{-2 pi j g i}
    //     = e^{-j pi g (N-1)} sin(pi g N)/sin(pi g), with sin(pi g N) = (-1)^(k+m) sin(pi m/(N-1))
    for (int k = 0; k < m2; ++k) {
        ld hr = 0, hi = 0;
        for (int f = 0; f < nf; ++f) {
            if (sc[f] == 0) continue;
            const ld g = (ld)k / n + (ld)mf[f] / (n - 1);
            ld gr, gi;
            if (k == 0 && mf[f] == 0) {
                gr = n, gi = 0;
            } else {
                const ld num = (((k + mf[f]) & 1) ? -1 : 1) * sinl(pi * (ld)mf[f] / (n - 1));
                const ld mag = num / sinl(pi * g);
                const ld ph = -pi * ((ld)k * (n - 1) / n + (ld)mf[f]);
                gr = mag * cosl(ph), gi = mag * sinl(ph);
            }
            hr += sc[f] * gr, hi += sc[f] * gi;
        }
        hw[2 * k] = (double)hr, hw[2 * k + 1] = (double)hi;
    }
    for (int m = 1; m <= nm; ++m)
        for (int i = 0; i < n; ++i) {
            const ld ang = -2 * pi * (ld)m * (ld)i / (n - 1);
            md[2 * ((size_t)(m - 1) * n + i)] = (double)cosl(ang);
            md[2 * ((size_t)(m - 1) * n + i) + 1] = (double)sinl(ang);
        }
    void *d = nullptr;
    HIP_OR(hipSetDevice(dev), MTB_BACKEND_UNAVAILABLE);
    HIP_OR(hipMalloc(&d, tab.size() * sizeof(double)), MTB_NO_MEM);
    HIP_OR(hipMemcpy(d, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice), MTB_INTERNAL_ERROR);
    (*g_slide_tables)[key] = d;
    *out = d;
    return MTB_OK;
}

// Longest sliding-DFT segment a caller may ask for: a tracker's rounding grows linearly with the
// number of slides (sliding_dft.hip), and parity is tested up to this length
// (tests/test_gpu_slide.py::test_slide_vs_fft_large_segments).
constexpr int64_t kSlideMaxSegment = 2048;

// ----------------------------------------------------------------- config
enum Op : int { kOpSpectrum = 0, kOpInverse = 1 };
struct Config {
    int op = kOpSpectrum;  // kOpInverse: rows of packed spectra -> rows of samples
    int n = 0, log2n = 0;
    int64_t hop = 0, n_windows = 0;
    int detrend = 0, window = 0, trend_period = 0, output = 0;
    int topk = 0, kmin = 0, kmax = -1;  // MTB_OUT_TOPK / MTB_OUT_TOPK_PHASE
    int algo = MTB_ALGO_AUTO;           // wsp_plan_set_algorithm
    int64_t slide_seg = 0;              // windows per sliding-DFT workgroup, 0 = auto (wsp_plan_set_slide_segment)
    int seed_chain = 0;                 // top-k segments per seed workgroup, 0 = auto (wsp_plan_set_seed_chain)
    long long *trace = nullptr;         // diagnostic timeline of the hop = 1 top-k kernels (wsp_plan_set_trace)
    int64_t trace_cap = 0;
    int variant = 0;                    // kernel form (wsp_plan_set_variant: ablations), 0 = the library's choice
    unsigned char *scan_flags = nullptr;  // wsp_plan_set_scan_flags: per-window path of the probe-threshold top-k scan
    int64_t chunk = 0;                  // N > 16384 two-pass path: windows per chunk, 0 = large_chunk (wsp_plan_set_chunk)
    int grid = 0;                       // workgroups of the FFT-kernel / inverse launch, 0 = the library's (wsp_plan_set_grid)
    int64_t chunk_windows() const;
    bool f32 = false;
    size_t elem() const { return f32 ? sizeof(float) : sizeof(double); }
    int64_t record() const {
        if (op == kOpInverse || output == MTB_OUT_PACKED) return n;
        switch (output) {
        case MTB_OUT_TOPK: return 4 * topk;
        case MTB_OUT_TOPK_PHASE: return 6 * topk;
        case MTB_OUT_PHASE: return 3 * (n / 2);
        default: return n / 2;
        }
    }
    int64_t series_elems() const { return (n_windows - 1) * hop + n; }
    int64_t unique_input_elems() const { return hop >= n ? n_windows * (int64_t)n : series_elems(); }
};

int64_t Config::chunk_windows() const { return chunk > 0 ? chunk : large_chunk(log2n, f32); }

int ilog2_exact(int n) {
    if (n <= 0 || (n & (n - 1))) return -1;
    int l = 0;
    while ((1 << l) < n) ++l;
    return l;
}

// Device workspace of one launch: [detrended windows][per-window means][chunk column results], or the
// segment seeds of a hop = 1 top-k launch by the sliding DFT (its only workspace)
struct WsLayout {
    size_t det = 0, means = 0, y = 0, total = 0;
};
size_t align256(size_t b) { return (b + 255) & ~size_t(255); }
bool use_slide_topk(const Config &c);
// Windows per top-k segment: whole rounds of resident one-wave workgroups (the default probe scan runs 4 per
// SIMD = 16 per CU) at <= 256 windows each -- C4 (1,048,576 windows): one round of 4096 segments of 256,
// 0.371-0.374 ms against 0.389 for 128-window segments (two rounds) and 0.41 / 0.50 for 192 / 384
// (1.33 rounds / a quarter of the slots idle; profiles/r03/s2/topk_seg.log).  At least 32 windows (below).
// CUs of device `dev`, looked up once per device (the segment policy of a plan follows its own GPU, not the
// calling thread's current one)
int cu_count(int dev) {
    static std::atomic<int> cache[64];
    if (dev < 0 || dev >= 64) return 256;
    int cus = cache[dev].load(std::memory_order_relaxed);
    if (cus > 0) return cus;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cache[dev].store(cus, std::memory_order_relaxed);
    return cus;
}
// Below one round of 64-window segments (a strong-scaled shard: 1/8 of C4 is 131072 windows) the segments go down to
// 32 windows, so the scan still fills the resident slots (4 waves per SIMD instead of 2), and their seeds come in
// chains (slide_topk_chain): 1/8 C4 top-8 0.0957 ms at 64-window segments, 0.0912 at 32 with one FFT seed each,
// 0.0773-0.0802 at 32 in chains of 4 (r05k, r05o; chains of 3 / 5 / 6 0.082-0.088 / 0.079-0.082 / 0.085).
int64_t slide_topk_seg(const Config &c, int dev) {
    if (c.slide_seg > 0) return c.slide_seg;
    const int64_t res = (int64_t)16 * cu_count(dev);
    const int64_t rounds = (c.n_windows + res * 256 - 1) / (res * 256);
    const int64_t seg = (c.n_windows + res * rounds - 1) / (res * rounds);
    return seg < 64 ? std::max<int64_t>(32, seg) : seg;
}
// segments per seed workgroup when the plan does not set it (wsp_plan_set_seed_chain): chains of ~128 windows at
// segments of <= 32 (variant 6, the round-5 ablation, chains of <= 256 windows at any length)
int slide_topk_chain(const Config &c, int64_t seg) {
    const int cap = (int)std::min<int64_t>(16, 1 + 256 / seg);
    if (c.seed_chain > 0) return std::min(cap, c.seed_chain);
    if (c.variant == 6) return cap;
    return seg <= 32 ? std::min<int>(cap, (int)((128 + seg - 1) / seg)) : 1;
}
WsLayout ws_layout(const Config &c, int dev) {
    WsLayout L;
    if (use_slide_topk(c)) {
        const int nf = window_coef(c.window).nf;
        const int64_t seg = slide_topk_seg(c, dev);
        const int64_t nseg = (c.n_windows + seg - 1) / seg;
        L.total = (size_t)nseg * (size_t)slide_topk_seed_stride(nf, c.kmax - c.kmin + 1) * 2 * sizeof(double);
        return L;
    }
    const size_t es = c.elem();
    const bool large = c.op == kOpSpectrum && c.log2n > kMaxLog2N;
    size_t det = 0, means = 0, y = 0;
    if (c.op == kOpSpectrum && (c.detrend == MTB_DETREND_KALMAN || (large && c.detrend == MTB_DETREND_IIR)))
        det = (size_t)(c.n_windows * c.n) * es;
    if (large && c.detrend == MTB_DETREND_MEAN) means = (size_t)c.n_windows * sizeof(double);
    if (large) y = (size_t)std::min<int64_t>(c.n_windows, c.chunk_windows()) * (size_t)(c.n / 2) * 2 * es;
    L.det = 0;
    L.means = align256(det);
    L.y = align256(L.means + means);
    L.total = y ? L.y + y : (means ? L.means + means : det);
    return L;
}

int config_set_topk(Config *c, int top_k, double min_period, double max_period);

int make_config(int window_len, int64_t hop, int64_t n_windows, int detrend, int window, int trend_period,
                int precision, int output, Config *c) {
    const int l = ilog2_exact(window_len);
    if (l < kMinLog2N || l > kMaxLog2NLarge) {
        set_error("window_len=%d: must be a power of two in [%d, %d]", window_len, 1 << kMinLog2N, 1 << kMaxLog2NLarge);
        return MTB_BAD_ARGS;
    }
    if (l > kMaxLog2N && output != MTB_OUT_POWER && output != MTB_OUT_PACKED) {
        set_error("window_len=%d: windows above %d support the power and packed outputs", window_len, 1 << kMaxLog2N);
        return MTB_BAD_ARGS;
    }
    if (hop < 1 || n_windows < 1) {
        set_error("hop=%lld n_windows=%lld: both must be >= 1", (long long)hop, (long long)n_windows);
        return MTB_BAD_ARGS;
    }
    if (detrend < MTB_DETREND_NONE || detrend > MTB_DETREND_KALMAN || window < MTB_WINDOW_NONE ||
        window > MTB_WINDOW_BARTLETT || (precision != MTB_PREC_F64 && precision != MTB_PREC_F32) ||
        output < MTB_OUT_POWER || output > MTB_OUT_TOPK_PHASE) {
        set_error("bad mode: detrend=%d window=%d precision=%d output=%d", detrend, window, precision, output);
        return MTB_BAD_ARGS;
    }
    if ((output == MTB_OUT_PHASE || output == MTB_OUT_TOPK_PHASE) && precision != MTB_PREC_F64) {
        set_error("output=%d (phase) is computed in fp64 only", output);
        return MTB_BAD_ARGS;
    }
    // the Kalman pre-pass addresses a 64-window tile with 32-bit offsets (kalman_core.h)
    if (detrend == MTB_DETREND_KALMAN &&
        (64 * hop + window_len) * (precision == MTB_PREC_F32 ? 4 : 8) >= (int64_t(1) << 31)) {
        set_error("hop=%lld: the Kalman detrend needs 64 * hop samples within 2 GiB", (long long)hop);
        return MTB_BAD_ARGS;
    }
    c->n = window_len;
    c->log2n = l;
    c->hop = hop;
    c->n_windows = n_windows;
    // InpTrendPeriod <= 0 skips the trend filter (L/WaveSpecZZ_1.0.3-pla-batch.mq5:3256,3279)
    c->detrend = (detrend == MTB_DETREND_IIR && trend_period <= 0) ? MTB_DETREND_NONE : detrend;
    c->window = window;
    c->trend_period = trend_period;
    c->output = output;
    c->f32 = precision == MTB_PREC_F32;
    // MTB_OUT_TOPK through the generic entry points: the reference's own scan
    // parameters (top 8, InpMinPeriod 18 / InpMaxPeriod 200, 1.1.0:22-23)
    if (output == MTB_OUT_TOPK || output == MTB_OUT_TOPK_PHASE) return config_set_topk(c, 8, 18.0, 200.0);
    return MTB_OK;
}

// Top-k range of L/WaveSpecZZ_1.0.3-pla-kalman-fast-gpuopt-nodetrend.mq5:539-541.
int config_set_topk(Config *c, int top_k, double min_period, double max_period) {
    if (top_k < 1 || top_k > 64 || !(min_period > 0.0) || !(max_period > 0.0)) {
        set_error("top_k=%d min_period=%g max_period=%g: need 1 <= top_k <= 64 and positive periods", top_k,
                  min_period, max_period);
        return MTB_BAD_ARGS;
    }
    if (c->log2n > kMaxLog2N) {
        set_error("window_len=%d: the top-k scan covers windows up to %d", c->n, 1 << kMaxLog2N);
        return MTB_BAD_ARGS;
    }
    if (c->output != MTB_OUT_TOPK_PHASE) c->output = MTB_OUT_TOPK;
    c->topk = top_k;
    c->kmin = (int)ceil((double)c->n / max_period);
    c->kmax = (int)floor((double)c->n / min_period);
    if (c->kmax >= c->n / 2) c->kmax = c->n / 2 - 1;
    if (c->kmin < 0) c->kmin = 0;
    return MTB_OK;
}

// Kalman parameters (process-wide), defaults of kalman-fast.mq5:886-901.
std::mutex g_kalman_mu;
double g_kalman[16] = {1.0, 0.01, 0.003, 0.0008, 0.0002, 0.8, 1.0, 16.0, 9.0, 4.0, 1.0, 0.0, 0.0, 0.0, 6.0, 0.0};

// hop = 1 power batches by the seeded sliding DFT (sliding_dft.hip) instead of an FFT per window:
// the windows' trackers slide by one sample exactly, ~2.5x less fp64 work per window.
bool slide_eligible(const Config &c) {
    const int nf = window_coef(c.window).nf;
    return c.op == kOpSpectrum && c.hop == 1 && c.output == MTB_OUT_POWER && c.log2n >= kSlideMinLog2N &&
           c.log2n <= kSlideMaxLog2N && (c.detrend == MTB_DETREND_NONE || c.detrend == MTB_DETREND_MEAN) &&
           nf > 0 && !(nf == 5 && c.log2n == kSlideMaxLog2N);  // Blackman at N = 8192 spills at 1024 threads
}
bool use_slide(const Config &c) {
    if (c.algo == MTB_ALGO_FFT || !slide_eligible(c)) return false;
    return c.algo == MTB_ALGO_SLIDE || c.n_windows >= 256;
}
// hop = 1 top-k records (MTB_OUT_TOPK, fp64) by the sliding DFT: only the band's bins are tracked (span <= 512)
bool slide_topk_eligible(const Config &c) {
    const int nf = window_coef(c.window).nf;
    const int span = c.kmax - c.kmin + 1;
    return c.op == kOpSpectrum && c.hop == 1 && c.output == MTB_OUT_TOPK && !c.f32 && c.log2n >= kSlideMinLog2N &&
           c.log2n <= kSlideMaxLog2N && (c.detrend == MTB_DETREND_NONE || c.detrend == MTB_DETREND_MEAN) && nf > 0 &&
           span >= 1 && span <= kSlideTopkMaxSpan;
}
bool use_slide_topk(const Config &c) {
    if (c.algo == MTB_ALGO_FFT || !slide_topk_eligible(c)) return false;
    return c.algo == MTB_ALGO_SLIDE || c.n_windows >= 256;
}

// Launch constants of the sliding DFT for a configuration (tables on `dev`, window coefficients,
// rotations); series / out / n_windows are the caller's.
int slide_args(int dev, const Config &c, SlideArgs *A) {
    Tables t64;
    void *stab = nullptr;
    int st;
    if ((st = get_tables(dev, c.log2n, false, &t64)) != MTB_OK) return st;
    if ((st = get_slide_table(dev, c.log2n, c.window, &stab)) != MTB_OK) return st;
    HIP_OR(hipSetDevice(dev), MTB_BACKEND_UNAVAILABLE);
    const WinCoef wc = window_coef(c.window);
    const long double th = 2.0L * 3.141592653589793238462643383279502884L / (long double)(c.n - 1);
    A->twiddle = t64.tw;
    A->omega = stab;
    A->seg = c.slide_seg;
    A->log2n = c.log2n;
    A->nf = wc.nf;
    A->detrend = c.detrend == MTB_DETREND_MEAN ? kDetrendMean : kDetrendNone;
    A->f32 = c.f32;
    A->s0 = wc.a0, A->s1 = wc.a1 / 2, A->s2 = wc.a2 / 2;
    A->c1 = (double)cosl(th), A->sn1 = (double)sinl(th), A->c2 = (double)cosl(2 * th), A->sn2 = (double)sinl(2 * th);
    A->inv_n = 1.0 / c.n;
    // hop = 1 power rows written through to memory (sc1; variant 7 = plain stores): C4 1.5683 / 1.5705 against 1.5729 /
    // 1.5739 ms (r05u, one box) -- the write stream itself is unchanged, what goes is the dirty-line writeback at the end
    A->store_wt = c.variant != 7;
    return MTB_OK;
}

// ------------------------------------------------------------ device path
// series (device) -> [Kalman pre-pass into ws] -> spectrum kernel -> out.
int enqueue(int dev, const Config &c, const double *kalman, const void *d_series, void *d_out, void *d_ws,
            hipStream_t s) {
    Tables t;
    int st = get_tables(dev, c.log2n, c.f32, &t);
    if (st != MTB_OK) return st;
    HIP_OR(hipSetDevice(dev), MTB_BACKEND_UNAVAILABLE);
    if (c.op == kOpInverse) {
        InverseLaunch I{};
        I.in = static_cast<const double *>(d_series);
        I.out = static_cast<double *>(d_out);
        I.twiddle = t.tw;
        I.n_windows = c.n_windows;
        I.log2n = c.log2n;
        I.variant = c.variant;
        I.grid = c.grid;
        HIP_OR(launch_inverse(I, s), MTB_INTERNAL_ERROR);
        return MTB_OK;
    }
    const WsLayout ws = ws_layout(c, dev);
    char *wsb = static_cast<char *>(d_ws);
    if (c.log2n > kMaxLog2N) {  // N > 16384: four-step transform (large_fft.hip)
        LargeLaunch G{};
        G.series = d_series;
        G.hop = c.hop;
        G.detrend = c.detrend;
        if (c.detrend == MTB_DETREND_KALMAN) {
            KalmanLaunch K{};
            K.series = d_series;
            K.detrended = wsb + ws.det;
            K.hop = c.hop;
            K.n_windows = c.n_windows;
            K.n = c.n;
            K.f32 = c.f32;
            K.variant = c.variant;  // the plan's Kalman pre-pass forms (wsp_plan_set_variant: 1, 2, 7, 8)
            memcpy(K.params, kalman, sizeof(K.params));
            HIP_OR(launch_kalman_detrend(K, s), MTB_INTERNAL_ERROR);
            G.series = wsb + ws.det;
            G.hop = c.n;
            G.detrend = kDetrendNone;
        } else if (c.detrend == MTB_DETREND_IIR) {
            const double omega = 2.0 * M_PI / c.trend_period;  // L/WaveSpecZZ_1.0.2.mq5:3041-3043
            G.iir_alpha = (1.0 - sin(omega)) / cos(omega);
            G.iir_c = (1.0 - G.iir_alpha) / 2.0;
        }
        G.out = d_out;
        G.twiddle = t.tw;
        G.detrended = wsb + ws.det;
        G.means = reinterpret_cast<double *>(wsb + ws.means);
        G.y = wsb + ws.y;
        G.n_windows = c.n_windows;
        G.chunk = c.chunk_windows();
        G.log2n = c.log2n;
        G.window = c.window;
        G.packed = c.output == MTB_OUT_PACKED;
        G.f32 = c.f32;
        G.variant = c.variant;
        G.trace = c.trace;
        G.trace_cap = c.trace_cap;
        HIP_OR(launch_large(G, s), MTB_INTERNAL_ERROR);
        return MTB_OK;
    }
    if (use_slide(c) || use_slide_topk(c)) {
        const bool topk = use_slide_topk(c);
        SlideArgs A{};
        if ((st = slide_args(dev, c, &A)) != MTB_OK) return st;
        A.series = d_series;
        A.out = d_out;
        A.n_windows = c.n_windows;
        if (topk) {
            A.seg = slide_topk_seg(c, dev);
            A.variant = c.variant;
            A.kmin = c.kmin;
            A.span = c.kmax - c.kmin + 1;
            A.topk = c.topk;
            A.ws = d_ws;
            A.flags = c.scan_flags;
            // variant 6 (ablation): seed chains of <= 256 windows -- one FFT seed per chain, the next segments' seeds
            // by sliding the band on; slower than one FFT seed per segment (C4 top-8 0.404 against 0.355 ms, a 1/8
            // shard 0.113 against 0.096, r05g: the chain's serial slide steps outlast the parallel FFT seeds)
            // (wsp_plan_set_seed_chain sets the length; a chain's slide is staged in LDS, <= 256 steps)
            A.seed_chain = slide_topk_chain(c, A.seg);
            A.trace = c.trace;
            A.trace_cap = c.trace_cap;
            HIP_OR(launch_slide_topk(A, s), MTB_INTERNAL_ERROR);
            return MTB_OK;
        }
        A.trace = c.trace;  // power slide: workgroup b writes 4 entries at 4 b (diagnostic, wsp_plan_set_trace)
        A.trace_cap = c.trace_cap;
        HIP_OR(launch_slide(A, s), MTB_INTERNAL_ERROR);
        return MTB_OK;
    }
    SpectrumLaunch L{};
    bool window_folded = false;  // the Kalman pre-pass applied the window (kalman_folds_window)
    L.grid = c.grid;
    L.series = d_series;
    L.hop = c.hop;
    L.detrend = c.detrend;
    if (c.detrend == MTB_DETREND_KALMAN) {
        KalmanLaunch K{};
        K.series = d_series;
        K.detrended = d_ws;
        K.hop = c.hop;
        K.n_windows = c.n_windows;
        K.n = c.n;
        K.f32 = c.f32;
        K.variant = c.variant;  // the plan's Kalman pre-pass forms (wsp_plan_set_variant: 1, 2, 7, 8)
        memcpy(K.params, kalman, sizeof(K.params));
        // the fp32 two-segment filter multiplies the window into its rows (round 6): one multiply per sample in a
        // filter bound by its IO instead of the window recurrence in the VALU-bound fp32 spectrum pass
        if (c.f32 && c.variant != 9) {
            st = get_window_pairs(dev, c.n, c.window, &K.window_pairs);
            if (st != MTB_OK) return st;
        }
        HIP_OR(launch_kalman_detrend(K, s), MTB_INTERNAL_ERROR);
        if (kalman_folds_window(K)) window_folded = true;
        L.series = d_ws;
        L.hop = c.n;
        L.detrend = kDetrendNone;
    }
    L.out = d_out;
    L.window = window_folded ? MTB_WINDOW_NONE : c.window;
    L.twiddle = t.tw;
    L.n_windows = c.n_windows;
    L.log2n = c.log2n;
    L.output = c.output;
    L.f32 = c.f32;
    L.topk = c.topk;
    L.kmin = c.kmin;
    L.kmax = c.kmax;
    L.variant = (c.output == MTB_OUT_TOPK_PHASE || c.output == MTB_OUT_PHASE) ? c.variant : 0;
    if (L.detrend == kDetrendIir) {
        // L/WaveSpecZZ_1.0.2.mq5:3041-3043, same double expressions as the CPU path
        const double omega = 2.0 * M_PI / c.trend_period;
        const double alpha = (1.0 - sin(omega)) / cos(omega);
        L.iir_alpha = alpha;
        L.iir_c = (1.0 - alpha) / 2.0;
        long double p = powl((long double)alpha, 32.0L);
        for (int j = 0; j < 8; ++j) {
            L.iir_apow[j] = (double)p;
            p = p * p;
        }
    }
    HIP_OR(launch_spectrum(L, s), MTB_INTERNAL_ERROR);
    return MTB_OK;
}

// ------------------------------------------------------------------ session
// A DeviceCtx owns its streams: they are destroyed with it, i.e. when the
// last holder of the Session (an in-flight call on another thread, or the
// session table) lets it go -- never under a call that still enqueues on them.
struct DeviceCtx {
    int dev = 0;
    std::vector<hipStream_t> streams;
    std::atomic<unsigned> rr{0};
    hipStream_t next_stream() { return streams[rr.fetch_add(1) % streams.size()]; }
    ~DeviceCtx() {
        if (streams.empty()) return;
        (void)hipSetDevice(dev);
        for (auto st : streams) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
    }
};

// Per-bar single-window path (gpu_fft_real_forward, 1.1.0:1249 -> :520): a
// private stream plus device-mapped pinned buffers.  The kernel reads the
// window from and writes the packed spectrum to host memory directly (8-32
// KiB over PCIe), so one call is one kernel launch and one stream sync, with
// no DMA copies and no allocation.  Contexts are checked out per call, so
// concurrent callers (one thread per chart) never share one.
struct LiveCtx {
    int dev = 0;
    hipStream_t stream = nullptr;
    double *h_in = nullptr, *h_out = nullptr;  // pinned, device-mapped
    double *d_in = nullptr, *d_out = nullptr;  // their device addresses
    int cap = 0;                               // doubles per buffer
    ~LiveCtx() {
        (void)hipSetDevice(dev);
        if (stream) {
            (void)hipStreamSynchronize(stream);
            (void)hipStreamDestroy(stream);
        }
        if (h_in) (void)hipHostFree(h_in);
        if (h_out) (void)hipHostFree(h_out);
    }
};

// Caller buffers registered by gpu_register_host (north star: "FeedCache.mqh rewired to stage price bars into
// pinned host buffers for hipMemcpyAsync").  Round 6: the library never page-locks caller memory.  A registration
// records the range (refusing overlaps) and nothing else; every call stages through the library's own pinned
// buffers -- the input through pinned staging, a synchronous call's output through a pinned ring drained while
// later parts are still copied off the device (batch_ring_out).  Page-locking the caller's array (hipHostRegister)
// was opt-in in round 5 and is withdrawn: after such an array was unregistered and freed, a later pageable copy
// into memory reused from its pages could fault (hipErrorIllegalAddress) inside the runtime, with every device
// synchronised around hipHostUnregister.  No exported mode can reach that sequence now.
struct HostRegistry {
    std::mutex mu;
    std::map<uintptr_t, size_t> regions;  // caller base -> bytes, caller ranges disjoint
};

struct Session {
    int device_index = 0;
    int64_t id = 0;  // gpu_session_id: distinct for every session opened in the process
    std::vector<std::unique_ptr<DeviceCtx>> devs;
    std::mutex live_mu;
    std::vector<std::unique_ptr<LiveCtx>> live_free;
    HostRegistry host_regs;  // recorded caller ranges (gpu_register_host); nothing of the caller is page-locked
};

// Session lifetime (SURVEY 8b "per-session refcount"): every successful
// gpu_init adds a reference, every gpu_shutdown drops one; the session is torn
// down only when the count reaches zero.  In MT5 each chart calls gpu_init
// once (EnsureGpu, 1.1.0:722-751) and gpu_shutdown once (OnDeinit,
// 1.1.0:706-716), and all charts share one process: closing one chart must not
// end the others' session.  References are also counted per calling thread
// (MT5 runs each symbol's indicators on one thread): when a thread's own count
// drops to zero its jobs are released, other threads' jobs are left alone.
std::mutex g_session_mu;
std::shared_ptr<Session> g_session;
int g_session_refs = 0;
std::map<std::thread::id, int> *g_thread_refs = new std::map<std::thread::id, int>();

std::shared_ptr<Session> session() {
    std::lock_guard<std::mutex> lk(g_session_mu);
    return g_session;
}

// -------------------------------------------------------------------- batch
// One request split over the session's devices; owns pinned staging and
// device buffers until released.  Used synchronously and as an async job.
struct Part {
    int dev = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    bool recorded = false;  // `done` follows every command of the part
    int64_t w0 = 0, nw = 0;
    void *d_in = nullptr, *d_out = nullptr, *d_ws = nullptr;
    size_t in_bytes = 0, out_bytes = 0, ws_bytes = 0;
};
struct Batch {
    Config cfg;
    double kalman[16];
    std::vector<Part> parts;
    void *h_in = nullptr, *h_out = nullptr;  // pinned staging (h_out: async jobs; synchronous calls use the ring)
    size_t h_in_bytes = 0, h_out_bytes = 0;
    std::vector<void *> ring;                // synchronous calls: pinned output slots, part i -> ring[i % size]
    std::map<int64_t, int64_t> staged;       // series element ranges [first, second) already in h_in
    size_t ring_bytes = 0;
    int status = MTB_OK;
    std::string error;
    ~Batch() {
        for (auto &p : parts) {
            (void)hipSetDevice(p.dev);
            if (p.recorded) (void)hipEventSynchronize(p.done);
            else if (p.stream) (void)hipStreamSynchronize(p.stream);  // a part abandoned mid-enqueue / not copied out
            event_free(p.dev, p.done);
            dev_free(p.dev, p.d_in, p.in_bytes);
            dev_free(p.dev, p.d_out, p.out_bytes);
            dev_free(p.dev, p.d_ws, p.ws_bytes);
        }
        host_free(h_in, h_in_bytes);
        host_free(h_out, h_out_bytes);
        for (void *r : ring) host_free(r, ring_bytes);
    }
};

// Host-side copies of large batches on several threads (one memcpy thread reaches ~10 GB/s, well below PCIe):
// f(begin, end) over [0, n) in slices of at least min_per_thread, on up to 8 threads -- the caller's and the
// copy pool's.  The pool's 7 workers are started once and live as long as the process (a synchronous batch of 64
// parts makes two such calls per part: thread start-up per call would cost milliseconds).  Calls from many
// threads at once (28 charts) share the workers; every caller runs its first slice itself, so each call progresses.
struct CopyPool {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    int started = 0;
    void submit(std::function<void()> f) {
        std::lock_guard<std::mutex> lk(mu);
        if (started < 7) {
            ++started;
            std::thread([this] {
                for (;;) {
                    std::function<void()> t;
                    {
                        std::unique_lock<std::mutex> l(mu);
                        cv.wait(l, [this] { return !q.empty(); });
                        t = std::move(q.front());
                        q.pop_front();
                    }
                    t();
                }
            }).detach();
        }
        q.push_back(std::move(f));
        cv.notify_one();
    }
};
CopyPool &copy_pool() {
    static CopyPool *p = new CopyPool();  // intentionally leaked with its detached workers (process lifetime)
    return *p;
}
template <typename F> void par_for(int64_t n, int64_t min_per_thread, F f) {
    const int64_t want = n / std::max<int64_t>(1, min_per_thread);
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(want, 8));
    if (nt == 1) {
        f(0, n);
        return;
    }
    struct Latch {
        std::mutex m;
        std::condition_variable cv;
        int left = 0;
    } L;
    const int64_t per = (n + nt - 1) / nt;
    for (int t = 1; t < nt; ++t) {
        const int64_t b0 = t * per, b1 = std::min<int64_t>(n, b0 + per);
        if (b0 >= b1) continue;
        {
            std::lock_guard<std::mutex> lk(L.m);
            ++L.left;
        }
        copy_pool().submit([&L, &f, b0, b1] {
            f(b0, b1);
            std::lock_guard<std::mutex> lk(L.m);  // notify under the lock: the waiter cannot return (and free L) first
            if (--L.left == 0) L.cv.notify_one();
        });
    }
    f(0, std::min<int64_t>(n, per));
    std::unique_lock<std::mutex> lk(L.m);
    L.cv.wait(lk, [&L] { return L.left == 0; });
}
constexpr int64_t kCopySlice = int64_t(1) << 19;  // elements per copy thread at least (4 MiB of fp64)
void stage_in(void *dst, const double *src, int64_t n, bool f32) {  // series -> pinned staging
    par_for(n, kCopySlice, [&](int64_t b0, int64_t b1) {
        if (f32) {
            float *d = static_cast<float *>(dst);
            for (int64_t i = b0; i < b1; ++i) d[i] = (float)src[i];
        } else {
            memcpy(static_cast<double *>(dst) + b0, src + b0, (size_t)(b1 - b0) * sizeof(double));
        }
    });
}
void stage_out(double *dst, const void *src, int64_t n, bool f32) {  // pinned results -> caller
    par_for(n, kCopySlice, [&](int64_t b0, int64_t b1) {
        if (f32) {
            const float *s = static_cast<const float *>(src);
            for (int64_t i = b0; i < b1; ++i) dst[i] = (double)s[i];
        } else {
            memcpy(dst + b0, static_cast<const double *>(src) + b0, (size_t)(b1 - b0) * sizeof(double));
        }
    });
}

// A batch is cut into parts: contiguous window ranges per device (the multi-GPU shard), each cut again into
// chunks on the device's streams, so that the host staging of chunk i+1, its H2D copy, the kernels and the D2H
// copies of earlier chunks overlap.  Each part stages and copies its own input slice (with the N - hop halo of
// overlapping windows).  Parts are ordered chunk-major across devices (chunk 0 of every device, then chunk 1,
// ...), so that enqueueing and draining alternate between the devices.
// `ring` (synchronous calls, run_sync): the parts are cut by input AND output bytes (>= WSP_PART_BYTES each, up to
// 64 per device) and their records come back through a ring of kRingSlots pinned slots: the host drains one slot
// into the caller's array while the D2H copies of the next parts are in flight, and stages the next parts' input
// whenever no slot is ready -- so an output-dominated call (C4 from host memory: 8.4 MB in, 8 GiB out) overlaps
// its copy-out with PCIe and holds a few hundred MiB of pinned memory instead of the whole result.  Asynchronous
// jobs (gpu_submit_spectrum_batch) keep the whole result in pinned staging until the caller polls.
#ifndef WSP_PART_BYTES
#define WSP_PART_BYTES (64 << 20)  // the sanitizer builds (tests/hostsan) cut at 64 KiB to exercise many parts
#endif
int batch_plan(Session &S, const Config &c, std::unique_ptr<Batch> *out, bool ring) {
    auto b = std::make_unique<Batch>();
    b->cfg = c;
    {
        std::lock_guard<std::mutex> lk(g_kalman_mu);
        memcpy(b->kalman, g_kalman, sizeof(g_kalman));
    }
    const size_t es = c.elem();
    const size_t in_bytes = (size_t)c.series_elems() * es, out_bytes = (size_t)(c.n_windows * c.record()) * es;
    b->h_in_bytes = in_bytes;
    if (!(b->h_in = host_alloc(in_bytes))) return MTB_NO_MEM;
    if (!ring) {
        b->h_out_bytes = out_bytes;
        if (!(b->h_out = host_alloc(out_bytes))) return MTB_NO_MEM;
    }
    const int G = (int)std::min<int64_t>((int64_t)S.devs.size(), c.n_windows);
    const int64_t per_dev = (c.n_windows + G - 1) / G;
    const int64_t dev_in = std::max<int64_t>(1, (per_dev - 1) * c.hop + c.n) * (int64_t)es;
    const int64_t dev_out = per_dev * c.record() * (int64_t)es;
    const int64_t cut_bytes = ring ? std::max(dev_in, dev_out) : dev_in;
    const int64_t K = std::max<int64_t>(1, std::min<int64_t>({ring ? int64_t(64) : int64_t(16),
                                                              cut_bytes / (int64_t)WSP_PART_BYTES, per_dev}));
    const int64_t per = (per_dev + K - 1) / K;
    for (int64_t k = 0; k < K; ++k)
        for (int g = 0; g < G; ++g) {
            const int64_t d1 = std::min<int64_t>(c.n_windows, (g + 1) * per_dev), w0 = g * per_dev + k * per;
            if (w0 >= d1) continue;
            DeviceCtx &D = *S.devs[g];
            Part p;
            p.dev = D.dev;
            p.w0 = w0;
            p.nw = std::min<int64_t>(per, d1 - w0);
            Config pc = c;
            pc.n_windows = p.nw;
            p.in_bytes = (size_t)pc.series_elems() * es;
            p.out_bytes = (size_t)(p.nw * c.record()) * es;
            p.ws_bytes = ws_layout(pc, D.dev).total;
            p.stream = D.next_stream();
            b->parts.push_back(p);
        }
    *out = std::move(b);
    return MTB_OK;
}

// Stages part i's input slice, copies it to the device and enqueues its kernels (and, outside the ring, its D2H
// copy into the pinned result buffer plus its completion event).
int part_enqueue(Batch &b, int i, const double *series, bool ring) {
    const Config &c = b.cfg;
    const size_t es = c.elem();
    Part &P = b.parts[i];
    Config pc = c;
    pc.n_windows = P.nw;
    HIP_OR(hipSetDevice(P.dev), MTB_BACKEND_UNAVAILABLE);
    P.d_in = dev_alloc(P.dev, P.in_bytes);
    P.d_out = dev_alloc(P.dev, P.out_bytes);
    if (P.ws_bytes) P.d_ws = dev_alloc(P.dev, P.ws_bytes);
    if (!P.d_in || !P.d_out || (P.ws_bytes && !P.d_ws)) return MTB_NO_MEM;
    P.done = event_alloc(P.dev);
    if (!P.done) return MTB_INTERNAL_ERROR;
    const int64_t e0 = P.w0 * c.hop, e1 = e0 + pc.series_elems();
    // stage the samples of [e0, e1) no earlier part staged (the N - hop halo is shared with the neighbouring parts,
    // whose H2D copies may still be reading it)
    {
        auto it = b.staged.upper_bound(e0);  // b.staged: disjoint, merged intervals
        if (it != b.staged.begin() && std::prev(it)->second > e0) --it;
        int64_t x = e0, lo = e0, hi = e1;
        while (it != b.staged.end() && it->first <= e1) {  // overlapping or touching [e0, e1): merged below
            if (it->first > x) stage_in((char *)b.h_in + (size_t)x * es, series + x, it->first - x, c.f32);
            x = std::max(x, it->second);
            lo = std::min(lo, it->first);
            hi = std::max(hi, it->second);
            it = b.staged.erase(it);
        }
        if (x < e1) stage_in((char *)b.h_in + (size_t)x * es, series + x, e1 - x, c.f32);
        b.staged[lo] = hi;
    }
    HIP_OR(hipMemcpyAsync(P.d_in, (const char *)b.h_in + (size_t)e0 * es, P.in_bytes, hipMemcpyHostToDevice, P.stream),
           MTB_INTERNAL_ERROR);
    int st = enqueue(P.dev, pc, b.kalman, P.d_in, P.d_out, P.d_ws, P.stream);
    if (st != MTB_OK) return st;
    if (ring) return MTB_OK;  // copied off the device by run_sync's ring
    const size_t o0 = (size_t)(P.w0 * c.record()) * es;
    HIP_OR(hipMemcpyAsync((char *)b.h_out + o0, P.d_out, P.out_bytes, hipMemcpyDeviceToHost, P.stream),
           MTB_INTERNAL_ERROR);
    HIP_OR(hipEventRecord(P.done, P.stream), MTB_INTERNAL_ERROR);
    P.recorded = true;
    return MTB_OK;
}

// Asynchronous jobs: every part enqueued at once, results into pinned staging.
int batch_start(Session &S, const Config &c, const double *series, std::unique_ptr<Batch> *out) {
    std::unique_ptr<Batch> b;
    int st = batch_plan(S, c, &b, false);
    for (int i = 0; st == MTB_OK && i < (int)b->parts.size(); ++i) st = part_enqueue(*b, i, series, false);
    if (st != MTB_OK) return st;
    *out = std::move(b);
    return MTB_OK;
}

// MTB_OK when every part finished, MTB_NOT_READY otherwise (non-blocking
// unless `wait`).
int part_poll(const Part &p, bool wait) {
    (void)hipSetDevice(p.dev);
    hipError_t e = wait ? hipEventSynchronize(p.done) : hipEventQuery(p.done);
    if (e == hipErrorNotReady) return MTB_NOT_READY;
    if (e != hipSuccess) {
        set_error("device %d: %s", p.dev, hipGetErrorString(e));
        return MTB_INTERNAL_ERROR;
    }
    return MTB_OK;
}
int batch_poll(Batch &b, bool wait) {
    for (auto &p : b.parts) {
        const int st = part_poll(p, wait);
        if (st != MTB_OK) return st;
    }
    return MTB_OK;
}

// Copies the finished records (converted to double) of an asynchronous job into the caller's buffer.
int batch_copy_out(const Batch &b, double *out, int64_t out_cap, int32_t *n_out) {
    const int64_t rec = b.cfg.record();
    const int64_t nrec = std::min<int64_t>(b.cfg.n_windows, out_cap / rec);
    for (const auto &p : b.parts) {
        if (p.w0 >= nrec) continue;
        const int64_t r1 = std::min<int64_t>(p.w0 + p.nw, nrec);
        stage_out(out + p.w0 * rec, (const char *)b.h_out + (size_t)(p.w0 * rec) * b.cfg.elem(), (r1 - p.w0) * rec,
                  b.cfg.f32);
    }
    *n_out = (int32_t)nrec;
    return MTB_OK;
}

// Synchronous batch: parts enqueued one by one, their records copied off the device into the pinned ring
// (part outs[j] -> ring[j % R], on the part's stream after its kernels) and drained into the caller's array.
// The host loop drains a slot as soon as its copy is complete, and otherwise stages and enqueues the next part;
// with nothing left to enqueue it waits for the oldest slot.  Slot j is refilled (outs[j + R]) once drained.
// Only the parts holding records below out_cap are copied.
constexpr int kRingSlots = 4;
int run_sync(const Config &c, const double *series, double *out, int64_t out_cap, int32_t *out_len) {
    auto S = session();
    if (!S) {
        set_error("gpu_init has not succeeded (no GPU session)");
        return MTB_BACKEND_UNAVAILABLE;
    }
    std::unique_ptr<Batch> bp;
    int st = batch_plan(*S, c, &bp, true);
    if (st != MTB_OK) return st;
    Batch &b = *bp;
    const int64_t rec = c.record();
    const size_t es = c.elem();
    const int64_t nrec = std::min<int64_t>(c.n_windows, out_cap / rec);
    std::vector<int> outs;  // parts holding records below out_cap, in enqueue order
    size_t slot = 0;
    for (int i = 0; i < (int)b.parts.size(); ++i)
        if (b.parts[i].w0 < nrec) {
            outs.push_back(i);
            slot = std::max(slot, b.parts[i].out_bytes);
        }
    const int R = std::min<int>(kRingSlots, (int)outs.size());
    b.ring_bytes = slot;
    for (int r = 0; r < R; ++r) {
        b.ring.push_back(host_alloc(slot));
        if (!b.ring.back()) return MTB_NO_MEM;
    }
    auto nrec_of = [&](const Part &p) { return std::min<int64_t>(p.w0 + p.nw, nrec) - p.w0; };
    const int np = (int)b.parts.size(), no = (int)outs.size();
    int enq = 0, issued = 0, drained = 0;
    auto issue_ready = [&]() -> int {  // D2H copies of enqueued parts into free slots
        while (issued < no && issued < drained + R && outs[issued] < enq) {
            Part &P = b.parts[outs[issued]];
            HIP_OR(hipSetDevice(P.dev), MTB_BACKEND_UNAVAILABLE);
            HIP_OR(hipMemcpyAsync(b.ring[issued % R], P.d_out, (size_t)(nrec_of(P) * rec) * es, hipMemcpyDeviceToHost,
                                  P.stream),
                   MTB_INTERNAL_ERROR);
            HIP_OR(hipEventRecord(P.done, P.stream), MTB_INTERNAL_ERROR);
            P.recorded = true;
            ++issued;
        }
        return MTB_OK;
    };
    while (drained < no || enq < np) {
        if (drained < issued) {
            const Part &P = b.parts[outs[drained]];
            st = part_poll(P, enq >= np);  // block only when there is nothing left to stage
            if (st == MTB_OK) {
                stage_out(out + P.w0 * rec, b.ring[drained % R], nrec_of(P) * rec, c.f32);
                ++drained;
                if ((st = issue_ready()) != MTB_OK) return st;
                continue;
            }
            if (st != MTB_NOT_READY) return st;
        }
        if (enq < np) {
            if ((st = part_enqueue(b, enq, series, true)) != MTB_OK) return st;
            ++enq;
            if ((st = issue_ready()) != MTB_OK) return st;
        }
    }
    if (out_len) *out_len = (int32_t)nrec;
    return MTB_OK;
}

// --------------------------------------------------------------------- jobs
// The table only maps ids to batches; a caller copies the shared_ptr out
// under the lock and polls / copies results with the lock released, so one
// chart's multi-GB copy-out never blocks another chart's submit or poll, and
// gpu_free_job during a copy-out only drops the table's reference.
struct Job {
    std::shared_ptr<Batch> batch;
    std::thread::id owner;  // submitting thread: its gpu_shutdown releases the job
};
std::mutex g_jobs_mu;
std::map<int64_t, Job> *g_jobs = new std::map<int64_t, Job>();
std::atomic<int64_t> g_next_id{1};

std::shared_ptr<Batch> find_job(int64_t id) {
    std::lock_guard<std::mutex> lk(g_jobs_mu);
    auto it = g_jobs->find(id);
    return it == g_jobs->end() ? nullptr : it->second.batch;
}

// Removes the jobs of one thread (all threads when `all`); the batches are
// destroyed (waiting for their device work) after the lock is released.
void release_jobs(bool all, std::thread::id owner) {
    std::vector<std::shared_ptr<Batch>> drop;
    {
        std::lock_guard<std::mutex> lk(g_jobs_mu);
        for (auto it = g_jobs->begin(); it != g_jobs->end();) {
            if (all || it->second.owner == owner) {
                drop.push_back(std::move(it->second.batch));
                it = g_jobs->erase(it);
            } else {
                ++it;
            }
        }
    }
}

// -------------------------------------------------------------------- plans
// Plans are shared: wsp_plan_execute holds a reference while it enqueues, so
// a concurrent wsp_plan_destroy cannot free the workspace under it (the last
// reference frees it, after the device has finished with it), and cfg is
// read and written under the plan's own mutex (wsp_plan_set_topk).
// The workspace is a shared_ptr: an execute holds the one it enqueued with, so a reconfiguration that
// needs a larger one (wsp_plan_set_topk / _set_algorithm / _set_slide_segment) swaps it without freeing
// memory a queued launch still uses (the last holder frees it after the device has finished).
//
// A plan with a workspace (Kalman / IIR pre-pass windows, large-N column results, hop = 1 top-k
// segment seeds) is stateful on the device: two executes may not overlap.  wsp_plan_execute orders
// them itself -- each records `done` on its stream, and an execute on a different stream first waits
// for it (hipStreamWaitEvent: device-side ordering, no host sync) -- so one plan may be driven from
// several streams and threads.  Plans without a workspace run concurrently.
struct Plan {
    int dev = 0;
    std::mutex mu;
    Config cfg;
    double kalman[16];
    std::shared_ptr<void> ws;
    size_t ws_bytes = 0;
    hipEvent_t done = nullptr;       // the last workspace execute's completion
    bool done_recorded = false;
    ~Plan() {
        if (done) (void)hipEventDestroy(done);
    }
};

// Retired plan workspaces.  Dropping the last reference to a workspace can happen at the end of a
// wsp_plan_execute (a reconfiguration or wsp_plan_destroy raced with it), and hipFree would wait for
// the whole device there -- every other chart's stream included.  So the deleter only parks the
// block; the configuration calls (plan create / set / destroy, gpu_shutdown), which may block, free
// the parked blocks after a device sync.
std::mutex g_ws_grave_mu;
std::vector<std::pair<int, void *>> *g_ws_grave = new std::vector<std::pair<int, void *>>();
void ws_reap() {
    std::vector<std::pair<int, void *>> v;
    {
        std::lock_guard<std::mutex> lk(g_ws_grave_mu);
        v.swap(*g_ws_grave);
    }
    for (auto &e : v) {
        (void)hipSetDevice(e.first);
        (void)hipDeviceSynchronize();  // queued launches may still read it
        (void)hipFree(e.second);
    }
}
std::shared_ptr<void> plan_ws_alloc(int dev, size_t bytes) {
    void *d = nullptr;
    if (hipSetDevice(dev) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return nullptr;
    return std::shared_ptr<void>(d, [dev](void *q) {
        std::lock_guard<std::mutex> lk(g_ws_grave_mu);
        g_ws_grave->emplace_back(dev, q);
    });
}
// (under p->mu) grow the workspace to what cfg needs
int plan_ws_fit(Plan &p) {
    ws_reap();
    const size_t need = ws_layout(p.cfg, p.dev).total;
    if (need <= p.ws_bytes) return MTB_OK;
    auto w = plan_ws_alloc(p.dev, need);
    if (!w) {
        set_error("hipMalloc(%zu) for the plan workspace failed", need);
        return MTB_NO_MEM;
    }
    p.ws = std::move(w);  // the old block is parked now, unless an execute still holds it
    p.ws_bytes = need;
    ws_reap();            // ... and freed here rather than at the next configuration call
    return MTB_OK;
}
std::mutex g_plans_mu;
std::map<int64_t, std::shared_ptr<Plan>> *g_plans = new std::map<int64_t, std::shared_ptr<Plan>>();

std::shared_ptr<Plan> find_plan(int64_t id) {
    std::lock_guard<std::mutex> lk(g_plans_mu);
    auto it = g_plans->find(id);
    return it == g_plans->end() ? nullptr : it->second;
}

// ------------------------------------------------------- live single window
std::unique_ptr<LiveCtx> live_checkout(Session &S, int n) {
    std::unique_ptr<LiveCtx> L;
    {
        std::lock_guard<std::mutex> lk(S.live_mu);
        if (!S.live_free.empty()) {
            L = std::move(S.live_free.back());
            S.live_free.pop_back();
        }
    }
    if (!L) {
        L = std::make_unique<LiveCtx>();
        L->dev = S.devs[0]->dev;
        if (hipSetDevice(L->dev) != hipSuccess ||
            hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking) != hipSuccess) {
            set_error("live context: stream creation failed on device %d", L->dev);
            return nullptr;
        }
    }
    if (L->cap < n) {
        (void)hipSetDevice(L->dev);
        if (L->h_in) (void)hipHostFree(L->h_in);
        if (L->h_out) (void)hipHostFree(L->h_out);
        L->h_in = L->h_out = nullptr;
        L->cap = 0;
        void *hi = nullptr, *ho = nullptr, *di = nullptr, *dd = nullptr;
        if (hipHostMalloc(&hi, (size_t)n * sizeof(double), hipHostMallocMapped) != hipSuccess ||
            hipHostMalloc(&ho, (size_t)n * sizeof(double), hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer(&di, hi, 0) != hipSuccess || hipHostGetDevicePointer(&dd, ho, 0) != hipSuccess) {
            if (hi) (void)hipHostFree(hi);
            if (ho) (void)hipHostFree(ho);
            set_error("live context: mapped pinned buffers of %d doubles failed", n);
            return nullptr;
        }
        L->h_in = static_cast<double *>(hi);
        L->h_out = static_cast<double *>(ho);
        L->d_in = static_cast<double *>(di);
        L->d_out = static_cast<double *>(dd);
        L->cap = n;
    }
    return L;
}
void live_checkin(Session &S, std::unique_ptr<LiveCtx> L) {
    std::lock_guard<std::mutex> lk(S.live_mu);
    S.live_free.push_back(std::move(L));
}

// ------------------------------------------------------------------ grouped hop = 1 plans
// A multi-symbol hop = 1 batch -- the WaveCyclesBatchFetcher shape, one series per symbol
// (WaveCyclesBatchFetcher.mq5:112-118), C5 = 28 symbols of 4 window lengths -- as one device plan:
// the members of each window length run in ONE sliding-DFT launch (launch_slide_group: workgroup ->
// (member, segment) table), longest windows first, on the caller's stream.  Against one plan per
// symbol this removes the per-plan launches and, above all, the short per-plan segments: the segment
// length follows the residency and the length's TOTAL window count, so a 19k-window symbol seeds its
// trackers once per 128-256 windows instead of once per 32.  No workspace: executes may overlap.
struct Group {
    int dev = 0;
    std::vector<Config> cfg;               // one per member (hop 1, power)
    std::vector<std::vector<int>> launch;  // member indices per launch: one window length, <= kSlideGroupMax
    std::vector<int64_t> launch_bytes;     // output bytes per launch: what the slide's time follows
    std::mutex mu;                         // executes on the internal streams are enqueued one at a time
    int64_t seg = 0;                       // windows per workgroup, 0 = the launcher's policy
    // one mixed-length persistent launch (slide_mixed.hip) when every member is 512..4096 with <= 3 window terms
    // and there are at most kMixMax members; wsp_group_set_mode(1) forces the per-length launches
    bool mix_ok = false;
    int mode = 0;
    int *ctr = nullptr;                    // 256 task-counter slots (counter, done) on the device, zeroed at create
    uint32_t exec_no = 0;
    // per slot: the event its last execute recorded -- every execute waits for the slot's previous user before
    // it reuses the counters (more than 256 executes in flight; a no-op on the same stream)
    std::vector<hipEvent_t> slot_ev;
    long long *trace = nullptr;            // wsp_group_set_trace: diagnostic per-task timeline of the mixed launch
    int64_t trace_cap = 0, last_tasks = 0;
    // wsp_group_set_streams(n > 1): n - 1 internal streams beside the caller's (wsp_group_execute)
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> events;  // [0] fork, [k] join of internal stream k - 1
    void release() {
        (void)hipSetDevice(dev);
        for (auto st : streams) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
        for (auto e : events) (void)hipEventDestroy(e);
        streams.clear();
        events.clear();
    }
    ~Group() {
        release();
        if (ctr) {
            (void)hipSetDevice(dev);
            (void)hipDeviceSynchronize();  // a queued execute may still count on its slot
            (void)hipFree(ctr);
        }
        for (auto e : slot_ev)
            if (e) (void)hipEventDestroy(e);
    }
};
std::mutex g_groups_mu;
std::map<int64_t, std::shared_ptr<Group>> *g_groups = new std::map<int64_t, std::shared_ptr<Group>>();

std::shared_ptr<Group> find_group(int64_t id) {
    std::lock_guard<std::mutex> lk(g_groups_mu);
    auto it = g_groups->find(id);
    return it == g_groups->end() ? nullptr : it->second;
}

// (under g.mu) n lanes for wsp_group_execute: the caller's stream + n - 1 internal streams and their events
constexpr int kMixSlots = 256;  // counter slots: executes of one group in flight at once on different streams

// One persistent launch over every member (slide_mixed.hip), on the caller's stream.  Members are laid out class by
// class, longest windows first; segment length S over the whole batch: about two tasks per resident workgroup (a task
// = S windows x 2048 bins, half that for N <= 1024), 128..256 windows (wsp_group_set_segment overrides it).  The
// floor of 128: a segment's seed (a full FFT) costs tens of slides, and at small batches (a one-eighth C5 shard)
// shorter segments lost more to seeds than they gained in balance (0.142 ms at 32 against 0.122 at 128, r04d).
int group_execute_mixed(Group &g, const void *const *d_series, void *const *d_out, hipStream_t s) {
    const int n = (int)g.cfg.size();
    std::vector<int> order(n);
    for (int i = 0; i < n; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return g.cfg[a].log2n > g.cfg[b].log2n; });
    SlideMix m{};
    m.bsmall = g.mode == 2 ? 4 : 2;  // measured: 0.737 ms (2) against 0.777 (4) for C5, profiles/r04/ab
    m.seed_lds = g.mode == 5;        // ablation: the round-4 seed FFTs
    // output rows written through to memory (sc1 stores; mode 6 = plain): no dirty output lines wait in the XCDs' L2s
    // for the writeback at the end of the launch -- C5 0.7275 / 0.7298 -> 0.7024 / 0.7114 ms (r05t, one box)
    m.wt = g.mode != 6;
    const Config &c0 = g.cfg[order[0]];
    const int nf = window_coef(c0.window).nf;
    const int det = c0.detrend == MTB_DETREND_MEAN ? kDetrendMean : kDetrendNone;
    const int res = slide_mix_resident(nf, det, c0.f32, m.bsmall, g.dev);
    int64_t bins = 0;
    for (const Config &c : g.cfg) bins += c.n_windows * (int64_t)(c.n / 2);
    int64_t S = g.seg;
    const bool policy = S <= 0;
    bool above_floor = false;
    // small batches (fewer than two tasks per resident workgroup at the floor -- a strong-scaled shard): every task the
    // same length.  A task of the N <= 1024 classes holds half the bins of a 2048 / 4096 task at the same segment length
    // (B = bsmall bins per thread instead of 4), so those classes take segments 4 / B times as long.  A 1/8 C5 shard
    // holding 2048- and 1024-point windows at one length had 395 tasks of two costs: the rank waited for its long
    // tasks while short ones doubled up on their CUs (r05m timeline: busy 0.56; 0.133-0.141 ms against 0.109-0.116
    // for the single-length ranks).  Measured and dropped (r05n): one task per CU at segments just covering the CUs
    // (S = 110 instead of 128 on a 2048-point shard) -- every rank 4-10 % slower: the shard's slide is bound by the
    // aggregate write rate, not by idle CUs, and the extra seeds cost more.
    // Round 6: such a batch takes 64-window segments instead of the floor's 128 -- several rounds of shorter tasks, so
    // that a CU whose tasks end early takes more instead of idling while its slowest one slides alone (the single-
    // length slide's finding, sliding_core.h launch_t): 1/8 C5 shards' worst rank 0.1172 -> 0.1115 ms with 64-window
    // segments on one box (r06c5, each rank the median of 3 passes), the whole batch (above the floor) unchanged.
    bool small = false;
    if (policy) {
        S = (int64_t)std::ceil((double)bins / (2.0 * res * 2048.0));
        above_floor = S > 128;
        small = !above_floor && (g.mode == 0 || g.mode == 6);
        S = above_floor ? std::min<int64_t>(256, S) : (g.mode == 0 || g.mode == 6 ? 64 : 128);
    }
    // Half-length segments for the last class (the shortest windows, picked up last, drain the launch) when the
    // batch is large enough that the policy's segments are above the floor: the full C5 batch 0.7322-0.7325 ms
    // against 0.7373-0.7398 with one length on three boxes (r04l, r04m), while a one-eighth shard (segments at the
    // floor, where halving only adds seeds) ran 5 % slower with them.  Mode 3: at every size; mode 4: never (A/B).
    const int last_l2 = g.cfg[order[n - 1]].log2n;
    const bool tail_half = policy && g.cfg[order[0]].log2n != last_l2 &&
                           (g.mode == 3 || ((g.mode == 0 || g.mode == 2 || g.mode == 5 || g.mode == 6) && above_floor));
    Tables t4096;
    int st = get_tables(g.dev, 12, false, &t4096);
    if (st != MTB_OK) return st;
    m.tw4096 = t4096.tw;
    int nc = -1, prev = -1;
    int64_t tasks = 0, segs = 0;
    auto close_class = [&]() {
        if (nc < 0) return;
        const int l2 = m.log2n[nc];
        const int P = kMixNT * 2 * (l2 <= 10 ? m.bsmall : 4) / (1 << l2);  // sub-workgroups: 512 / (N / 2B)
        m.nseg[nc] = (int)segs;
        m.task0[nc] = (int)tasks;
        tasks += (segs + P - 1) / P;
    };
    for (int i = 0; i < n; ++i) {
        const Config &c = g.cfg[order[i]];
        if (c.log2n != prev) {
            close_class();
            ++nc;
            prev = c.log2n;
            SlideArgs A{};
            if ((st = slide_args(g.dev, c, &A)) != MTB_OK) return st;
            m.log2n[nc] = c.log2n;
            m.seg[nc] = small && c.log2n <= 10 ? (int)(S * 4 / m.bsmall)
                                               : (int)(tail_half && c.log2n == last_l2 ? std::max<int64_t>(64, S / 2) : S);
            m.mem0[nc] = i;
            m.c1[nc] = A.c1, m.sn1[nc] = A.sn1, m.c2[nc] = A.c2, m.sn2[nc] = A.sn2, m.inv_n[nc] = A.inv_n;
            m.omega[nc] = A.omega;
            m.s0 = A.s0, m.s1 = A.s1, m.s2 = A.s2;
            segs = 0;
        }
        m.sg0[i] = segs;
        m.n_windows[i] = c.n_windows;
        m.series[i] = d_series[order[i]];
        m.out[i] = d_out[order[i]];
        segs += (c.n_windows + m.seg[nc] - 1) / m.seg[nc];
    }
    close_class();
    m.nclass = nc + 1;
    m.mem0[m.nclass] = n;
    if (tasks > INT32_MAX) {
        set_error("wsp_group_execute: %lld tasks", (long long)tasks);
        return MTB_BAD_ARGS;
    }
    m.n_tasks = (int)tasks;
    g.last_tasks = tasks;
    m.trace = g.trace && tasks <= g.trace_cap ? g.trace : nullptr;
    const int slot = (int)(g.exec_no++ % kMixSlots);
    m.counter = g.ctr + 2 * slot;
    m.done = g.ctr + 2 * slot + 1;
    if (g.slot_ev.empty()) g.slot_ev.assign(kMixSlots, nullptr);
    hipEvent_t &ev = g.slot_ev[slot];
    if (!ev) HIP_OR(hipEventCreateWithFlags(&ev, hipEventDisableTiming), MTB_INTERNAL_ERROR);
    else HIP_OR(hipStreamWaitEvent(s, ev, 0), MTB_INTERNAL_ERROR);  // always: a destroyed stream's handle can come back
    const int grid = (int)std::min<int64_t>(res, tasks);
    HIP_OR(launch_slide_mix(m, nf, det, c0.f32, grid, s), MTB_INTERNAL_ERROR);
    HIP_OR(hipEventRecord(ev, s), MTB_INTERNAL_ERROR);
    return MTB_OK;
}

int group_lanes(Group &g, int n_streams) {
    g.release();
    if (n_streams == 1) return MTB_OK;
    HIP_OR(hipSetDevice(g.dev), MTB_BACKEND_UNAVAILABLE);
    for (int i = 0; i < n_streams - 1; ++i) {  // + the caller's stream = n_streams lanes
        hipStream_t st = nullptr;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
            g.release();
            set_error("wsp_group_set_streams: stream creation failed");
            return MTB_INTERNAL_ERROR;
        }
        g.streams.push_back(st);
    }
    for (int i = 0; i < n_streams; ++i) {  // [0] fork, [k] join of internal stream k
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            g.release();
            set_error("wsp_group_set_streams: event creation failed");
            return MTB_INTERNAL_ERROR;
        }
        g.events.push_back(e);
    }
    return MTB_OK;
}


}  // namespace

// =========================================================================
extern "C" {

MTB_API const char *wsp_version(void) { return "mtbridge-mi355x 0.1.0 gfx950"; }

MTB_API int32_t gpu_init(int32_t device_index, int32_t stream_count) {
    std::lock_guard<std::mutex> lk(g_session_mu);
    if (g_session) {
        if (g_session->device_index != device_index) {
            set_error("gpu_init(%d): a session is open on device %d for %d caller(s); gpu_shutdown them first",
                      device_index, g_session->device_index, g_session_refs);
            return MTB_BAD_ARGS;
        }
        ++g_session_refs;
        ++(*g_thread_refs)[std::this_thread::get_id()];
        return MTB_OK;
    }
    const int n = device_count();
    if (n <= 0) {
        set_error("no HIP device visible (hipGetDeviceCount=0); the spectrum path has no CPU fallback");
        return MTB_BACKEND_UNAVAILABLE;
    }
    if (device_index < -1 || device_index >= n) {
        set_error("device_index=%d out of range (%d devices, -1 = all)", device_index, n);
        return MTB_BAD_ARGS;
    }
    const int streams = std::max(1, std::min(512, (int)stream_count));
    auto S = std::make_shared<Session>();  // on failure below, ~DeviceCtx destroys the streams made so far
    S->device_index = device_index;
    const int first = device_index < 0 ? 0 : device_index;
    const int last = device_index < 0 ? n - 1 : device_index;
    for (int d = first; d <= last; ++d) {
        S->devs.push_back(std::make_unique<DeviceCtx>());
        DeviceCtx &D = *S->devs.back();
        D.dev = d;
        HIP_OR(hipSetDevice(d), MTB_BACKEND_UNAVAILABLE);
        for (int k = 0; k < streams; ++k) {
            hipStream_t st;
            HIP_OR(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), MTB_BACKEND_UNAVAILABLE);
            D.streams.push_back(st);
        }
    }
    static int64_t next_id = 0;  // under g_session_mu
    S->id = ++next_id;
    g_session = S;
    g_session_refs = 1;
    g_thread_refs->clear();
    (*g_thread_refs)[std::this_thread::get_id()] = 1;
    return MTB_OK;
}

MTB_API void gpu_shutdown(void) {
    const std::thread::id me = std::this_thread::get_id();
    std::shared_ptr<Session> S;
    bool mine = false;
    {
        std::lock_guard<std::mutex> lk(g_session_mu);
        if (!g_session) return;
        auto it = g_thread_refs->find(me);
        if (it != g_thread_refs->end() && --it->second <= 0) {
            g_thread_refs->erase(it);
            mine = true;
        } else if (it == g_thread_refs->end()) {
            mine = true;  // a thread that holds no reference of its own: only its own jobs (if any) go
        }
        if (--g_session_refs <= 0) {
            S = std::move(g_session);
            g_session.reset();
            g_session_refs = 0;
            g_thread_refs->clear();
        }
    }
    if (S) {
        release_jobs(true, me);  // ~Batch waits for in-flight work
        S.reset();               // streams go with the last holder (calls in flight keep their own reference)
        pool_release_all();
        ws_reap();
    } else if (mine) {
        release_jobs(false, me);
    }
}

// gpu_set_host_locking: round 5 made page-locking of caller memory opt-in (mode 1); round 6 withdraws it.
// Mode 0 (record the range, stage through the library's pinned buffers) is the only mode: 0 returns 0, 1 is
// refused with MTB_BAD_ARGS and an explanation, anything else is refused as before.  See HostRegistry.
MTB_API int32_t gpu_set_host_locking(int32_t mode) {
    if (mode == 1) {
        set_error("gpu_set_host_locking(1): page-locking caller memory was withdrawn (a pageable copy into pages of an "
                  "unregistered, freed buffer could fault, DESIGN.md 4.2); registrations record the range and calls "
                  "stage through the library's pinned buffers");
        return MTB_BAD_ARGS;
    }
    if (mode != 0) {
        set_error("gpu_set_host_locking(%d): mode must be 0 (record only)", mode);
        return MTB_BAD_ARGS;
    }
    return 0;
}

MTB_API int32_t gpu_register_host(const double *ptr, int64_t count) {
    if (!ptr || count <= 0) {
        set_error("gpu_register_host: null buffer or count %lld <= 0", (long long)count);
        return MTB_BAD_ARGS;
    }
    auto S = session();
    if (!S) {
        set_error("gpu_init has not succeeded (no GPU session)");
        return MTB_BACKEND_UNAVAILABLE;
    }
    const uintptr_t a = (uintptr_t)ptr;
    const size_t bytes = (size_t)count * sizeof(double);
    if ((size_t)count > SIZE_MAX / sizeof(double) || a + bytes < a) {
        set_error("gpu_register_host: [%p, +%lld doubles) wraps the address space", (const void *)ptr, (long long)count);
        return MTB_BAD_ARGS;
    }
    HostRegistry &R = S->host_regs;
    std::lock_guard<std::mutex> lk(R.mu);
    auto it = R.regions.lower_bound(a);  // caller ranges are disjoint
    const bool overlaps = (it != R.regions.end() && it->first < a + bytes) ||
                          (it != R.regions.begin() && std::prev(it)->first + std::prev(it)->second > a);
    if (overlaps) {
        set_error("gpu_register_host: [%p, +%zu B) overlaps a registered buffer", (const void *)ptr, bytes);
        return MTB_BAD_ARGS;
    }
    R.regions.emplace(a, bytes);
    return MTB_OK;
}

MTB_API int64_t gpu_session_id(void) {
    auto S = session();
    return S ? S->id : 0;
}

MTB_API int32_t gpu_unregister_host(const double *ptr) {
    auto S = session();
    if (!S) {
        set_error("gpu_init has not succeeded (no GPU session)");
        return MTB_BACKEND_UNAVAILABLE;
    }
    HostRegistry &R = S->host_regs;
    std::lock_guard<std::mutex> lk(R.mu);
    auto it = R.regions.find((uintptr_t)ptr);
    if (!ptr || it == R.regions.end()) {
        set_error("gpu_unregister_host: %p is not the start of a registered buffer", (const void *)ptr);
        return MTB_BAD_ARGS;
    }
    R.regions.erase(it);
    return MTB_OK;
}

MTB_API int32_t gpu_fft_real_forward(const double *in, int32_t len, double *out) {
    if (!in || !out) {
        set_error("gpu_fft_real_forward: null buffer");
        return MTB_BAD_ARGS;
    }
    Config c;
    int st = make_config(len, len, 1, MTB_DETREND_NONE, MTB_WINDOW_NONE, 0, MTB_PREC_F64, MTB_OUT_PACKED, &c);
    if (st != MTB_OK) return st;
    auto S = session();
    if (!S) {
        set_error("gpu_init has not succeeded (no GPU session)");
        return MTB_BACKEND_UNAVAILABLE;
    }
    if (c.log2n > kMaxLog2N) {  // four-step transform: needs its chunk workspace, take the batch path
        int32_t n = 0;
        return run_sync(c, in, out, len, &n);
    }
    std::unique_ptr<LiveCtx> L = live_checkout(*S, len);
    if (!L) return MTB_NO_MEM;
    memcpy(L->h_in, in, (size_t)len * sizeof(double));
    st = enqueue(L->dev, c, nullptr, L->d_in, L->d_out, nullptr, L->stream);
    if (st == MTB_OK) {
        const hipError_t e = hipStreamSynchronize(L->stream);
        if (e != hipSuccess) {
            set_error("gpu_fft_real_forward: %s", hipGetErrorString(e));
            st = MTB_INTERNAL_ERROR;
        } else {
            memcpy(out, L->h_out, (size_t)len * sizeof(double));
        }
    }
    live_checkin(*S, std::move(L));
    return st;
}

MTB_API int32_t gpu_fft_real_forward_batch(const double *in, int32_t window_len, int32_t n_windows, double *out) {
    if (!in || !out) {
        set_error("gpu_fft_real_forward_batch: null buffer");
        return MTB_BAD_ARGS;
    }
    Config c;
    int st = make_config(window_len, window_len, n_windows, MTB_DETREND_NONE, MTB_WINDOW_NONE, 0, MTB_PREC_F64,
                         MTB_OUT_PACKED, &c);
    if (st != MTB_OK) return st;
    int32_t n = 0;
    return run_sync(c, in, out, (int64_t)window_len * n_windows, &n);
}

static int inverse_config(int32_t window_len, int32_t n_windows, Config *c) {
    int st = make_config(window_len, window_len, n_windows, MTB_DETREND_NONE, MTB_WINDOW_NONE, 0, MTB_PREC_F64,
                         MTB_OUT_PACKED, c);
    c->op = kOpInverse;
    if (st == MTB_OK && c->log2n > kMaxLog2N) {
        set_error("window_len=%d: the inverse transform covers windows up to %d", window_len, 1 << kMaxLog2N);
        return MTB_BAD_ARGS;
    }
    return st;
}

MTB_API int32_t gpu_fft_real_inverse(const double *in_spec, int32_t len, double *out) {
    if (!in_spec || !out) {
        set_error("gpu_fft_real_inverse: null buffer");
        return MTB_BAD_ARGS;
    }
    Config c;
    int st = inverse_config(len, 1, &c);
    if (st != MTB_OK) return st;
    int32_t n = 0;
    return run_sync(c, in_spec, out, len, &n);
}

MTB_API int32_t gpu_fft_real_inverse_batch(const double *in, int32_t window_len, int32_t n_windows, double *out) {
    if (!in || !out) {
        set_error("gpu_fft_real_inverse_batch: null buffer");
        return MTB_BAD_ARGS;
    }
    Config c;
    int st = inverse_config(window_len, n_windows, &c);
    if (st != MTB_OK) return st;
    int32_t n = 0;
    return run_sync(c, in, out, (int64_t)window_len * n_windows, &n);
}

MTB_API int32_t gpu_spectral_phase_unwrap(const double *spectrum, int32_t spectrum_len, int32_t method, double *out,
                                          int32_t out_len) {
    if (!spectrum || !out || spectrum_len < 2 || (spectrum_len & 1) || method < 0 || method > 2 ||
        out_len < spectrum_len / 2) {
        set_error("gpu_spectral_phase_unwrap: spectrum_len=%d (even, >= 2) method=%d (0..2) out_len=%d (>= %d)",
                  spectrum_len, method, out_len, spectrum_len / 2);
        return MTB_BAD_ARGS;
    }
    auto S = session();
    if (!S) {
        set_error("gpu_init has not succeeded (no GPU session)");
        return MTB_BACKEND_UNAVAILABLE;
    }
    DeviceCtx &D = *S->devs[0];
    const int nb = spectrum_len / 2;
    const size_t in_bytes = (size_t)spectrum_len * sizeof(double), out_bytes = (size_t)nb * sizeof(double);
    HIP_OR(hipSetDevice(D.dev), MTB_BACKEND_UNAVAILABLE);
    void *d_in = dev_alloc(D.dev, in_bytes), *d_out = dev_alloc(D.dev, out_bytes);
    if (!d_in || !d_out) {
        dev_free(D.dev, d_in, in_bytes);
        dev_free(D.dev, d_out, out_bytes);
        return MTB_NO_MEM;
    }
    const hipStream_t s = D.next_stream();
    int st = MTB_OK;
    hipError_t e = hipMemcpyAsync(d_in, spectrum, in_bytes, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = launch_phase_row((const double *)d_in, nb, method, (double *)d_out, s);
    if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        set_error("gpu_spectral_phase_unwrap: %s", hipGetErrorString(e));
        st = MTB_INTERNAL_ERROR;
    }
    dev_free(D.dev, d_in, in_bytes);
    dev_free(D.dev, d_out, out_bytes);
    return st;
}

static int spectrum_config(const double *series, int32_t series_len, int32_t window_len, int32_t hop,
                           int32_t detrend, int32_t window, int32_t trend_period, int32_t precision, int32_t output,
                           Config *c) {
    if (!series) {
        set_error("null series");
        return MTB_BAD_ARGS;
    }
    if (window_len <= 0 || series_len < window_len || hop <= 0) {
        set_error("series_len=%d window_len=%d hop=%d: need series_len >= window_len > 0, hop > 0", series_len,
                  window_len, hop);
        return MTB_BAD_ARGS;
    }
    const int64_t nwin = 1 + ((int64_t)series_len - window_len) / hop;  // 1.1.0:1016
    return make_config(window_len, hop, nwin, detrend, window, trend_period, precision, output, c);
}

MTB_API int32_t gpu_spectrum_batch(const double *series, int32_t series_len, int32_t window_len, int32_t hop,
                                   int32_t detrend, int32_t window, int32_t trend_period, int32_t precision,
                                   int32_t output, double *out, int32_t out_cap, int32_t *out_len) {
    if (out_len) *out_len = 0;
    Config c;
    int st = spectrum_config(series, series_len, window_len, hop, detrend, window, trend_period, precision, output, &c);
    if (st != MTB_OK) return st;
    if (!out || out_cap < c.record()) {
        set_error("out_cap=%d smaller than one record (%lld doubles)", out_cap, (long long)c.record());
        return MTB_BAD_ARGS;
    }
    // only the records that fit are computed
    c.n_windows = std::min<int64_t>(c.n_windows, out_cap / c.record());
    return run_sync(c, series, out, out_cap, out_len);
}

MTB_API int32_t gpu_spectrum_topk_batch(const double *series, int32_t series_len, int32_t window_len, int32_t hop,
                                        int32_t detrend, int32_t window, int32_t trend_period, int32_t precision,
                                        int32_t top_k, double min_period, double max_period, double *out,
                                        int32_t out_cap, int32_t *out_len) {
    if (out_len) *out_len = 0;
    Config c;
    int st = spectrum_config(series, series_len, window_len, hop, detrend, window, trend_period, precision,
                             MTB_OUT_POWER, &c);
    if (st != MTB_OK) return st;
    st = config_set_topk(&c, top_k, min_period, max_period);
    if (st != MTB_OK) return st;
    if (!out || out_cap < c.record()) {
        set_error("out_cap=%d smaller than one record (%lld doubles)", out_cap, (long long)c.record());
        return MTB_BAD_ARGS;
    }
    c.n_windows = std::min<int64_t>(c.n_windows, out_cap / c.record());
    return run_sync(c, series, out, out_cap, out_len);
}

MTB_API int32_t gpu_spectrum_topk_phase_batch(const double *series, int32_t series_len, int32_t window_len,
                                              int32_t hop, int32_t detrend, int32_t window, int32_t trend_period,
                                              int32_t top_k, double min_period, double max_period, double *out,
                                              int32_t out_cap, int32_t *out_len) {
    if (out_len) *out_len = 0;
    Config c;
    int st = spectrum_config(series, series_len, window_len, hop, detrend, window, trend_period, MTB_PREC_F64,
                             MTB_OUT_TOPK_PHASE, &c);
    if (st != MTB_OK) return st;
    st = config_set_topk(&c, top_k, min_period, max_period);
    if (st != MTB_OK) return st;
    if (!out || out_cap < c.record()) {
        set_error("out_cap=%d smaller than one record (%lld doubles)", out_cap, (long long)c.record());
        return MTB_BAD_ARGS;
    }
    c.n_windows = std::min<int64_t>(c.n_windows, out_cap / c.record());
    return run_sync(c, series, out, out_cap, out_len);
}

MTB_API int32_t gpu_submit_spectrum_batch(const double *series, int32_t series_len, int32_t window_len,
                                          int32_t hop, int32_t detrend, int32_t window, int32_t trend_period,
                                          int32_t precision, int32_t output, int64_t *job_id) {
    if (!job_id) {
        set_error("null job_id");
        return MTB_BAD_ARGS;
    }
    *job_id = 0;
    Config c;
    int st = spectrum_config(series, series_len, window_len, hop, detrend, window, trend_period, precision, output, &c);
    if (st != MTB_OK) return st;
    auto S = session();
    if (!S) {
        set_error("gpu_init has not succeeded (no GPU session)");
        return MTB_BACKEND_UNAVAILABLE;
    }
    std::unique_ptr<Batch> b;
    st = batch_start(*S, c, series, &b);
    if (st != MTB_OK) return st;
    const int64_t id = g_next_id.fetch_add(1);
    {
        std::lock_guard<std::mutex> lk(g_jobs_mu);
        (*g_jobs)[id] = Job{std::shared_ptr<Batch>(std::move(b)), std::this_thread::get_id()};
    }
    *job_id = id;
    return MTB_OK;
}

MTB_API int32_t gpu_try_get_spectrum_batch(int64_t job_id, double *out, int32_t out_cap, int32_t *out_len,
                                           int32_t *ready) {
    if (ready) *ready = 0;
    if (out_len) *out_len = 0;
    std::shared_ptr<Batch> b = find_job(job_id);  // the table lock is held only for the lookup
    if (!b) {
        set_error("unknown job id %lld", (long long)job_id);
        return MTB_BAD_ARGS;
    }
    const int st = batch_poll(*b, false);
    // pending: MTB_OK + ready = 0.  WaveCyclesBatchFetcher.mq5:127-131 sleeps only on OK with
    // ready == 0 and re-polls at once on NOT_READY (4000 tries spent in microseconds); the
    // indicator's warm-up loop (1.1.0:1029-1039) accepts both conventions.
    if (st == MTB_NOT_READY) return MTB_OK;
    if (ready) *ready = 1;
    if (st != MTB_OK) return st;
    if (!out || out_cap < b->cfg.record()) {
        set_error("out_cap=%d smaller than one record (%lld doubles)", out_cap, (long long)b->cfg.record());
        return MTB_BAD_ARGS;
    }
    int32_t n = 0;
    const int cst = batch_copy_out(*b, out, out_cap, &n);
    if (cst != MTB_OK) return cst;
    if (out_len) *out_len = n;
    return MTB_OK;
}

MTB_API int32_t gpu_free_job(int64_t job_id) {
    std::shared_ptr<Batch> b;
    {
        std::lock_guard<std::mutex> lk(g_jobs_mu);
        auto it = g_jobs->find(job_id);
        if (it == g_jobs->end()) {
            set_error("unknown job id %lld", (long long)job_id);
            return MTB_BAD_ARGS;
        }
        b = std::move(it->second.batch);
        g_jobs->erase(it);
    }
    return MTB_OK;  // the last reference's ~Batch waits for the device and recycles buffers
}

MTB_API int32_t gpu_set_kalman_params(const double *params, int32_t n) {
    if (!params || n != 16) {
        set_error("gpu_set_kalman_params: need 16 parameters, got %d", n);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(g_kalman_mu);
    memcpy(g_kalman, params, sizeof(g_kalman));
    return MTB_OK;
}

// ---- cycle extraction: not part of the spectrum hot path -----------------
#define CYCLES_UNAVAILABLE(name)                                                                         \
    set_error(name ": MUSIC/ESPRIT cycle extraction is outside the MI355X spectrum path (SURVEY 2 row 13)"); \
    return MTB_BACKEND_UNAVAILABLE

MTB_API int32_t gpu_extract_cycles(const double *, int32_t, int32_t, double, double, double, int32_t, int32_t,
                                   double *, int32_t, int32_t, int32_t *out_len) {
    if (out_len) *out_len = 0;
    CYCLES_UNAVAILABLE("gpu_extract_cycles");
}
MTB_API int32_t gpu_submit_extract_cycles(const double *, int32_t, int32_t, double, double, double, int32_t, int32_t,
                                          int64_t *job_id) {
    if (job_id) *job_id = 0;
    CYCLES_UNAVAILABLE("gpu_submit_extract_cycles");
}
MTB_API int32_t gpu_try_get_cycles(int64_t, double *, int32_t, int32_t, int32_t *out_len, int32_t *ready) {
    if (out_len) *out_len = 0;
    if (ready) *ready = 0;
    CYCLES_UNAVAILABLE("gpu_try_get_cycles");
}
MTB_API int32_t gpu_submit_extract_cycles_batch(const double *, int32_t, int32_t, int32_t, int32_t, double, double,
                                                double, int32_t, int32_t, int32_t, int64_t *job_id) {
    if (job_id) *job_id = 0;
    CYCLES_UNAVAILABLE("gpu_submit_extract_cycles_batch");
}
MTB_API int32_t gpu_try_get_cycles_batch(int64_t, double *, int32_t, int32_t *out_len, int32_t *ready) {
    if (out_len) *out_len = 0;
    if (ready) *ready = 0;
    CYCLES_UNAVAILABLE("gpu_try_get_cycles_batch");
}

MTB_API int32_t gpu_get_last_error_w(uint16_t *buf, int32_t buf_len) {
    const std::string &e = t_last_error;
    if (!buf || buf_len <= 0 || e.empty()) return 0;
    const int32_t n = (int32_t)std::min<size_t>(e.size(), (size_t)buf_len - 1);
    for (int32_t i = 0; i < n; ++i) buf[i] = (uint16_t)(unsigned char)e[i];
    buf[n] = 0;
    return n + 1;
}

// ---- device-resident plans -------------------------------------------------
static int64_t plan_register(std::shared_ptr<Plan> p) {
    const int64_t id = g_next_id.fetch_add(1);
    std::lock_guard<std::mutex> lk(g_plans_mu);
    (*g_plans)[id] = std::move(p);
    return id;
}

static bool plan_device_ok(int32_t device) {
    const int n = device_count();
    if (n <= 0) {
        set_error("no HIP device visible; the spectrum path has no CPU fallback");
        return false;
    }
    if (device < 0 || device >= n) {
        set_error("device %d out of range (%d devices)", device, n);
        return false;
    }
    return true;
}

MTB_API int64_t wsp_plan_create(int32_t device, int32_t window_len, int64_t hop, int64_t n_windows, int32_t detrend,
                                int32_t window, int32_t trend_period, int32_t precision, int32_t output) {
    if (!plan_device_ok(device)) return 0;
    auto p = std::make_shared<Plan>();
    if (make_config(window_len, hop, n_windows, detrend, window, trend_period, precision, output, &p->cfg) != MTB_OK)
        return 0;
    p->dev = device;
    {
        std::lock_guard<std::mutex> lk(g_kalman_mu);
        memcpy(p->kalman, g_kalman, sizeof(g_kalman));
    }
    Tables t;
    if (get_tables(device, p->cfg.log2n, p->cfg.f32, &t) != MTB_OK) return 0;
    if (plan_ws_fit(*p) != MTB_OK) return 0;
    return plan_register(std::move(p));
}

MTB_API int64_t wsp_plan_create_inverse(int32_t device, int32_t window_len, int64_t n_windows) {
    if (!plan_device_ok(device)) return 0;
    auto p = std::make_shared<Plan>();
    if (make_config(window_len, window_len, n_windows, MTB_DETREND_NONE, MTB_WINDOW_NONE, 0, MTB_PREC_F64,
                    MTB_OUT_PACKED, &p->cfg) != MTB_OK)
        return 0;
    p->cfg.op = kOpInverse;
    if (p->cfg.log2n > kMaxLog2N) {
        set_error("window_len=%d: the inverse transform covers windows up to %d", window_len, 1 << kMaxLog2N);
        return 0;
    }
    p->dev = device;
    Tables t;
    if (get_tables(device, p->cfg.log2n, false, &t) != MTB_OK) return 0;
    return plan_register(std::move(p));
}

MTB_API int32_t wsp_plan_execute(int64_t plan, const void *d_series, void *d_out, void *hip_stream) {
    std::shared_ptr<Plan> p = find_plan(plan);  // keeps the plan (and its workspace) alive through the enqueue
    if (!p) {
        set_error("unknown plan %lld", (long long)plan);
        return MTB_BAD_ARGS;
    }
    if (!d_series || !d_out) {
        set_error("wsp_plan_execute: null device buffer");
        return MTB_BAD_ARGS;
    }
    const hipStream_t stream = (hipStream_t)hip_stream;
    Config c;
    std::shared_ptr<void> ws;
    {
        std::lock_guard<std::mutex> lk(p->mu);
        c = p->cfg;
        ws = p->ws;
        if (ws) {  // stateful on the device: ordered after the previous execute (struct Plan)
            if (!p->done) {
                if (hipSetDevice(p->dev) != hipSuccess || hipEventCreateWithFlags(&p->done, hipEventDisableTiming) != hipSuccess) {
                    p->done = nullptr;
                    set_error("wsp_plan_execute: cannot create the plan's event");
                    return MTB_INTERNAL_ERROR;
                }
            }
            // always (as for the counter slots): a destroyed stream's handle can come back as a new stream's
            if (p->done_recorded) HIP_OR(hipStreamWaitEvent(stream, p->done, 0), MTB_INTERNAL_ERROR);
            const int st = enqueue(p->dev, c, p->kalman, d_series, d_out, ws.get(), stream);
            if (st != MTB_OK) return st;
            HIP_OR(hipEventRecord(p->done, stream), MTB_INTERNAL_ERROR);
            p->done_recorded = true;
            return MTB_OK;
        }
    }
    return enqueue(p->dev, c, p->kalman, d_series, d_out, nullptr, stream);
}

MTB_API int32_t wsp_plan_set_topk(int64_t plan, int32_t top_k, double min_period, double max_period) {
    std::shared_ptr<Plan> p = find_plan(plan);
    if (!p) {
        set_error("unknown plan %lld", (long long)plan);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->cfg.op != kOpSpectrum) {
        set_error("plan %lld is not a spectrum plan", (long long)plan);
        return MTB_BAD_ARGS;
    }
    Config c = p->cfg;  // applied only when valid
    const int st = config_set_topk(&c, top_k, min_period, max_period);
    if (st != MTB_OK) return st;
    const Config old = p->cfg;
    p->cfg = c;
    const int sw = plan_ws_fit(*p);
    if (sw != MTB_OK) p->cfg = old;
    return sw;
}

MTB_API int32_t wsp_plan_set_algorithm(int64_t plan, int32_t algo) {
    std::shared_ptr<Plan> p = find_plan(plan);
    if (!p) {
        set_error("unknown plan %lld", (long long)plan);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    if (algo < MTB_ALGO_AUTO || algo > MTB_ALGO_SLIDE) {
        set_error("algorithm %d: MTB_ALGO_AUTO, MTB_ALGO_FFT or MTB_ALGO_SLIDE", algo);
        return MTB_BAD_ARGS;
    }
    Config c = p->cfg;
    c.algo = algo;
    if (algo == MTB_ALGO_SLIDE && !slide_eligible(c) && !slide_topk_eligible(c)) {
        set_error("plan %lld: the sliding DFT takes hop = 1, N = 512..8192, detrend none/mean, a cosine window "
                  "and power output (or fp64 top-k records over at most 512 bins)", (long long)plan);
        return MTB_BAD_ARGS;
    }
    const Config old = p->cfg;
    p->cfg = c;
    const int sw = plan_ws_fit(*p);
    if (sw != MTB_OK) p->cfg = old;
    return sw;
}

MTB_API int32_t wsp_plan_set_variant(int64_t plan, int32_t variant) {
    std::shared_ptr<Plan> p = find_plan(plan);
    constexpr int kMaxVariant = 9;  // kernel forms of the ablations (wsp_internal.h)
    if (!p || variant < 0 || variant > kMaxVariant) {
        set_error("wsp_plan_set_variant(%lld, %d): unknown plan or variant outside 0..9", (long long)plan, variant);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    p->cfg.variant = variant;
    return MTB_OK;
}

MTB_API int32_t wsp_plan_set_scan_flags(int64_t plan, void *d_flags) {
    std::shared_ptr<Plan> p = find_plan(plan);
    if (!p) {
        set_error("wsp_plan_set_scan_flags(%lld): unknown plan", (long long)plan);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    p->cfg.scan_flags = static_cast<unsigned char *>(d_flags);
    return MTB_OK;
}


MTB_API int32_t wsp_plan_set_slide_segment(int64_t plan, int64_t windows) {
    std::shared_ptr<Plan> p = find_plan(plan);
    if (!p || windows < 0 || windows > kSlideMaxSegment) {
        set_error("wsp_plan_set_slide_segment(%lld, %lld): unknown plan or length outside 0..%lld", (long long)plan,
                  (long long)windows, (long long)kSlideMaxSegment);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    const Config old = p->cfg;
    p->cfg.slide_seg = windows;
    const int sw = plan_ws_fit(*p);
    if (sw != MTB_OK) p->cfg = old;
    return sw;
}

MTB_API int32_t wsp_plan_set_seed_chain(int64_t plan, int32_t segments) {
    std::shared_ptr<Plan> p = find_plan(plan);
    if (!p || segments < 0 || segments > 16) {
        set_error("wsp_plan_set_seed_chain(%lld, %d): unknown plan or chain outside 0..16", (long long)plan, segments);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    p->cfg.seed_chain = segments;
    return MTB_OK;
}

MTB_API int32_t wsp_plan_set_trace(int64_t plan, void *d_trace, int64_t capacity) {
    std::shared_ptr<Plan> p = find_plan(plan);
    if (!p || capacity < 0 || (capacity > 0 && !d_trace)) {
        set_error("wsp_plan_set_trace(%lld): unknown plan or null buffer", (long long)plan);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    p->cfg.trace = capacity > 0 ? static_cast<long long *>(d_trace) : nullptr;
    p->cfg.trace_cap = capacity;
    return MTB_OK;
}

MTB_API int32_t wsp_plan_set_chunk(int64_t plan, int64_t windows) {
    std::shared_ptr<Plan> p = find_plan(plan);
    if (!p || windows < 0 || windows > (int64_t(1) << 20)) {
        set_error("wsp_plan_set_chunk(%lld, %lld): unknown plan or windows outside 0..2^20", (long long)plan,
                  (long long)windows);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    const Config old = p->cfg;
    p->cfg.chunk = windows;
    const int sw = plan_ws_fit(*p);
    if (sw != MTB_OK) p->cfg = old;
    return sw;
}

MTB_API int32_t wsp_plan_set_grid(int64_t plan, int32_t workgroups) {
    std::shared_ptr<Plan> p = find_plan(plan);
    if (!p || workgroups < 0 || workgroups > 65536) {
        set_error("wsp_plan_set_grid(%lld, %d): unknown plan or workgroups outside 0..65536", (long long)plan, workgroups);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    p->cfg.grid = workgroups;
    return MTB_OK;
}

MTB_API int32_t wsp_plan_get_algorithm(int64_t plan) {
    std::shared_ptr<Plan> p = find_plan(plan);
    if (!p) return MTB_BAD_ARGS;
    std::lock_guard<std::mutex> lk(p->mu);
    return (use_slide(p->cfg) || use_slide_topk(p->cfg)) ? MTB_ALGO_SLIDE : MTB_ALGO_FFT;
}

MTB_API int64_t wsp_plan_algorithmic_bytes(int64_t plan) {
    std::shared_ptr<Plan> p = find_plan(plan);
    if (!p) return -1;
    std::lock_guard<std::mutex> lk(p->mu);
    const Config &c = p->cfg;
    return (c.unique_input_elems() + c.n_windows * c.record()) * (int64_t)c.elem();
}

MTB_API int32_t wsp_plan_destroy(int64_t plan) {
    std::shared_ptr<Plan> p;
    {
        std::lock_guard<std::mutex> lk(g_plans_mu);
        auto it = g_plans->find(plan);
        if (it == g_plans->end()) {
            set_error("unknown plan %lld", (long long)plan);
            return MTB_BAD_ARGS;
        }
        p = std::move(it->second);
        g_plans->erase(it);
    }
    p.reset();  // the last reference (here, or an execute in flight) retires the workspace
    ws_reap();
    return MTB_OK;
}

MTB_API int64_t wsp_group_create(int32_t device, int32_t n_members, const int32_t *window_len, const int64_t *n_windows,
                                 int32_t detrend, int32_t window, int32_t precision) {
    if (!plan_device_ok(device)) return 0;
    if (n_members < 1 || n_members > 4096 || !window_len || !n_windows) {
        set_error("wsp_group_create: n_members=%d (1..4096) and non-null window_len / n_windows arrays needed", n_members);
        return 0;
    }
    auto g = std::make_shared<Group>();
    g->dev = device;
    std::map<int, std::vector<int>, std::greater<int>> by_len;  // longest first
    for (int m = 0; m < n_members; ++m) {
        Config c;
        if (make_config(window_len[m], 1, n_windows[m], detrend, window, 0, precision, MTB_OUT_POWER, &c) != MTB_OK) return 0;
        if (!slide_eligible(c)) {
            set_error("wsp_group_create: member %d (window_len=%d, detrend=%d, window=%d) is not a sliding-DFT batch "
                      "(window_len 512..8192, detrend none / mean, Hann / Hamming / Blackman / none)",
                      m, window_len[m], detrend, window);
            return 0;
        }
        Tables t;
        SlideArgs A{};
        if (get_tables(device, c.log2n, c.f32, &t) != MTB_OK || slide_args(device, c, &A) != MTB_OK) return 0;
        g->cfg.push_back(c);
        by_len[c.n].push_back(m);
    }
    for (auto &kv : by_len)
        for (size_t i = 0; i < kv.second.size(); i += kSlideGroupMax) {
            g->launch.emplace_back(kv.second.begin() + i,
                                   kv.second.begin() + std::min(kv.second.size(), i + (size_t)kSlideGroupMax));
            int64_t b = 0;
            for (int m : g->launch.back()) b += g->cfg[m].n_windows * g->cfg[m].record() * (int64_t)g->cfg[m].elem();
            g->launch_bytes.push_back(b);
        }
    g->mix_ok = (int)g->cfg.size() <= kMixMax;
    for (const Config &c : g->cfg)
        g->mix_ok = g->mix_ok && c.log2n >= 9 && c.log2n <= 12 && window_coef(c.window).nf <= 3;
    if (g->mix_ok) {
        if (hipSetDevice(device) != hipSuccess || hipMalloc(&g->ctr, 2 * kMixSlots * sizeof(int)) != hipSuccess ||
            hipMemset(g->ctr, 0, 2 * kMixSlots * sizeof(int)) != hipSuccess) {
            set_error("wsp_group_create: task counters could not be allocated");
            return 0;
        }
    }
    // per-length form: the launches run side by side, one lane each, up to 4 lanes (the HIP hardware queues a
    // process gets): C5 0.705-0.709 -> 0.669-0.671 ms against one lane (profiles/r03/s2/c5_lanes.log)
    {
        std::lock_guard<std::mutex> glk(g->mu);
        const int lanes = (int)std::min<size_t>(g->launch.size(), 4);
        if (lanes > 1 && group_lanes(*g, lanes) != MTB_OK) return 0;
    }
    const int64_t id = g_next_id.fetch_add(1);
    std::lock_guard<std::mutex> lk(g_groups_mu);
    (*g_groups)[id] = std::move(g);
    return id;
}

MTB_API int32_t wsp_group_execute(int64_t group, const void *const *d_series, void *const *d_out, void *hip_stream) {
    std::shared_ptr<Group> g = find_group(group);
    if (!g) {
        set_error("unknown group %lld", (long long)group);
        return MTB_BAD_ARGS;
    }
    if (!d_series || !d_out) {
        set_error("wsp_group_execute: null member array");
        return MTB_BAD_ARGS;
    }
    for (size_t m = 0; m < g->cfg.size(); ++m)
        if (!d_series[m] || !d_out[m]) {
            set_error("wsp_group_execute: member %zu has a null device buffer", m);
            return MTB_BAD_ARGS;
        }
    std::lock_guard<std::mutex> lk(g->mu);
    const hipStream_t caller = (hipStream_t)hip_stream;
    if (g->mix_ok && g->mode != 1) {
        HIP_OR(hipSetDevice(g->dev), MTB_BACKEND_UNAVAILABLE);
        return group_execute_mixed(*g, d_series, d_out, caller);
    }
    // wsp_group_set_streams(n > 1): the launches run side by side on n lanes -- the caller's stream and n - 1
    // internal streams (n HIP hardware queues in all) -- assigned greedily by output bytes, longest first, and
    // each lane's launches sized for the lane's share of the resident workgroup slots (its bytes / all bytes),
    // so that the lanes finish together and one length's seed phase and drain overlap the others' slides
    const int ns = g->streams.empty() ? 1 : (int)g->streams.size();
    HIP_OR(hipSetDevice(g->dev), MTB_BACKEND_UNAVAILABLE);
    std::vector<int> lane(g->launch.size(), 0);
    std::vector<int64_t> load(ns, 0);
    int64_t all = 0;
    for (size_t li = 0; li < g->launch.size(); ++li) {  // longest windows first; greedy by output bytes
        const int k = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        lane[li] = k;
        load[k] += g->launch_bytes[li];
        all += g->launch_bytes[li];
    }
    auto lane_stream = [&](int k) { return k == 0 ? caller : g->streams[k - 1]; };
    if (ns > 1) {
        HIP_OR(hipEventRecord(g->events[0], caller), MTB_INTERNAL_ERROR);
        for (int k = 1; k < ns; ++k) HIP_OR(hipStreamWaitEvent(lane_stream(k), g->events[0], 0), MTB_INTERNAL_ERROR);
    }
    for (size_t li = 0; li < g->launch.size(); ++li) {
        const auto &L = g->launch[li];
        SlideArgs A{};
        const int st = slide_args(g->dev, g->cfg[L[0]], &A);
        if (st != MTB_OK) return st;
        A.seg = g->seg;
        A.share = ns > 1 && load[lane[li]] > 0 ? (double)all / (double)load[lane[li]] : 1.0;
        SlideGroup G;
        G.n = (int)L.size();
        for (int i = 0; i < G.n; ++i) {
            G.series[i] = d_series[L[i]];
            G.out[i] = d_out[L[i]];
            G.n_windows[i] = g->cfg[L[i]].n_windows;
        }
        HIP_OR(launch_slide_group(A, G, lane_stream(lane[li])), MTB_INTERNAL_ERROR);
    }
    if (ns > 1)
        for (int k = 1; k < ns; ++k) {
            HIP_OR(hipEventRecord(g->events[k], lane_stream(k)), MTB_INTERNAL_ERROR);
            HIP_OR(hipStreamWaitEvent(caller, g->events[k], 0), MTB_INTERNAL_ERROR);
        }
    return MTB_OK;
}

MTB_API int32_t wsp_group_set_streams(int64_t group, int32_t n_streams) {
    std::shared_ptr<Group> g = find_group(group);
    if (!g || n_streams < 1 || n_streams > 8) {
        set_error("wsp_group_set_streams(%lld, %d): unknown group or n_streams outside 1..8", (long long)group, n_streams);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(g->mu);
    return group_lanes(*g, n_streams);
}

MTB_API int32_t wsp_group_set_segment(int64_t group, int64_t windows) {
    std::shared_ptr<Group> g = find_group(group);
    if (!g || windows < 0 || windows > kSlideMaxSegment) {
        set_error("wsp_group_set_segment(%lld, %lld): unknown group or length outside 0..%lld", (long long)group,
                  (long long)windows, (long long)kSlideMaxSegment);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(g->mu);
    g->seg = windows;
    return MTB_OK;
}

MTB_API int64_t wsp_group_algorithmic_bytes(int64_t group) {
    std::shared_ptr<Group> g = find_group(group);
    if (!g) return -1;
    int64_t b = 0;
    for (const Config &c : g->cfg) b += (c.unique_input_elems() + c.n_windows * c.record()) * (int64_t)c.elem();
    return b;
}

MTB_API int32_t wsp_group_launches(int64_t group) {
    std::shared_ptr<Group> g = find_group(group);
    if (!g) return -1;
    std::lock_guard<std::mutex> lk(g->mu);
    return g->mix_ok && g->mode != 1 ? 1 : (int32_t)g->launch.size();
}

MTB_API int32_t wsp_group_set_mode(int64_t group, int32_t mode) {
    std::shared_ptr<Group> g = find_group(group);
    if (!g || mode < 0 || mode > 6) {
        set_error("wsp_group_set_mode(%lld, %d): unknown group or mode outside 0..6", (long long)group, mode);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(g->mu);
    g->mode = mode;
    return MTB_OK;
}

MTB_API int32_t wsp_group_set_trace(int64_t group, void *d_trace, int64_t capacity_tasks) {
    std::shared_ptr<Group> g = find_group(group);
    if (!g || capacity_tasks < 0 || (capacity_tasks > 0 && !d_trace)) {
        set_error("wsp_group_set_trace(%lld): unknown group or null buffer", (long long)group);
        return MTB_BAD_ARGS;
    }
    std::lock_guard<std::mutex> lk(g->mu);
    g->trace = capacity_tasks ? static_cast<long long *>(d_trace) : nullptr;
    g->trace_cap = capacity_tasks;
    return MTB_OK;
}

MTB_API int64_t wsp_group_last_tasks(int64_t group) {
    std::shared_ptr<Group> g = find_group(group);
    if (!g) return -1;
    std::lock_guard<std::mutex> lk(g->mu);
    return g->last_tasks;
}

MTB_API int32_t wsp_group_destroy(int64_t group) {
    std::lock_guard<std::mutex> lk(g_groups_mu);
    if (!g_groups->erase(group)) {
        set_error("unknown group %lld", (long long)group);
        return MTB_BAD_ARGS;
    }
    return MTB_OK;
}

}  // extern "C"
