// fake_hip.cpp -- TEST DOUBLE of the HIP runtime calls and kernel launches that
// fft-wavespec_amd/csrc/mtbridge.cpp makes, for sanitizer builds of the host
// layer on a machine without a GPU ("TSAN on the host harness, ASAN
// builds").  Never linked into the product: tests/hostsan/Makefile builds
// mtbridge.cpp + this file into a separate libmtbridge_{tsan,asan}.so.
//
// Streams are real asynchronous queues (one worker thread each), so copies,
// "kernels" and event completions run concurrently with the calling threads,
// as on the device: the sanitizers see the same cross-thread hand-offs as the
// real runtime would impose (job copy-out vs completion, session teardown vs
// calls in flight, plan destroy vs execute).  "Device" memory is host memory.
// The launch stubs write a deterministic function of each window's own input
// samples, so a driver can check that every record was routed to the right
// place: record element k of window w = series[w*hop + k % N] + k.
//
// Devices: WSP_FAKE_DEVICES (default 1).  Streams, events and hipMalloc'd
// blocks remember the device current at their creation; every copy and launch
// checks that its stream and every device buffer it touches belong to the
// device current on the calling thread (a part of a multi-GPU batch enqueued on
// another device's stream or buffer counts as a violation), and launches count
// the windows each device computed (fakehip_windows / fakehip_violations,
// driven by multidev.cpp).
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <initializer_list>
#include <map>
#include <mutex>
#include <set>
#include <thread>

#include "../../fft-wavespec_amd/csrc/wsp_internal.h"

struct ihipStream_t {
    int dev = 0;
    std::mutex mu;
    std::condition_variable cv, idle;
    std::deque<std::function<void()>> q;
    bool stop = false, busy = false;
    std::thread worker;
    ihipStream_t() {
        worker = std::thread([this] {
            std::unique_lock<std::mutex> lk(mu);
            for (;;) {
                cv.wait(lk, [this] { return stop || !q.empty(); });
                if (q.empty() && stop) break;
                auto f = std::move(q.front());
                q.pop_front();
                busy = true;
                lk.unlock();
                f();
                lk.lock();
                busy = false;
                if (q.empty()) idle.notify_all();
            }
        });
    }
    void push(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> lk(mu);
            q.push_back(std::move(f));
        }
        cv.notify_one();
    }
    void drain() {
        std::unique_lock<std::mutex> lk(mu);
        idle.wait(lk, [this] { return q.empty() && !busy; });
    }
    ~ihipStream_t() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_one();
        worker.join();
    }
};

struct ihipEvent_t {
    std::mutex mu;
    std::condition_variable cv;
    uint64_t recorded = 0, reached = 0;
};

namespace {
std::mutex g_streams_mu;
std::deque<ihipStream_t *> g_streams;  // live streams, for hipDeviceSynchronize
thread_local int t_device = 0;
int n_devices() {
    const char *e = getenv("WSP_FAKE_DEVICES");
    return e ? atoi(e) : 1;
}
// the null stream: executes synchronously on the caller
void run_on(hipStream_t s, std::function<void()> f) {
    if (s) s->push(std::move(f));
    else f();
}
// device memory: base -> (bytes, device)
std::mutex g_alloc_mu;
std::map<uintptr_t, std::pair<size_t, int>> g_allocs;
int dev_of(const void *p) {  // -1: not device memory (host, pinned or registered)
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    auto it = g_allocs.upper_bound(a);
    if (it == g_allocs.begin()) return -1;
    --it;
    return a < it->first + it->second.first ? it->second.second : -1;
}
// Round 6: the library never page-locks caller memory (gpu_set_host_locking(1) withdrawn) and
// every host <-> device copy it makes goes through its own pinned (hipHostMalloc) buffers.  Any hipHostRegister /
// hipHostUnregister call counts as a violation, and a copy whose host side is not hipHostMalloc'd memory counts
// as a direct copy of caller memory (fakehip_direct_copies, which the stress driver requires to stay 0).
std::atomic<int64_t> g_direct{0};
// hipHostMalloc'd blocks: base -> bytes
std::mutex g_pinned_mu;
std::map<uintptr_t, size_t> g_pinned;
bool host_locked(const void *p) {
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> lk(g_pinned_mu);
    auto it = g_pinned.upper_bound(a);
    if (it == g_pinned.begin()) return false;
    --it;
    return a < it->first + it->second;
}
constexpr int kMaxDev = 64;
std::atomic<int64_t> g_windows[kMaxDev];
std::atomic<int64_t> g_violations{0};
// an operation enqueued on stream s touching the given buffers, on the thread's current device
void check_op(hipStream_t s, std::initializer_list<const void *> bufs, int64_t windows = 0) {
    const int d = t_device;
    bool bad = s && s->dev != d;
    for (const void *b : bufs) {
        const int bd = b ? dev_of(b) : -1;
        if (bd >= 0 && bd != d) bad = true;
    }
    if (bad) g_violations++;
    if (d >= 0 && d < kMaxDev) g_windows[d] += windows;
}
}  // namespace

extern "C" {
hipError_t hipGetDeviceCount(int *n) {
    *n = n_devices();
    return hipSuccess;
}
hipError_t hipSetDevice(int d) {
    if (d < 0 || d >= n_devices()) return hipErrorInvalidDevice;
    t_device = d;
    return hipSuccess;
}
hipError_t hipGetDevice(int *d) {
    *d = t_device;
    return hipSuccess;
}
hipError_t hipDeviceGetAttribute(int *v, hipDeviceAttribute_t attr, int d) {
    if (d < 0 || d >= n_devices()) return hipErrorInvalidDevice;
    *v = attr == hipDeviceAttributeMultiprocessorCount ? 256 : 0;  // an MI355X's CUs; nothing else is asked
    return hipSuccess;
}
hipError_t hipMalloc(void **p, size_t n) {
    *p = aligned_alloc(256, (n + 255) & ~size_t(255));
    if (!*p) return hipErrorOutOfMemory;
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    g_allocs[(uintptr_t)*p] = {n ? n : 1, t_device};
    return hipSuccess;
}
hipError_t hipFree(void *p) {
    {
        std::lock_guard<std::mutex> lk(g_alloc_mu);
        g_allocs.erase((uintptr_t)p);
    }
    free(p);
    return hipSuccess;
}
hipError_t hipHostMalloc(void **p, size_t n, unsigned int) {
    *p = aligned_alloc(256, (n + 255) & ~size_t(255));
    if (!*p) return hipErrorOutOfMemory;
    std::lock_guard<std::mutex> lk(g_pinned_mu);
    g_pinned[(uintptr_t)*p] = n ? n : 1;
    return hipSuccess;
}
hipError_t hipHostFree(void *p) {
    {
        std::lock_guard<std::mutex> lk(g_pinned_mu);
        g_pinned.erase((uintptr_t)p);
    }
    free(p);
    return hipSuccess;
}
hipError_t hipHostRegister(void *, size_t, unsigned int) {
    g_violations++;
    return hipErrorInvalidValue;
}
hipError_t hipHostUnregister(void *) {
    g_violations++;
    return hipErrorHostMemoryNotRegistered;
}
// pinned host memory: hipMemoryTypeHost; device memory: hipMemoryTypeDevice; anything else
// (pageable memory) an error, as the real runtime answers (scripts/hostreg_probe.py)
hipError_t hipPointerGetAttributes(hipPointerAttribute_t *attr, const void *p) {
    memset(attr, 0, sizeof(*attr));
    if (host_locked(p)) {
        attr->type = hipMemoryTypeHost;
        attr->hostPointer = const_cast<void *>(p);
        attr->devicePointer = const_cast<void *>(p);
        return hipSuccess;
    }
    const int d = dev_of(p);
    if (d >= 0) {
        attr->type = hipMemoryTypeDevice;
        attr->device = d;
        attr->devicePointer = const_cast<void *>(p);
        return hipSuccess;
    }
    return hipErrorInvalidValue;
}
hipError_t hipGetLastError(void) { return hipSuccess; }
hipError_t hipHostGetDevicePointer(void **d, void *h, unsigned int) {
    *d = h;
    return hipSuccess;
}
hipError_t hipMemcpy(void *d, const void *s, size_t n, hipMemcpyKind) {
    memcpy(d, s, n);
    return hipSuccess;
}
hipError_t hipMemset(void *d, int v, size_t n) {
    memset(d, v, n);
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void *d, const void *s, size_t n, hipMemcpyKind k, hipStream_t st) {
    check_op(st, {d, s});
    const void *host = k == hipMemcpyHostToDevice ? s : (k == hipMemcpyDeviceToHost ? d : nullptr);
    if (host && (!host_locked(host) || !host_locked((const char *)host + n - 1))) g_direct++;
    run_on(st, [=] { memcpy(d, s, n); });
    return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned int) {
    *s = new ihipStream_t();
    (*s)->dev = t_device;
    std::lock_guard<std::mutex> lk(g_streams_mu);
    g_streams.push_back(*s);
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t s) {
    if (s) s->drain();
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
    {
        std::lock_guard<std::mutex> lk(g_streams_mu);
        for (auto it = g_streams.begin(); it != g_streams.end(); ++it)
            if (*it == s) {
                g_streams.erase(it);
                break;
            }
    }
    s->drain();
    delete s;
    return hipSuccess;
}
hipError_t hipDeviceSynchronize(void) {
    {
        std::lock_guard<std::mutex> lk(g_streams_mu);
        for (auto *s : g_streams) s->drain();
    }
    return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned int) {
    *e = new ihipEvent_t();
    return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) {
    delete e;
    return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
    uint64_t gen;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        gen = ++e->recorded;
    }
    run_on(s, [e, gen] {
        {
            std::lock_guard<std::mutex> lk(e->mu);
            if (gen > e->reached) e->reached = gen;
        }
        e->cv.notify_all();
    });
    return hipSuccess;
}
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned int) {
    uint64_t gen;
    {
        std::lock_guard<std::mutex> lk(e->mu);
        gen = e->recorded;  // the most recent record at the time of the call
    }
    run_on(s, [e, gen] {
        std::unique_lock<std::mutex> lk(e->mu);
        e->cv.wait(lk, [e, gen] { return e->reached >= gen; });
    });
    return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t e) {
    std::lock_guard<std::mutex> lk(e->mu);
    return e->reached >= e->recorded ? hipSuccess : hipErrorNotReady;
}
hipError_t hipEventSynchronize(hipEvent_t e) {
    std::unique_lock<std::mutex> lk(e->mu);
    e->cv.wait(lk, [e] { return e->reached >= e->recorded; });
    return hipSuccess;
}
const char *hipGetErrorString(hipError_t e) { return e == hipSuccess ? "hipSuccess" : "fake hip error"; }

// test hooks (multidev.cpp): windows computed per device since the last reset, routing violations
void fakehip_reset(void) {
    for (auto &w : g_windows) w = 0;
    g_violations = 0;
}
int64_t fakehip_windows(int dev) { return dev >= 0 && dev < kMaxDev ? g_windows[dev].load() : -1; }
int64_t fakehip_violations(void) { return g_violations.load(); }
int64_t fakehip_direct_copies(void) { return g_direct.load(); }
int64_t fakehip_registered_ranges(void) { return 0; }  // nothing is ever page-locked (round 6)
}  // extern "C"

// ---- kernel launch stubs (wsp_internal.h): record element k of window w = x_w[k % N] + k
namespace wsp {
namespace {
template <typename T> void fill(const void *series, int64_t hop, int n, int64_t nw, int64_t rec, void *out) {
    const T *x = static_cast<const T *>(series);
    T *o = static_cast<T *>(out);
    for (int64_t w = 0; w < nw; ++w)
        for (int64_t k = 0; k < rec; ++k) o[w * rec + k] = x[w * hop + k % n] + (T)k;
}
int64_t record_of(int n, int output, int topk) {
    switch (output) {
    case kOutPacked: return n;
    case kOutTopK: return 4 * topk;
    case kOutPhase: return 3 * (n / 2);
    case kOutTopKPhase: return 6 * topk;
    default: return n / 2;
    }
}
}  // namespace

hipError_t launch_spectrum(const SpectrumLaunch &L, hipStream_t s) {
    check_op(s, {L.series, L.out, L.twiddle}, L.n_windows);
    const SpectrumLaunch c = L;
    run_on(s, [c] {
        const int n = 1 << c.log2n;
        const int64_t rec = record_of(n, c.output, c.topk);
        if (c.f32) fill<float>(c.series, c.hop, n, c.n_windows, rec, c.out);
        else fill<double>(c.series, c.hop, n, c.n_windows, rec, c.out);
    });
    return hipSuccess;
}
hipError_t launch_spectrum_f32(const SpectrumLaunch &L, hipStream_t s) { return launch_spectrum(L, s); }
hipError_t launch_slide_topk(const SlideArgs &a, hipStream_t s) {  // hop = 1 top-k records, same record function
    check_op(s, {a.series, a.out}, a.n_windows);
    const SlideArgs c = a;
    run_on(s, [c] { fill<double>(c.series, 1, 1 << c.log2n, c.n_windows, 4 * c.topk, c.out); });
    return hipSuccess;
}
hipError_t launch_slide(const SlideArgs &a, hipStream_t s) {  // hop = 1 power rows, same record function
    check_op(s, {a.series, a.out}, a.n_windows);
    const SlideArgs c = a;
    run_on(s, [c] {
        const int n = 1 << c.log2n;
        if (c.f32) fill<float>(c.series, 1, n, c.n_windows, n / 2, c.out);
        else fill<double>(c.series, 1, n, c.n_windows, n / 2, c.out);
    });
    return hipSuccess;
}
hipError_t launch_slide_group(const SlideArgs &a, const SlideGroup &g, hipStream_t s) {
    int64_t total = 0;
    for (int m = 0; m < g.n; ++m) {
        check_op(s, {g.series[m], g.out[m]});
        total += g.n_windows[m];
    }
    check_op(s, {}, total);
    const SlideArgs c = a;
    const SlideGroup gg = g;
    run_on(s, [c, gg] {
        const int n = 1 << c.log2n;
        for (int m = 0; m < gg.n; ++m) {
            if (c.f32) fill<float>(gg.series[m], 1, n, gg.n_windows[m], n / 2, gg.out[m]);
            else fill<double>(gg.series[m], 1, n, gg.n_windows[m], n / 2, gg.out[m]);
        }
    });
    return hipSuccess;
}
int slide_mix_resident(int, int, bool, int, int) { return 512; }
hipError_t launch_slide_mix(const SlideMix &m, int, int, bool f32, int grid, hipStream_t s) {  // every member, same records
    if (grid < 1 || m.nclass < 1 || m.n_tasks < 1 || !m.counter || !m.done) return hipErrorInvalidValue;
    int64_t total = 0;
    for (int i = 0; i < m.mem0[m.nclass]; ++i) {
        check_op(s, {m.series[i], m.out[i]});
        total += m.n_windows[i];
    }
    check_op(s, {}, total);
    const SlideMix c = m;
    run_on(s, [c, f32] {
        for (int k = 0; k < c.nclass; ++k) {
            const int n = 1 << c.log2n[k];
            for (int i = c.mem0[k]; i < c.mem0[k + 1]; ++i) {
                if (f32) fill<float>(c.series[i], 1, n, c.n_windows[i], n / 2, c.out[i]);
                else fill<double>(c.series[i], 1, n, c.n_windows[i], n / 2, c.out[i]);
            }
        }
    });
    return hipSuccess;
}
hipError_t launch_spectrum_phase(const SpectrumLaunch &L, hipStream_t s) { return launch_spectrum(L, s); }
hipError_t launch_kalman_detrend(const KalmanLaunch &L, hipStream_t s) {  // detrended = the window itself
    check_op(s, {L.series, L.detrended});
    const KalmanLaunch c = L;
    run_on(s, [c] {
        const size_t es = c.f32 ? 4 : 8;
        for (int64_t w = 0; w < c.n_windows; ++w)
            memcpy(static_cast<char *>(c.detrended) + (size_t)(w * c.n) * es,
                   static_cast<const char *>(c.series) + (size_t)(w * c.hop) * es, (size_t)c.n * es);
    });
    return hipSuccess;
}
// the real filter folds the window into its rows at N <= 4096 (kalman_kernels.hip); the fake never does, so the
// fake spectrum launch sees the plan's window as before
bool kalman_folds_window(const KalmanLaunch &) { return false; }
void kalman_pair_geometry(int n, int *l0, int *seg_off) {
    *l0 = (n + 256) / 2;
    *seg_off = *l0 - 256;
}
hipError_t launch_inverse(const InverseLaunch &L, hipStream_t s) {
    check_op(s, {L.in, L.out}, L.n_windows);
    const InverseLaunch c = L;
    run_on(s, [c] { fill<double>(c.in, int64_t(1) << c.log2n, 1 << c.log2n, c.n_windows, int64_t(1) << c.log2n, c.out); });
    return hipSuccess;
}
hipError_t launch_phase_row(const double *spec, int n_bins, int, double *out, hipStream_t s) {
    run_on(s, [=] { fill<double>(spec, 0, 2 * n_bins, 1, n_bins, out); });
    return hipSuccess;
}
hipError_t launch_large(const LargeLaunch &L, hipStream_t s) {
    check_op(s, {L.series, L.out}, L.n_windows);
    const LargeLaunch c = L;
    run_on(s, [c] {
        const int n = 1 << c.log2n;
        fill<double>(c.series, c.hop, n, c.n_windows, c.packed ? n : n / 2, c.out);
    });
    return hipSuccess;
}
int64_t large_chunk(int, bool) { return 64; }
}  // namespace wsp
