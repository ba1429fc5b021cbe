// multidev.cpp -- the library's own multi-GPU sharding (gpu_init(-1): every visible GPU, batch windows
// split across them) driven on the fake runtime with WSP_FAKE_DEVICES = 2 or 8 devices, under
// the sanitizer builds (tests/hostsan/Makefile).  No GPU: fake_hip.cpp tags streams and device buffers
// with the device current at their creation and counts, per device, the windows its launches computed.
// Checked, batch by batch (synchronous and submit / poll / free, from several threads at once):
//   * every record equals the fake kernels' function of its own window's samples (record element k of
//     window w = x[w*hop + k % N] + k): each device's input slice carries the N - hop halo, and the
//     devices' output ranges are disjoint and complete;
//   * the window split: device g computes windows [g*ceil(W/G'), ...), G' = min(devices, W), i.e. the
//     per-device window counts the library's batch_start promises (include/mtbridge.h gpu_init);
//   * no copy or launch touches a stream or buffer of another device than the one current on the
//     enqueuing thread (per-device streams and buffers).
// Usage: multidev <lib.so> <devices>.  Exit 0 = all good.
#include <dlfcn.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mtbridge.h"

namespace {
struct Api {
    decltype(&gpu_init) init;
    decltype(&gpu_shutdown) shutdown;
    decltype(&gpu_spectrum_batch) batch;
    decltype(&gpu_submit_spectrum_batch) submit;
    decltype(&gpu_try_get_spectrum_batch) try_get;
    decltype(&gpu_free_job) free_job;
    decltype(&wsp_plan_create) plan_create;
    decltype(&wsp_plan_destroy) plan_destroy;
    void (*reset)(void);
    int64_t (*windows)(int);
    int64_t (*violations)(void);
} A;
std::atomic<int> g_fail{0};

#define CHECK(c, ...)                                           \
    do {                                                        \
        if (!(c)) {                                             \
            fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                       \
            fprintf(stderr, "\n");                              \
            g_fail++;                                           \
        }                                                       \
    } while (0)

template <typename F> void sym(void *h, F &f, const char *n) {
    f = reinterpret_cast<F>(dlsym(h, n));
    if (!f) {
        fprintf(stderr, "missing %s\n", n);
        exit(3);
    }
}

std::vector<double> series_of(int seed, int len) {
    std::vector<double> s(len);
    for (int i = 0; i < len; ++i) s[i] = 1.0 + 0.01 * seed + 1e-6 * (double)(((int64_t)i * 7919 + seed) % 1000);
    return s;
}

int record_of(int n, int output) { return output == MTB_OUT_PACKED ? n : n / 2; }

bool check_records(const std::vector<double> &s, const std::vector<double> &out, int n, int hop, int nwin, int rec,
                   int f32) {
    for (int w = 0; w < nwin; ++w)
        for (int k = 0; k < rec; ++k) {
            double want = s[(size_t)w * hop + k % n];
            if (f32) want = (double)((float)want + (float)k);  // the fp32 plan's arithmetic
            else want += (double)k;
            if (out[(size_t)w * rec + k] != want) {
                fprintf(stderr, "record w=%d k=%d: %.17g != %.17g\n", w, k, out[(size_t)w * rec + k], want);
                return false;
            }
        }
    return true;
}

struct Case {
    int n, hop, nwin, detrend, output, prec;
};

// one synchronous batch on the whole machine; checks records and the per-device window split
void one_sync(const Case &c, int devices, int seed) {
    const int len = (c.nwin - 1) * c.hop + c.n, rec = record_of(c.n, c.output);
    const std::vector<double> s = series_of(seed, len);
    std::vector<double> out((size_t)c.nwin * rec, -1.0);
    A.reset();
    int got = 0;
    const int st = A.batch(s.data(), len, c.n, c.hop, c.detrend, MTB_WINDOW_HANN, 64, c.prec, c.output, out.data(),
                           (int)out.size(), &got);
    CHECK(st == MTB_OK && got == c.nwin, "batch n=%d hop=%d nwin=%d: st %d got %d", c.n, c.hop, c.nwin, st, got);
    CHECK(check_records(s, out, c.n, c.hop, c.nwin, rec, c.prec == MTB_PREC_F32), "records n=%d hop=%d nwin=%d", c.n,
          c.hop, c.nwin);
    const int g_used = c.nwin < devices ? c.nwin : devices;
    const int64_t per = (c.nwin + g_used - 1) / g_used;
    int64_t sum = 0;
    for (int g = 0; g < devices; ++g) {
        int64_t want = g < g_used ? std::min<int64_t>(per, c.nwin - g * per) : 0;
        if (want < 0) want = 0;
        const int64_t have = A.windows(g);
        CHECK(have == want, "n=%d nwin=%d: device %d computed %lld windows, expected %lld", c.n, c.nwin, g, (long long)have,
              (long long)want);
        sum += have;
    }
    CHECK(sum == c.nwin, "windows over all devices %lld != %d", (long long)sum, c.nwin);
    CHECK(A.violations() == 0, "n=%d nwin=%d: %lld cross-device operations", c.n, c.nwin, (long long)A.violations());
}

// a chart thread: jobs through submit / poll / free on the sharded session (records checked)
void chart(int id, int rounds) {
    CHECK(A.init(-1, 16) == MTB_OK, "init chart %d", id);
    const int n = 128 << (id % 3), hop = 1 + id % 5, nwin = 300 + 97 * id, len = (nwin - 1) * hop + n, rec = n / 2;
    const std::vector<double> s = series_of(100 + id, len);
    std::vector<double> out((size_t)nwin * rec);
    for (int r = 0; r < rounds; ++r) {
        int64_t jid = 0;
        CHECK(A.submit(s.data(), len, n, hop, MTB_DETREND_NONE, MTB_WINDOW_HANN, 0, MTB_PREC_F64, MTB_OUT_POWER, &jid) ==
                      MTB_OK && jid > 0,
              "submit chart %d", id);
        int ready = 0, got = 0, st = MTB_OK;
        for (int tries = 0; tries < 100000 && ready == 0; ++tries) {  // WaveCyclesBatchFetcher.mq5:127-131
            st = A.try_get(jid, out.data(), (int)out.size(), &got, &ready);
            if (st == MTB_OK && ready == 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
            else if (st != MTB_OK && st != MTB_NOT_READY) break;
        }
        CHECK(st == MTB_OK && ready == 1 && got == nwin, "poll chart %d: st %d ready %d got %d", id, st, ready, got);
        CHECK(check_records(s, out, n, hop, nwin, rec, 0), "records chart %d round %d", id, r);
        CHECK(A.free_job(jid) == MTB_OK, "free chart %d", id);
    }
    A.shutdown();
}
}  // namespace

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    const int devices = atoi(argv[2]);
    setenv("WSP_FAKE_DEVICES", argv[2], 1);
    void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        fprintf(stderr, "dlopen: %s\n", dlerror());
        return 3;
    }
    sym(h, A.init, "gpu_init");
    sym(h, A.shutdown, "gpu_shutdown");
    sym(h, A.batch, "gpu_spectrum_batch");
    sym(h, A.submit, "gpu_submit_spectrum_batch");
    sym(h, A.try_get, "gpu_try_get_spectrum_batch");
    sym(h, A.free_job, "gpu_free_job");
    sym(h, A.plan_create, "wsp_plan_create");
    sym(h, A.plan_destroy, "wsp_plan_destroy");
    sym(h, A.reset, "fakehip_reset");
    sym(h, A.windows, "fakehip_windows");
    sym(h, A.violations, "fakehip_violations");

    CHECK(A.init(-1, 8) == MTB_OK, "gpu_init(-1) over %d devices", devices);
    const Case cases[] = {
        {256, 37, 1001, MTB_DETREND_NONE, MTB_OUT_POWER, MTB_PREC_F64},     // overlapping, odd hop: halo N - hop
        {1024, 1, 5000, MTB_DETREND_NONE, MTB_OUT_POWER, MTB_PREC_F64},     // hop = 1 (C4 / C5 shape)
        {512, 512, 3, MTB_DETREND_NONE, MTB_OUT_POWER, MTB_PREC_F64},       // fewer windows than devices
        {512, 700, 41, MTB_DETREND_MEAN, MTB_OUT_PACKED, MTB_PREC_F64},     // gaps between windows, packed
        {1024, 1024, 333, MTB_DETREND_KALMAN, MTB_OUT_POWER, MTB_PREC_F32}, // Kalman pre-pass workspace per device
        {256, 64, 777, MTB_DETREND_IIR, MTB_OUT_POWER, MTB_PREC_F64},
        {32768, 32768, 11, MTB_DETREND_NONE, MTB_OUT_POWER, MTB_PREC_F64},  // large N (four-step path)
    };
    int seed = 0;
    for (const Case &c : cases) one_sync(c, devices, ++seed);
    // concurrent charts on the sharded session, then the checks again with the jobs gone
    std::vector<std::thread> th;
    for (int c = 0; c < 8; ++c) th.emplace_back(chart, c, 4);
    for (auto &t : th) t.join();
    one_sync(cases[0], devices, 99);
    // device plans address one device each: every device accepts one, one past the end is refused
    for (int g = 0; g < devices; ++g) {
        const int64_t p = A.plan_create(g, 1024, 1024, 64, MTB_DETREND_NONE, MTB_WINDOW_HANN, 0, MTB_PREC_F64, MTB_OUT_POWER);
        CHECK(p > 0 && A.plan_destroy(p) == MTB_OK, "plan on device %d", g);
    }
    CHECK(A.plan_create(devices, 1024, 1024, 64, MTB_DETREND_NONE, MTB_WINDOW_HANN, 0, MTB_PREC_F64, MTB_OUT_POWER) == 0,
          "plan on device %d (past the end) refused", devices);
    A.shutdown();
    printf("hostsan multidev %d: %s (%d failures)\n", devices, g_fail ? "FAIL" : "ok", g_fail.load());
    return g_fail ? 1 : 0;
}
