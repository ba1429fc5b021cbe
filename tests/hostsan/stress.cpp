// stress.cpp -- concurrency driver of the C ABI for the sanitizer builds
// (tests/hostsan/Makefile: mtbridge.cpp + the fake_hip.cpp test double, built
// with -fsanitize=thread or -fsanitize=address,undefined).  It dlopen()s the
// library like the MT5 terminal (Include/imports.mqh:4) and replays, from many
// threads at once, the call sequences the reference makes:
//   * 28 charts (WaveCyclesBatchFetcher.mq5:104-133 / 1.1.0:722-757, 706-716):
//     gpu_init, submit + poll + free batch jobs, per-bar gpu_fft_real_forward,
//     then gpu_shutdown -- half of them early, while the others keep working;
//   * a poller racing gpu_free_job on the same job;
//   * device plans executed while another thread re-targets (set_topk) and
//     destroys them;
//   * gpu_init on another device while the session is open (must be refused);
//   * grouped plans (wsp_group_*, the mixed-length launch and its per-length form) executed from
//     two threads while a third toggles the mode / segment and destroys them;
//   * pinned feeds (gpu_register_host): threads registering their series and
//     output arrays, running synchronous batches through them, unregistering,
//     and two threads racing to register overlapping ranges of one buffer;
//     buffers that neither start nor end on a page (only their whole inner
//     pages may be page-locked, the head / tail go through the bounce buffer).
// Every record is checked against the fake kernels' formula
// (record element k of window w = x[w*hop + k % N] + k).  Exit 0 = all good.
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/mtbridge.h"

namespace {
struct Api {
    decltype(&gpu_init) init;
    decltype(&gpu_shutdown) shutdown;
    decltype(&gpu_fft_real_forward) fft;
    decltype(&gpu_submit_spectrum_batch) submit;
    decltype(&gpu_try_get_spectrum_batch) try_get;
    decltype(&gpu_free_job) free_job;
    decltype(&gpu_spectrum_batch) batch;
    decltype(&wsp_plan_create) plan_create;
    decltype(&wsp_plan_execute) plan_execute;
    decltype(&wsp_plan_set_topk) plan_set_topk;
    decltype(&wsp_plan_destroy) plan_destroy;
    decltype(&gpu_register_host) reg;
    decltype(&gpu_unregister_host) unreg;
    decltype(&wsp_group_create) group_create;
    decltype(&wsp_group_execute) group_execute;
    decltype(&wsp_group_set_mode) group_set_mode;
    decltype(&wsp_group_set_segment) group_set_segment;
    decltype(&wsp_group_destroy) group_destroy;
} A;
std::atomic<int> g_fail{0};

#define CHECK(c, ...)                              \
    do {                                           \
        if (!(c)) {                                \
            fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);          \
            fprintf(stderr, "\n");                 \
            g_fail++;                              \
        }                                          \
    } while (0)

template <typename F> void sym(void *h, F &f, const char *n) {
    f = reinterpret_cast<F>(dlsym(h, n));
    if (!f) {
        fprintf(stderr, "missing %s\n", n);
        exit(3);
    }
}

std::vector<double> series_of(int sym, int len) {
    std::vector<double> s(len);
    for (int i = 0; i < len; ++i) s[i] = 1.0 + 0.001 * sym + 1e-6 * (double)((i * 7919) % 1000);
    return s;
}

bool check_records(const std::vector<double> &s, const double *out, int n, int hop, int nrec, int rec) {
    for (int w = 0; w < nrec; ++w)
        for (int k = 0; k < rec; ++k)
            if (out[(size_t)w * rec + k] != s[(size_t)w * hop + k % n] + (double)k) return false;
    return true;
}

// one chart: EnsureGpu, batch jobs + live per-bar calls, OnDeinit
void chart(int sym, bool early, std::atomic<int> &early_done, int rounds) {
    CHECK(A.init(0, 16) == MTB_OK, "init sym %d", sym);
    const int n = 64 << (sym % 4), hop = 1 + sym % 3, len = 40 * hop + n;
    const std::vector<double> s = series_of(sym, len);
    const int nwin = 1 + (len - n) / hop, rec = n / 2;
    std::vector<double> out((size_t)nwin * rec);
    for (int r = 0; r < rounds; ++r) {
        if (early && r == rounds / 2) {
            A.shutdown();  // this chart closes mid-way; the others must keep their session
            early_done++;
            return;
        }
        int64_t jid = 0;
        CHECK(A.submit(s.data(), len, n, hop, MTB_DETREND_NONE, MTB_WINDOW_HANN, 0, MTB_PREC_F64, MTB_OUT_POWER, &jid) == MTB_OK &&
                  jid > 0, "submit sym %d round %d", sym, r);
        int ready = 0, got = 0, st = MTB_NOT_READY;
        for (int p = 0; p < 100000 && !ready; ++p) {
            st = A.try_get(jid, out.data(), (int)out.size(), &got, &ready);
            if (!ready) std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        CHECK(st == MTB_OK && ready == 1 && got == nwin, "poll sym %d st %d ready %d got %d", sym, st, ready, got);
        CHECK(check_records(s, out.data(), n, hop, nwin, rec), "records sym %d round %d", sym, r);
        CHECK(A.free_job(jid) == MTB_OK, "free sym %d", sym);
        std::vector<double> win(s.begin(), s.begin() + n), packed(n);  // per-bar live call (1.1.0:1249)
        CHECK(A.fft(win.data(), n, packed.data()) == MTB_OK, "live sym %d", sym);
        CHECK(check_records(win, packed.data(), n, n, 1, n), "live records sym %d", sym);
    }
    A.shutdown();
}

void free_race() {  // try_get copying out while another thread frees the job
    CHECK(A.init(0, 16) == MTB_OK, "init");
    const int n = 256, len = 4096;
    const std::vector<double> s = series_of(99, len);
    for (int r = 0; r < 40; ++r) {
        int64_t jid = 0;
        CHECK(A.submit(s.data(), len, n, 1, MTB_DETREND_NONE, MTB_WINDOW_NONE, 0, MTB_PREC_F32, MTB_OUT_POWER, &jid) == MTB_OK,
              "submit");
        std::vector<double> out((size_t)(len - n + 1) * (n / 2));
        std::thread poller([&] {
            int ready = 0, got = 0;
            for (int p = 0; p < 2000; ++p) {
                const int st = A.try_get(jid, out.data(), (int)out.size(), &got, &ready);
                if (st == MTB_BAD_ARGS || ready) break;  // freed under us, or done
            }
        });
        std::this_thread::sleep_for(std::chrono::microseconds(20 * (r % 5)));
        CHECK(A.free_job(jid) == MTB_OK, "free");
        poller.join();
    }
    A.shutdown();
}

void plan_race() {  // execute vs set_topk vs destroy on shared plans
    const int n = 512, W = 64;
    std::vector<double> x((size_t)W * n, 1.5), y((size_t)W * n);
    for (int r = 0; r < 30; ++r) {
        const int64_t p = A.plan_create(0, n, n, W, MTB_DETREND_KALMAN, MTB_WINDOW_HANN, 0, MTB_PREC_F64, MTB_OUT_POWER);
        CHECK(p > 0, "plan_create");
        std::atomic<bool> stop{false};
        std::thread ex([&] {
            while (!stop) {
                const int st = A.plan_execute(p, x.data(), y.data(), nullptr);
                if (st == MTB_BAD_ARGS) break;  // destroyed
            }
        });
        std::thread tk([&] {
            for (int i = 0; i < 50 && !stop; ++i) A.plan_set_topk(p, 1 + i % 8, 18.0, 200.0);
        });
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        CHECK(A.plan_destroy(p) == MTB_OK, "destroy");
        stop = true;
        ex.join();
        tk.join();
        CHECK(A.plan_destroy(p) == MTB_BAD_ARGS, "double destroy");
    }
}
// grouped hop = 1 plans: executes racing mode / segment changes and destroy; the buffers live for the whole
// program (the fake streams may still write them after a destroy returns)
const int kGLens[5] = {512, 1024, 2048, 4096, 512};
const int64_t kGWins[5] = {40, 33, 20, 7, 1};
std::vector<std::vector<double>> g_gin, g_gout[2];
void group_race() {
    CHECK(A.init(0, 16) == MTB_OK, "init group");
    for (int r = 0; r < 30; ++r) {
        const int64_t g = A.group_create(0, 5, kGLens, kGWins, MTB_DETREND_NONE, MTB_WINDOW_HANN, MTB_PREC_F64);
        CHECK(g > 0, "group_create");
        std::atomic<bool> stop{false};
        auto exec = [&](int k) {
            const void *in[5];
            void *out[5];
            for (int m = 0; m < 5; ++m) {
                in[m] = g_gin[m].data();
                out[m] = g_gout[k][m].data();
            }
            while (!stop) {
                const int st = A.group_execute(g, in, out, nullptr);
                if (st == MTB_BAD_ARGS) break;  // destroyed
                CHECK(st == MTB_OK, "group_execute %d", st);
            }
        };
        std::thread e0(exec, 0), e1(exec, 1);
        std::thread tg([&] {
            for (int i = 0; i < 40 && !stop; ++i) {
                A.group_set_mode(g, i % 2);
                A.group_set_segment(g, i % 3 == 0 ? 0 : 7 * i);
            }
        });
        std::this_thread::sleep_for(std::chrono::microseconds(300));
        CHECK(A.group_destroy(g) == MTB_OK, "group destroy");
        stop = true;
        e0.join();
        e1.join();
        tg.join();
        CHECK(A.group_destroy(g) == MTB_BAD_ARGS, "double group destroy");
    }
    A.shutdown();
}

void pinned_feed(int sym) {  // FeedCache rewired to pinned buffers, one chart's view
    CHECK(A.init(0, 16) == MTB_OK, "init pinned %d", sym);
    const int n = 128 << (sym % 3), hop = 1 + sym % 4, len = 64 * hop + n;
    const std::vector<double> s = series_of(40 + sym, len);
    const int nwin = 1 + (len - n) / hop, rec = n / 2;
    std::vector<double> out((size_t)nwin * rec);
    for (int r = 0; r < 20; ++r) {
        CHECK(A.reg(s.data(), len) == MTB_OK, "register series %d", sym);
        CHECK(A.reg(s.data() + 1, 8) == MTB_BAD_ARGS, "overlap refused %d", sym);
        CHECK(A.reg(out.data(), (int64_t)out.size()) == MTB_OK, "register out %d", sym);
        std::fill(out.begin(), out.end(), -1.0);
        int got = 0;
        CHECK(A.batch(s.data(), len, n, hop, MTB_DETREND_NONE, MTB_WINDOW_HANN, 0, MTB_PREC_F64, MTB_OUT_POWER, out.data(),
                      (int)out.size(), &got) == MTB_OK && got == nwin, "pinned batch %d", sym);
        CHECK(check_records(s, out.data(), n, hop, nwin, rec), "pinned records %d round %d", sym, r);
        CHECK(A.unreg(out.data()) == MTB_OK && A.unreg(s.data()) == MTB_OK, "unregister %d", sym);
        CHECK(A.unreg(s.data()) == MTB_BAD_ARGS, "double unregister %d", sym);
    }
    A.shutdown();
}

// registered ranges that do not start or end on a page (round 6: registration only records the range): every
// record must land, no copy may touch the caller's memory directly (the fake runtime counts host sides that are
// not hipHostMalloc'd), and the batch goes through the library's pinned output ring (the sanitizer builds cut
// parts at 64 KiB, WSP_PART_BYTES, so these outputs wrap the 4-slot ring many times)
int64_t (*g_direct_copies)(void) = nullptr;
int64_t (*g_violations)(void) = nullptr;
int64_t (*g_registered)(void) = nullptr;
void pinned_edges(int sym) {
    CHECK(A.init(0, 16) == MTB_OK, "init edges %d", sym);
    const int n = 256, hop = 1 + sym, len = 5000 + 37 * sym;
    std::vector<double> sbuf(len + 1024), obuf;
    const std::vector<double> s0 = series_of(80 + sym, len);
    double *s = sbuf.data() + 3 + 61 * sym;  // not page-aligned, several pages long
    std::copy(s0.begin(), s0.end(), s);
    const int nwin = 1 + (len - n) / hop, rec = n / 2;
    obuf.resize((size_t)nwin * rec + 1024);
    double *out = obuf.data() + 5 + 13 * sym;
    for (int r = 0; r < 10; ++r) {
        const int64_t d0 = g_direct_copies();
        CHECK(A.reg(s, len) == MTB_OK && A.reg(out, (int64_t)nwin * rec) == MTB_OK, "register edges %d", sym);
        std::fill(out, out + (size_t)nwin * rec, -1.0);
        int got = 0;
        CHECK(A.batch(s, len, n, hop, MTB_DETREND_NONE, MTB_WINDOW_HANN, 0, MTB_PREC_F64, MTB_OUT_POWER, out,
                      nwin * rec, &got) == MTB_OK && got == nwin, "edges batch %d", sym);
        CHECK(check_records(s0, out, n, hop, nwin, rec), "edges records %d round %d", sym, r);
        CHECK(g_direct_copies() == d0, "edges: a copy touched caller memory directly %d", sym);
        // a truncated output (out_cap inside a part): exactly the records below the cap, nothing past it
        const int cap_rec = nwin / 3 + 1;
        std::fill(out, out + (size_t)nwin * rec, -7.0);
        CHECK(A.batch(s, len, n, hop, MTB_DETREND_NONE, MTB_WINDOW_HANN, 0, MTB_PREC_F64, MTB_OUT_POWER, out,
                      cap_rec * rec + rec / 2, &got) == MTB_OK && got == cap_rec, "edges truncated batch %d", sym);
        CHECK(check_records(s0, out, n, hop, cap_rec, rec), "edges truncated records %d", sym);
        CHECK(out[(size_t)cap_rec * rec] == -7.0 && out[(size_t)nwin * rec - 1] == -7.0, "edges: past out_cap %d", sym);
        CHECK(A.unreg(out) == MTB_OK && A.unreg(s) == MTB_OK, "unregister edges %d", sym);
    }
    // a buffer with no whole page inside: registered (nothing locked), its batches stage
    std::vector<double> tiny(400);
    const std::vector<double> t0 = series_of(90 + sym, 300);
    std::copy(t0.begin(), t0.end(), tiny.begin() + 1);
    CHECK(A.reg(tiny.data() + 1, 300) == MTB_OK, "register tiny %d", sym);
    std::vector<double> tout(45 * 32);
    int got = 0;
    CHECK(A.batch(tiny.data() + 1, 300, 64, 5, MTB_DETREND_NONE, MTB_WINDOW_HANN, 0, MTB_PREC_F64, MTB_OUT_POWER,
                  tout.data(), (int)tout.size(), &got) == MTB_OK && got == 48 - 3, "tiny batch %d", sym);
    CHECK(check_records(t0, tout.data(), 64, 5, got, 32), "tiny records %d", sym);
    CHECK(A.unreg(tiny.data() + 1) == MTB_OK, "unregister tiny %d", sym);
    A.shutdown();
}

void register_race() {  // two threads register overlapping ranges of one buffer: exactly one wins
    CHECK(A.init(0, 16) == MTB_OK, "init race");
    std::vector<double> buf(1 << 16);
    for (int r = 0; r < 50; ++r) {
        std::atomic<int> ok{0};
        std::thread a([&] { ok += A.reg(buf.data(), 1 << 15) == MTB_OK; });
        std::thread b([&] { ok += A.reg(buf.data() + 1000, 1 << 14) == MTB_OK; });
        a.join();
        b.join();
        CHECK(ok == 1, "overlapping registrations: %d succeeded", ok.load());
        CHECK(A.unreg(buf.data()) == MTB_OK || A.unreg(buf.data() + 1000) == MTB_OK, "unregister the winner");
    }
    A.shutdown();
}
}  // namespace

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        fprintf(stderr, "dlopen: %s\n", dlerror());
        return 3;
    }
    sym(h, A.init, "gpu_init");
    sym(h, A.shutdown, "gpu_shutdown");
    sym(h, A.fft, "gpu_fft_real_forward");
    sym(h, A.submit, "gpu_submit_spectrum_batch");
    sym(h, A.try_get, "gpu_try_get_spectrum_batch");
    sym(h, A.free_job, "gpu_free_job");
    sym(h, A.batch, "gpu_spectrum_batch");
    sym(h, A.plan_create, "wsp_plan_create");
    sym(h, A.plan_execute, "wsp_plan_execute");
    sym(h, A.plan_set_topk, "wsp_plan_set_topk");
    sym(h, A.plan_destroy, "wsp_plan_destroy");
    sym(h, A.reg, "gpu_register_host");
    sym(h, A.unreg, "gpu_unregister_host");
    {  // page-locking caller memory: opt-in in round 5, withdrawn in round 6 (mode 1 refused, 0 the only mode)
        decltype(&gpu_set_host_locking) lock_mode = nullptr;
        sym(h, lock_mode, "gpu_set_host_locking");
        CHECK(lock_mode(1) == MTB_BAD_ARGS && lock_mode(0) == 0 && lock_mode(2) == MTB_BAD_ARGS, "host locking mode");
    }
    sym(h, A.group_create, "wsp_group_create");
    sym(h, A.group_execute, "wsp_group_execute");
    sym(h, A.group_set_mode, "wsp_group_set_mode");
    sym(h, A.group_set_segment, "wsp_group_set_segment");
    sym(h, A.group_destroy, "wsp_group_destroy");
    sym(h, g_direct_copies, "fakehip_direct_copies");
    sym(h, g_violations, "fakehip_violations");
    sym(h, g_registered, "fakehip_registered_ranges");
    for (int m = 0; m < 5; ++m) {
        g_gin.push_back(series_of(60 + m, (int)kGWins[m] + kGLens[m] - 1));
        for (int k = 0; k < 2; ++k) g_gout[k].emplace_back((size_t)kGWins[m] * (kGLens[m] / 2));
    }

    // the session outlives every chart below; a different device is refused while it is open
    CHECK(A.init(0, 8) == MTB_OK, "main init");
    CHECK(A.init(-1, 8) == MTB_BAD_ARGS, "device switch while open");
    std::atomic<int> early_done{0};
    std::vector<std::thread> th;
    for (int c = 0; c < 28; ++c) th.emplace_back(chart, c, c % 2 == 0, std::ref(early_done), 6);
    th.emplace_back(free_race);
    th.emplace_back(plan_race);
    for (int c = 0; c < 4; ++c) th.emplace_back(pinned_feed, c);
    for (int c = 0; c < 3; ++c) th.emplace_back(pinned_edges, c);
    th.emplace_back(register_race);
    th.emplace_back(group_race);
    for (auto &t : th) t.join();
    CHECK(early_done == 14, "early charts %d", early_done.load());
    // main's own reference still holds the session: a sync batch works
    const std::vector<double> s = series_of(5, 1024);
    std::vector<double> out(8 * 64);
    int got = 0;
    CHECK(A.batch(s.data(), 1024, 128, 128, MTB_DETREND_MEAN, MTB_WINDOW_HANN, 0, MTB_PREC_F64, MTB_OUT_POWER, out.data(),
                  (int)out.size(), &got) == MTB_OK && got == 8, "final batch");
    CHECK(check_records(s, out.data(), 128, 128, 8, 64), "final records");
    A.shutdown();
    CHECK(g_registered() == 0, "page-locked ranges left after the last shutdown: %lld", (long long)g_registered());
    CHECK(g_violations() == 0, "fake runtime violations (unaligned / overlapping registrations): %lld",
          (long long)g_violations());
    CHECK(A.init(-1, 4) == MTB_OK, "device switch after the last shutdown");
    A.shutdown();
    printf("hostsan stress: %s (%d failures)\n", g_fail ? "FAIL" : "ok", g_fail.load());
    return g_fail ? 1 : 0;
}
