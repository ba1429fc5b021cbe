// oncalculate_harness.cpp -- plays the MT5 terminal: loads libmtbridge.so with
// dlopen (as `#import "mt-bridge.dll"` does, Include/imports.mqh:4) and drives
// it with the reference's own call sequences:
//
//   live   -- the per-bar OnCalculate loop of WaveSpecZZ_1.1.0-gpuopt.mq5:
//             EnsureFeedCache (Include/FeedCache.mqh:36-115) -> per bar
//             FeedBuilder::Build / BuildPlaPriceSeries (1.1.0:760-771) ->
//             EnsureGpu (1.1.0:722-757) -> FftProcessor::Run (1.1.0:518-531:
//             gpu_fft_real_forward + unpack + |X|^2).
//   batch  -- the WaveCyclesBatchFetcher / batch-warmup shape
//             (WaveCyclesBatchFetcher.mq5:91-143, 1.1.0:997-1040): one
//             submit over the whole series, poll with Sleep(5), free.
//
// Usage: oncalculate_harness <libmtbridge.so> <mode live|batch> <feed.bin>
//                            <N> <bars> <out.bin> [detrend window period prec]
// feed.bin is the FeedCache file format (FeedCache.mqh:49-67, 102-111):
// int32 count, then `count` doubles, newest first (series order).
// out.bin receives `bars` spectra of N/2 doubles, oldest window first.
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mtbridge.h"

namespace {

struct Bridge {
    void *h = nullptr;
    decltype(&gpu_init) init;
    decltype(&gpu_shutdown) shutdown;
    decltype(&gpu_fft_real_forward) fft;
    decltype(&gpu_submit_spectrum_batch) submit;
    decltype(&gpu_try_get_spectrum_batch) try_get;
    decltype(&gpu_free_job) free_job;
    decltype(&gpu_get_last_error_w) last_error;

    template <typename F> bool sym(F &f, const char *name) {
        f = reinterpret_cast<F>(dlsym(h, name));
        if (!f) fprintf(stderr, "[harness] missing export %s\n", name);
        return f != nullptr;
    }
    bool load(const char *path) {
        h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            fprintf(stderr, "[harness] dlopen(%s): %s\n", path, dlerror());
            return false;
        }
        return sym(init, "gpu_init") && sym(shutdown, "gpu_shutdown") && sym(fft, "gpu_fft_real_forward") &&
               sym(submit, "gpu_submit_spectrum_batch") && sym(try_get, "gpu_try_get_spectrum_batch") &&
               sym(free_job, "gpu_free_job") && sym(last_error, "gpu_get_last_error_w");
    }
    std::string error() {
        uint16_t w[256];
        const int n = last_error(w, 256);  // count includes the terminator (1.1.0:742-744)
        std::string s;
        for (int i = 0; i + 1 < n; ++i) s.push_back((char)w[i]);
        return n > 0 ? s : "n/a";
    }
};

// struct FeedCache (Include/FeedCache.mqh:20-27); close[] is newest first (:12, :69).
struct FeedCache {
    std::vector<double> close;
    bool loaded = false;
};

bool load_feed_cache(const char *file, FeedCache &c) {  // FeedCache.mqh:49-67
    FILE *f = fopen(file, "rb");
    if (!f) return false;
    int32_t cnt = 0;
    bool ok = fread(&cnt, sizeof(cnt), 1, f) == 1 && cnt > 0;
    if (ok) {
        c.close.resize((size_t)cnt);
        ok = fread(c.close.data(), sizeof(double), (size_t)cnt, f) == (size_t)cnt;
    }
    fclose(f);
    c.loaded = ok;
    return ok;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 7) {
        fprintf(stderr, "usage: %s lib mode(live|batch) feed.bin N bars out.bin [detrend window period prec]\n", argv[0]);
        return 2;
    }
    const char *lib = argv[1];
    const std::string mode = argv[2];
    const int N = atoi(argv[4]);
    const int bars = atoi(argv[5]);
    const int detrend = argc > 7 ? atoi(argv[7]) : MTB_DETREND_NONE;
    const int window = argc > 8 ? atoi(argv[8]) : MTB_WINDOW_NONE;
    const int period = argc > 9 ? atoi(argv[9]) : 0;
    const int prec = argc > 10 ? atoi(argv[10]) : MTB_PREC_F64;

    Bridge br;
    if (!br.load(lib)) return 3;
    FeedCache cache;
    if (!load_feed_cache(argv[3], cache)) {
        fprintf(stderr, "[harness] cannot read feed cache %s\n", argv[3]);
        return 3;
    }
    const int total = (int)cache.close.size();
    if (total < N + bars - 1) {
        fprintf(stderr, "[harness] feed has %d bars, need %d\n", total, N + bars - 1);
        return 3;
    }
    // EnsureGpu: lazy gpu_init(0, clamp(InpGpuStreams,16,512)) (1.1.0:729-735)
    const int streams = 64;
    int st = br.init(0, streams);
    if (st != MTB_OK) {
        fprintf(stderr, "[WaveSpecZZ][ERR] gpu_init failed st=%d reason=%s\n", st, br.error().c_str());
        return 4;
    }
    std::vector<double> spectra((size_t)bars * (N / 2));
    std::vector<double> call_us;  // live mode: wall time of each gpu_fft_real_forward call
    const auto t0 = std::chrono::steady_clock::now();

    if (mode == "live") {
        if (detrend != MTB_DETREND_NONE || window != MTB_WINDOW_NONE) {
            fprintf(stderr, "[harness] live mode follows 1.1.0 (no detrend, no window)\n");
            return 2;
        }
        std::vector<double> feed_data(N), g_fft_interleaved(N), fft_real(N), fft_imag(N);
        // bars processed oldest -> newest; shift_end_feed = bars-1 ... 0
        for (int b = 0; b < bars; ++b) {
            const int shift_end_feed = bars - 1 - b;
            for (int j = 0; j < N; ++j)  // BuildPlaPriceSeries 1.1.0:765-769
                feed_data[j] = cache.close[(size_t)shift_end_feed + (N - 1 - j)];
            // FftProcessor::Run (1.1.0:518-531)
            const auto c0 = std::chrono::steady_clock::now();
            st = br.fft(feed_data.data(), N, g_fft_interleaved.data());
            call_us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c0).count());
            if (st != MTB_OK) {
                fprintf(stderr, "[harness] gpu_fft_real_forward st=%d reason=%s\n", st, br.error().c_str());
                return 5;
            }
            const int bins = N / 2;
            for (int k = 0; k < bins; ++k) {
                const int base = 2 * k;
                fft_real[k] = g_fft_interleaved[base];
                fft_imag[k] = (base + 1 < N) ? g_fft_interleaved[base + 1] : 0.0;
            }
            double *spectrum = &spectra[(size_t)b * bins];
            for (int k = 0; k < bins; ++k) spectrum[k] = fft_real[k] * fft_real[k] + fft_imag[k] * fft_imag[k];
        }
    } else if (mode == "batch") {
        // CopyClose into an as-series array: physical memory is chronological
        const int len = N + bars - 1;
        std::vector<double> prices((size_t)len);
        for (int i = 0; i < len; ++i) prices[i] = cache.close[(size_t)(len - 1 - i)];
        int64_t jid = 0;
        st = br.submit(prices.data(), len, N, 1, detrend, window, period, prec, MTB_OUT_POWER, &jid);
        if (st != MTB_OK || jid == 0) {
            fprintf(stderr, "[harness] submit st=%d reason=%s\n", st, br.error().c_str());
            return 5;
        }
        int ready = 0, out_len = 0;
        const int cap = bars * (N / 2);
        // WaveCyclesBatchFetcher.mq5:126-132, unchanged: 4000 tries, Sleep(5) only on OK with ready == 0,
        // break on any status other than OK / NOT_READY (a NOT_READY re-polls at once)
        for (int tries = 0; tries < 4000 && ready == 0; ++tries) {
            st = br.try_get(jid, spectra.data(), cap, &out_len, &ready);
            if (st == MTB_OK && ready == 0) std::this_thread::sleep_for(std::chrono::milliseconds(5));
            else if (st != MTB_OK && st != MTB_NOT_READY) break;
        }
        br.free_job(jid);
        if (st != MTB_OK || ready != 1 || out_len != bars) {
            fprintf(stderr, "[harness] batch st=%d ready=%d out_len=%d reason=%s\n", st, ready, out_len,
                    br.error().c_str());
            return 5;
        }
    } else {
        fprintf(stderr, "[harness] unknown mode %s\n", mode.c_str());
        return 2;
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    FILE *f = fopen(argv[6], "wb");
    if (!f || fwrite(spectra.data(), sizeof(double), spectra.size(), f) != spectra.size()) {
        fprintf(stderr, "[harness] cannot write %s\n", argv[6]);
        return 6;
    }
    fclose(f);
    br.shutdown();  // OnDeinit 1.1.0:706-716
    printf("[harness] mode=%s N=%d bars=%d seconds=%.6f bars_per_s=%.1f\n", mode.c_str(), N, bars, secs,
           bars / (secs > 0 ? secs : 1e-9));
    if (!call_us.empty()) {  // per-bar latency of the synchronous DLL call (1.1.0:1249 -> :520)
        std::vector<double> v = call_us;
        std::sort(v.begin(), v.end());
        auto pct = [&](double q) { return v[std::min(v.size() - 1, (size_t)(q * (double)(v.size() - 1) + 0.5))]; };
        double sum = 0.0;
        for (double x : v) sum += x;
        printf("[harness] gpu_fft_real_forward N=%d calls=%zu us: first=%.1f p50=%.1f p90=%.1f p99=%.1f max=%.1f "
               "mean=%.1f\n",
               N, v.size(), call_us[0], pct(0.5), pct(0.9), pct(0.99), v.back(), sum / (double)v.size());
    }
    return 0;
}
