// wsp_internal.h -- internal interface between the C-ABI layer (mtbridge.cpp)
// and the gfx950 kernels (spectrum_kernels.hip, kalman_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wsp {

// Smallest / largest window the single-workgroup kernel handles.  N = 2M,
// M complex points per window live in one workgroup's registers (16 per
// thread, M/16 threads) and LDS (AoS 16 B per point + pad: 136 KiB at
// N = 16384, within gfx950's 160 KiB per workgroup).
constexpr int kMinLog2N = 5;   // N = 32
constexpr int kMaxLog2N = 14;  // N = 16384
constexpr int kBlock = 128;    // minimum threads per workgroup (2 waves); M/16 when larger

enum Detrend : int { kDetrendNone = 0, kDetrendMean = 1, kDetrendIir = 2, kDetrendKalman = 3 };
enum Output : int { kOutPower = 0, kOutPacked = 1, kOutTopK = 2, kOutPhase = 3, kOutTopKPhase = 4 };

// Everything a spectrum launch needs; pointer types are erased so one
// struct serves the f64 and f32 instantiations.
struct SpectrumLaunch {
    const void *series;   // window w starts at series + w*hop (elements)
    void *out;            // n_windows records of N/2 (power) or N (packed)
    const void *twiddle;  // N/2 complex W_N^k, element type
    int window;           // MTB_WINDOW_* (enum WINDOW_TYPE, L/WaveSpecZZ_1.0.2.mq5:626-632)
    int64_t hop;
    int64_t n_windows;
    int log2n;
    int detrend;          // kDetrendNone/Mean/Iir (Kalman runs as a pre-pass)
    int output;
    bool f32;
    // top-k scan (kOutTopK): k slots, bins [kmin, kmax] (gpuopt-nodetrend.mq5:536-554)
    int topk, kmin, kmax;
    // IIR trend coefficients (L/WaveSpecZZ_1.0.2.mq5:3041-3043), always fp64
    double iir_alpha, iir_c;
    double iir_apow[8];   // alpha^(32 * 2^j), j = 0..7
    int grid;             // 0 = auto
    int nt_mode;          // non-temporal sample loads: 0 = auto (hop >= N), 1 = off, 2 = on
    int vec_mode;         // pair loads: 0 = auto (aligned only), 1 = scalar, 2 = vector even if unaligned
    int variant;          // wsp_plan_set_variant: kOutTopKPhase 1 = the AoS form (ablation)
};

hipError_t launch_spectrum(const SpectrumLaunch &L, hipStream_t stream);
hipError_t launch_spectrum_f32(const SpectrumLaunch &L, hipStream_t stream);
hipError_t launch_spectrum_phase(const SpectrumLaunch &L, hipStream_t stream);  // kOutPhase, kOutTopKPhase (f64)
// the same for log2 N >= 12, compiled in translation units of their own (spectrum_*_hi.hip)
hipError_t launch_spectrum_f64_hi(const SpectrumLaunch &L, hipStream_t stream);
hipError_t launch_spectrum_f32_hi(const SpectrumLaunch &L, hipStream_t stream);
hipError_t launch_spectrum_phase_hi(const SpectrumLaunch &L, hipStream_t stream);

// Inverse real FFT of packed spectra (gpu_fft_real_inverse,
// L/WaveSpecZZ_1.0.4-core.mq5:65,426): n_windows rows of N doubles in the
// gpu_fft_real_forward layout -> n_windows rows of N samples.
struct InverseLaunch {
    const double *in;
    double *out;
    const void *twiddle;  // N complex W_N^k (double)
    int64_t n_windows;
    int log2n;
    int grid;             // 0 = auto
    int variant;          // wsp_plan_set_variant: 1 = the LDS pre-step form, 2 = register pre-step + AoS exchange
};
hipError_t launch_inverse(const InverseLaunch &L, hipStream_t stream);

// Phase / unwrap / group delay of one packed spectrum of n_bins bins
// (gpu_spectral_phase_unwrap, L/WaveSpecZZ_1.0.4-core.mq5:72,416):
// method 0 unwrapped phase, 1 wrapped phase, 2 group delay; out[n_bins].
hipError_t launch_phase_row(const double *spec, int n_bins, int method, double *out, hipStream_t stream);

// Windows of N = 32768 .. 262144 (large_fft.hip): four-step transform over
// a chunk of windows at a time, with the chunk's column results in `y`.
constexpr int kMaxLog2NLarge = 18;
struct LargeLaunch {
    const void *series;   // window w at series + w*hop
    void *out;            // n_windows records of N/2 (power) or N (packed)
    const void *twiddle;  // N complex W_N^k, element type
    void *detrended;      // IIR detrend: n_windows * N elements (else unused)
    double *means;        // mean detrend: n_windows doubles (else unused)
    void *y;              // chunk * N/2 complex elements
    int64_t hop, n_windows, chunk;
    int log2n, window, detrend;
    int packed;           // 0 power, 1 packed (Re, Im)
    bool f32;
    double iir_alpha, iir_c;
    long long *trace;     // diagnostic (wsp_plan_set_trace): fused kernel, workgroup b's first window -> 32 ticks at 32 b
    int64_t trace_cap;
    int variant;          // wsp_plan_set_variant (include/mtbridge.h): 0 = the library's choice (fused non-temporal kernel for
                          // fp64 N = 65536, two passes otherwise), 1 two passes, 2 two passes pipelined over two streams,
                          // 3 fused (512 threads), 4 fused (256 threads, register prefetch), 5 fused with plain stores,
                          // 6 fp64 N = 262144 column pass at 16 columns per workgroup (default 8), 7 row pass in plain
                          // block order (default XCD-aware), 8 two passes with 8-column column workgroups at M2 = 256
};
hipError_t launch_large(const LargeLaunch &L, hipStream_t stream);
// windows per chunk: about 192 MiB of column results (measured best of 16..2048 MiB,
// profiles/r01/large_chunk_sweep.log)
int64_t large_chunk(int log2n, bool f32);

// Per-window Kalman 4D detrend pre-pass: d[w*N + j] = x_j - trend_j
// (one lane per window; trend arithmetic in fp64 like the MQL5 source).
struct KalmanLaunch {
    const void *series;
    void *detrended;      // n_windows * N elements, element type of the plan
    int64_t hop;
    int64_t n_windows;
    int n;
    bool f32;
    double params[16];    // L/WaveSpecZZ_1.0.3-pla-kalman-fast.mq5:886-901 order
    int variant;          // 0 auto, 1 = single-wave workgroups only, 2 = sequential fp32 filter (ablations)
    // fp32 two-segment filter only (kalman_folds_window): the window, as (h_j, h_(j + seg_off)) float pairs for
    // j < L0 (kalman_window_pairs), multiplied into the detrended rows it writes; the spectrum launch then runs
    // with no window.  nullptr = rows leave unwindowed.
    const float *window_pairs;
};

hipError_t launch_kalman_detrend(const KalmanLaunch &L, hipStream_t stream);
// does launch_kalman_detrend multiply the window into the rows of this launch (n <= 4096, the fp32 two-segment
// filter, a window table given)?  Then the spectrum kernel after it must run with no window.
bool kalman_folds_window(const KalmanLaunch &L);
// window pairs of the two-segment filter for window length n: {L0 = (n + WU) / 2, seg_off = L0 - WU}
void kalman_pair_geometry(int n, int *l0, int *seg_off);

// hop = 1 batches by a seeded sliding DFT (sliding_dft.hip): N = 512 .. 8192, detrend none or
// mean, windows none / Hann / Hamming / Blackman (sums of nf = 1, 3, 5 complex exponentials),
// power output.  Arithmetic in fp64 for both element types.
constexpr int kSlideMinLog2N = 9;
constexpr int kSlideMaxLog2N = 13;
struct SlideArgs {
    const void *series;   // window w at series + w (elements)
    void *out;            // n_windows rows of N/2 powers
    const void *twiddle;  // N complex W_N^k (double) -- the seed FFTs
    const void *omega;    // slide table (double complex): [nf][N/2] e^{2 pi j f}, [N/2] H_k, [(nf-1)/2][N] e^{-j m th i}
    int64_t n_windows;
    int64_t seg;          // windows per workgroup; 0 = the launcher's policy
    int log2n, nf, detrend;
    bool f32;
    double s0, s1, s2;    // a0, a1/2, a2/2
    double c1, sn1, c2, sn2;  // cos / sin of th and 2 th, th = 2 pi/(N-1)
    double inv_n;
    // top-k records (launch_slide_topk, fp64): bins [kmin, kmin + span), topk slots, seeds workspace
    int kmin, span, topk;
    void *ws;             // ceil(n_windows / seg) * slide_topk_seed_stride(nf, span) double complex
    int variant;          // top-k scan (wsp_plan_set_variant): 0 = probe threshold (16 windows x 16 candidates, 4 waves
                          // per SIMD), 1 = one wave per window, 2 / 3 = transposed, 16 / 8 windows per batch,
                          // 4 / 5 = probe threshold at 32 windows x 16 / 12 candidates
    unsigned char *flags; // probe-threshold top-k scan: per-window path (wsp_plan_set_scan_flags), nullptr = off
    double share;         // launches running side by side (grouped plan on several streams): the launcher's
                          // segments fill 1/share of the resident workgroup slots; 0 / 1 = all of them
    int seed_chain;       // top-k seeds (N >= 1024): segments per seed workgroup -- one FFT seed, the next ones by
                          // sliding the band's trackers seg windows at a time (<= 1: one FFT seed per segment)
    int store_wt;         // slide_kernel power rows: 1 = written through to memory (sc1 buffer stores), 0 = plain
    long long *trace;     // diagnostic (wsp_plan_set_trace): top-k seed workgroup b writes 6 ticks at 6 b, scan workgroup
    int64_t trace_cap;    // b 2 ticks at trace_cap / 2 + 2 b, while they fit in trace_cap int64 entries; nullptr = off
};
hipError_t launch_slide(const SlideArgs &a, hipStream_t stream);
// Grouped launch: several series of the same window length (the symbols of one length in a
// WaveCyclesBatchFetcher-shaped multi-symbol batch, WaveCyclesBatchFetcher.mq5:112-118) in ONE
// slide_kernel launch.  Member m owns workgroups [blk0[m], blk0[m + 1]); a workgroup's segment is
// windows [(blockIdx - blk0[m]) * seg, ...) of member m.  a.series / a.out / a.n_windows are ignored;
// a.seg = 0 takes the launcher's policy over the members' total window count.
constexpr int kSlideGroupMax = 16;
struct SlideGroup {
    int n = 0;
    const void *series[kSlideGroupMax];
    void *out[kSlideGroupMax];
    int64_t n_windows[kSlideGroupMax];
    int64_t blk0[kSlideGroupMax + 1];  // filled by the launcher
};
hipError_t launch_slide_group(const SlideArgs &a, const SlideGroup &g, hipStream_t stream);
// Mixed-length grouped launch (slide_mixed.hip): the members of a group of window lengths 512 .. 4096 in ONE
// persistent launch.  A 512-thread workgroup takes tasks from a device counter; a task is one segment of a
// 4096-pt member, or 512 / NT(N) segments of a shorter length side by side (one sub-workgroup of NT = N / (2 B)
// threads each).  Tasks run longest windows first, so the four lengths' seed
// phases and drains overlap instead of each launch paying its own (with 4 bins per thread at every length, a task
// is 1 / 2 / 4 / 8 segments at N = 4096 / 2048 / 1024 / 512).  Members are laid out class by class
// (class c = one window length, longest first); series / out are the caller's pointers of this execute.
constexpr int kMixMax = 32;    // members per mixed launch
constexpr int kMixClass = 4;   // window lengths 4096, 2048, 1024, 512
constexpr int kMixNT = 512;    // threads per workgroup
struct SlideMix {
    int nclass, n_tasks;
    int bsmall;                         // bins per thread for N <= 1024: 2 (default) or 4; N >= 2048 always 4
    int seed_lds;                       // 1: the round-4 seed FFTs (staged inputs, radix-4 LDS passes; ablation)
    int wt;                             // 1: output rows written through to memory (sc1 buffer stores; default), 0: plain
    int log2n[kMixClass], seg[kMixClass];
    int task0[kMixClass], nseg[kMixClass], mem0[kMixClass + 1];  // first task / segments / first member of class c
    double c1[kMixClass], sn1[kMixClass], c2[kMixClass], sn2[kMixClass], inv_n[kMixClass];
    double s0, s1, s2;                  // a0, a1/2, a2/2 of the (common) window
    const void *omega[kMixClass];       // slide table of class c (SlideArgs::omega)
    const void *tw4096;                 // W_4096^k, double complex: the quarter table of every length
    int *counter, *done;                // this execute's task counter slot (zero on entry, reset by the last workgroup)
    long long *trace;                   // diagnostic timeline (wsp_group_set_trace), null = off: per task
                                        // [wg | xcc << 32, start, seeds done, end] in wall-clock ticks (100 MHz)
    int64_t sg0[kMixMax];               // member i: its first segment within its class
    int64_t n_windows[kMixMax];
    const void *series[kMixMax];
    void *out[kMixMax];
};
// One launch of `grid` persistent workgroups (grid <= the resident count, slide_mix_resident).
hipError_t launch_slide_mix(const SlideMix &m, int nf, int detrend, bool f32, int grid, hipStream_t stream);
// Resident 512-thread workgroups of the mixed kernel on device `dev` (occupancy x CUs).
int slide_mix_resident(int nf, int detrend, bool f32, int bsmall, int dev);

// hop = 1 top-k records ([bin, power, Re, Im] x topk per window, MTB_OUT_TOPK) by the sliding DFT: the
// band's trackers only (span <= 512), one wave per segment, the FFT kernel's one-wave scan per window.
constexpr int kSlideTopkMaxSpan = 512;
__host__ __device__ inline int64_t slide_topk_seed_stride(int nf, int span) { return (int64_t)nf * span + 1; }
hipError_t launch_slide_topk(const SlideArgs &a, hipStream_t stream);

}  // namespace wsp
