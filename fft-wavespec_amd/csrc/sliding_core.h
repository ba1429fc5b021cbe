// sliding_core.h -- device code of the hop = 1 seeded sliding DFT (gfx950), included by
// sliding_dft.hip (power rows, grouped launches) and slide_topk_l*.hip (top-k records, one
// translation unit per window length so that the library builds in parallel).
//
// The same quantity as spectrum_kernel -- per window w: x[w .. w+N) -> [mean detrend] -> cosine
// window (L/WaveSpecZZ_1.0.2.mq5:884-922) -> DFT (FourierTransformManual, :938-974) -> |X_k|^2,
// k < N/2 (1.1.0:529-530) -- for consecutive windows (hop = 1 bar, the batch-warmup and
// fetcher shape: 1.1.0:1014-1020, WaveCyclesBatchFetcher.mq5:106-133), computed by a different
// exact-in-real-arithmetic route that does ~2.5x less fp64 work per window than an FFT.
//
// With the window a0 + a1 cos(th i) + a2 cos(2 th i), th = 2 pi/(N-1), and
// S_w(f) = sum_i x[w+i] e^{-2 pi j f i}:
//     X_w[k] = a0 S_w(k/N) + a1/2 (S_w(k/N + phi) + S_w(k/N - phi)) + a2/2 (S_w(k/N +- 2 phi)),
//     phi = 1/(N-1).
// Each S slides by one sample exactly:
//     S_{w+1}(f) = e^{2 pi j f} (S_w(f) - x[w] + x[w+N] e^{-2 pi j f N}),
// and for f = k/N + m phi the factor e^{-2 pi j f N} = e^{-j m th} is the same for every bin, so
// one step of one tracker T_f = s_f S_f is T <- omega_f (T + u_m) with a per-step uniform u_m:
// 5-6 fp64 operations per tracker, 23 per bin and window for Hann (|X|^2 included) against
// ~57 for the radix-16/8 FFT at N = 2048.  The mean detrend is linear:
// X_w - mean_w * H[k], H = DFT of the window.
//
// Layout: one workgroup per segment of consecutive windows (32..128 windows since round 6: several rounds of
// resident workgroups: launch_t), N/(2B) threads; thread t owns bins k = 2 (t + NT q) + e (q < B/2,
// e < 2), so every store instruction of a wave writes 128 consecutive bins (1 KiB fp64) as one 16-B
// store per lane.  The segment's trackers are SEEDED exactly, not slid from the previous segment:
// Y_m = FFT_N(x[w0 + i] e^{-j m th i}) in LDS (radix-4 Stockham, quarter twiddle table in LDS) gives
// S(k/N + m phi) = Y_m[k] and S(k/N - m phi) = conj(Y_m[N-k]).  The per-step uniforms
// (u_0, u_1, u_2, x[w+N] - x[w]) are staged in LDS a chunk at a time and read by broadcast.
// With the mean detrend the trackers follow the samples minus the segment's first sample.
// Rounding: a tracker's error grows at most linearly with the segment length (<= 256 steps by
// default: ~3e-14 of its own magnitude); the parity bars are BASELINE.md 2's (tests/test_gpu_slide.py,
// tests/test_gpu_fullgrid.py, the CPU model tests/test_slide_model.py).
//
// Top-k records (MTB_OUT_TOPK, fp64) at hop = 1 track only the scan band's bins: slide_seed_kernel writes every
// segment's band trackers to the plan workspace, slide_topk_kernel slides them one wave per segment and runs the FFT
// kernel's one-wave scan (core::topk_wave64) on each window's band, staged in LDS.
#pragma once
#include <atomic>

#include "spectrum_core.h"  // topk_wave64: the one-wave top-k scan of the FFT kernel
#include "wg_fft.h"        // the register-resident workgroup FFT of the top-k seeds
#include "wsp_internal.h"

namespace wsp {
namespace {

typedef double d2 __attribute__((ext_vector_type(2)));

// bins per thread: 4, or 2 for windows up to 1024 (C5's short-window plans: twice the threads per
// workgroup for the same segment)
template <int LOG2N> constexpr int slide_b() { return LOG2N <= 10 ? 2 : 4; }
constexpr int kSlideRMax = 512;  // most steps whose uniforms are staged in LDS at once

template <int NF> struct Rec { static constexpr int n = NF + 1; };  // [u0, (u1r, u1i), (u2r, u2i), d]

__device__ __forceinline__ d2 cmul(d2 a, d2 b) { return d2{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }

// In-place natural-order complex FFT of N points in LDS: Stockham DIT, one radix-2 stage first when
// log2 N is odd, then radix 4; NT threads.  twl[k] = W_N^k for k < N/4 (LDS, or the global table at
// N = 8192 where LDS is full); a radix-4 butterfly loads W^k and forms W^2k, W^3k by products.
// Ends after a barrier.
template <int LOG2N, int NT> __device__ __forceinline__ void fft_lds(d2 *buf, const d2 *twl) {
    constexpr int N = 1 << LOG2N, H = N / 2, N4 = N / 4;
    const int t = threadIdx.x;
    int ns = 1;
    if constexpr (LOG2N & 1) {  // radix 2, Ns = 1: no twiddles
        constexpr int Q = H / NT;
        d2 a[Q], b[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            a[q] = buf[t + NT * q];
            b[q] = buf[t + NT * q + H];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int j = t + NT * q;
            buf[2 * j] = a[q] + b[q];
            buf[2 * j + 1] = a[q] - b[q];
        }
        __syncthreads();
        ns = 2;
    }
    constexpr int Q = N4 / NT;
#pragma unroll 1
    for (; ns < N; ns *= 4) {
        const int tws = N / (4 * ns);  // W_{4 Ns}^k = W_N^{k N/(4 Ns)}
        d2 v[Q][4], w1[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int j = t + NT * q;
            w1[q] = twl[(j & (ns - 1)) * tws];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[q][r] = buf[j + r * N4];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int j = t + NT * q, k = j & (ns - 1);
            const d2 w2 = cmul(w1[q], w1[q]), w3 = cmul(w1[q], w2);
            const d2 x1 = cmul(v[q][1], w1[q]), x2 = cmul(v[q][2], w2), x3 = cmul(v[q][3], w3);
            const d2 t0 = v[q][0] + x2, t1 = v[q][0] - x2, t2 = x1 + x3, d = x1 - x3;
            const d2 t3 = d2{d.y, -d.x};  // -i (x1 - x3)
            const int o = ((j - k) << 2) + k;
            buf[o] = t0 + t2;
            buf[o + ns] = t1 + t3;
            buf[o + 2 * ns] = t0 - t2;
            buf[o + 3 * ns] = t1 - t3;
        }
        __syncthreads();
    }
}

// The same transform with the data in registers between passes (round 5): R = N / NT points per thread (8 at
// N = 4096 / 2048, 4 at 1024 / 512 with two bins per thread), Stockham passes of radix R (the last one of the
// remaining factor), the thread's pass-0 inputs x[t + NT r] straight from the caller's registers (no input
// staging round trip), LDS only to exchange between passes.  N = 4096: 4 passes and 7 barriers instead of 6
// radix-4 LDS passes, 12 barriers and the input staging -- the seeds were 14 % of every C5 task (33 of 242 us,
// the r05c timeline) and all of the first round's latency.  Twiddles W_{Ns R}^k from the W_4096 quarter table
// (k N / (Ns R) < N / 4 for R = 4 / 8; a final radix-2 pass folds its upper quarter by W^(N/4) = -i), their powers
// by products (<= 7 steps).  TS: the quarter table's stride for W_N (4096 / N for the mixed launch's W_4096 table,
// 1 for slide_kernel's own W_N table, round 6).
template <int LOG2N, int NT, int RP, int NS, int TS>
__device__ __forceinline__ void reg_pass_write(d2 (&v)[(1 << LOG2N) / NT], d2 *buf, const d2 *twq, int t) {
    constexpr int N = 1 << LOG2N, R = N / NT, Q = R / RP;
    static_assert(Q * RP == R && RP >= 2, "pass geometry");
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int j = t + NT * q, k = j & (NS - 1);
        d2 *a = v + q * RP;
        if constexpr (NS > 1) {
            // W_N^m, m = k N / (Ns R): below N/4 (the quarter table) for R = 4 / 8; a last radix-2 pass reaches
            // m < N/2, whose upper quarter is W_N^(m - N/4) (-i)
            const int m = k * (N / (NS * RP));
            d2 w;
            if constexpr (RP == 2) {
                const d2 q = twq[(m & (N / 4 - 1)) * TS];
                w = m < N / 4 ? q : d2{q.y, -q.x};
            } else {
                w = twq[m * TS];
            }
            d2 wr = w;
#pragma unroll
            for (int r = 1; r < RP; ++r) {
                a[r] = cmul(a[r], wr);
                if (r + 1 < RP) wr = cmul(wr, w);
            }
        }
        core::cpx<double> c[RP];  // by value: a d2 / cpx type pun through pointers breaks type-based alias analysis
#pragma unroll
        for (int r = 0; r < RP; ++r) c[r] = {a[r].x, a[r].y};
        core::dft<double, RP>(c);
#pragma unroll
        for (int r = 0; r < RP; ++r) a[r] = d2{c[r].re, c[r].im};
        const int o = (j - k) * RP + k;
#pragma unroll
        for (int r = 0; r < RP; ++r) buf[o + NS * r] = a[r];
    }
}
template <int LOG2N, int NT, int NS, int TS>
__device__ __forceinline__ void reg_passes(d2 *buf, const d2 *twq, int t) {
    constexpr int N = 1 << LOG2N, R = N / NT;
    if constexpr (NS < N) {
        constexpr int RP = N / NS >= R ? R : N / NS;
        d2 v[R];
#pragma unroll
        for (int q = 0; q < R / RP; ++q)
#pragma unroll
            for (int r = 0; r < RP; ++r) v[q * RP + r] = buf[t + NT * q + (N / RP) * r];
        __syncthreads();
        reg_pass_write<LOG2N, NT, RP, NS, TS>(v, buf, twq, t);
        __syncthreads();
        reg_passes<LOG2N, NT, NS * RP, TS>(buf, twq, t);
    }
}
// a[r] = this thread's input x[t + NT r]; buf must be free (no reads pending).  Natural order in buf, ends after a
// barrier.
template <int LOG2N, int NT, int TS>
__device__ __forceinline__ void fft_reg_sub(d2 (&a)[(1 << LOG2N) / NT], d2 *buf, const d2 *twq, int t) {
    constexpr int N = 1 << LOG2N, R = N / NT;
    static_assert(R == 4 || R == 8, "4 or 8 points per thread");
    reg_pass_write<LOG2N, NT, R, 1, TS>(a, buf, twq, t);
    __syncthreads();
    reg_passes<LOG2N, NT, R, TS>(buf, twq, t);
}

// Bin b of thread t: pairs of adjacent bins, 2 (t + NT (b / 2)) + b % 2, so that a wave's store of a pair
// of powers is one 16-B access per lane (1 KiB contiguous per wave instruction).
template <int NT> __device__ __forceinline__ int kbin_of(int t, int b) { return 2 * (t + NT * (b >> 1)) + (b & 1); }

// The segment's seeds: Y_m = FFT_N((x[w0 + i] - L) e^{-j m th i}), m = 0 .. (NF-1)/2, in LDS; pick(m, s_m, Y)
// takes what it needs from each transform (every thread calls it between the transform's barriers).
template <typename T, int LOG2N, int NF, int DETREND, int NT, typename PICK>
__device__ __forceinline__ void seed_ffts(const SlideArgs &a, const T *__restrict__ x, double lvl, d2 *lds, d2 *twq,
                                          PICK pick) {
    constexpr int N = 1 << LOG2N, M = N / 2, NM = (NF - 1) / 2;
    constexpr bool TWL = N <= 4096;  // the quarter twiddle table fits LDS beside the FFT buffer
    const int t = threadIdx.x;
    const d2 *__restrict__ tw = static_cast<const d2 *>(a.twiddle);
    const d2 *__restrict__ mod = static_cast<const d2 *>(a.omega) + (NF + 1) * M;  // [NM][N]
    const d2 *twl = tw;
    if constexpr (TWL) {
        for (int i = t; i < N / 4; i += NT) twq[i] = tw[i];
        twl = twq;
    }
    // round 6: with the quarter table in LDS (N <= 4096) the transforms run as register passes (fft_reg_sub, the
    // mixed launch's seeds since round 5: N = 2048 in 4 passes and 7 barriers instead of a radix-2 stage, 5 radix-4
    // LDS passes, 12 barriers and the input staging round trip), inputs straight from global memory into registers
    // (twq is complete at the first pass's barrier: pass 0 uses no twiddles)
#pragma unroll
    for (int m = 0; m <= NM; ++m) {
        if constexpr (TWL && (N / NT == 4 || N / NT == 8)) {
            d2 v[N / NT];
#pragma unroll
            for (int r = 0; r < N / NT; ++r) {
                const int i = t + NT * r;
                const double xi = (double)x[i] - lvl;
                v[r] = m == 0 ? d2{xi, 0.0} : xi * mod[(m - 1) * N + i];
            }
            fft_reg_sub<LOG2N, NT, 1>(v, lds, twl, t);
        } else {
            for (int i = t; i < N; i += NT) {
                const double xi = (double)x[i] - lvl;
                lds[i] = m == 0 ? d2{xi, 0.0} : xi * mod[(m - 1) * N + i];
            }
            __syncthreads();
            fft_lds<LOG2N, NT>(lds, twl);
        }
        pick(m, m == 0 ? a.s0 : (m == 1 ? a.s1 : a.s2), lds);
        __syncthreads();
    }
}

// Per-step uniforms of steps c0 .. c0 + clen - 1 into u[st * REC]: u_m = s_m (x[w+N] e^{-j m th} - x[w]),
// d = x[w+N] - x[w] (samples minus the segment's level L); no step after the segment's last window.
template <typename T, int NF, int N>
__device__ __forceinline__ void stage_uniforms(const SlideArgs &a, const T *__restrict__ x, double lvl, int c0,
                                               int clen, int len, double *u, int t, int nt) {
    constexpr int REC = Rec<NF>::n;
    for (int st = t; st < clen; st += nt) {
        if (c0 + st + 1 >= len) break;
        const double xw = (double)x[c0 + st] - lvl, xn = (double)x[c0 + st + N] - lvl;
        double *r = u + st * REC;
        r[0] = a.s0 * (xn - xw);
        if constexpr (NF >= 3) {
            r[1] = a.s1 * (xn * a.c1 - xw);
            r[2] = -(a.s1 * (xn * a.sn1));
        }
        if constexpr (NF >= 5) {
            r[3] = a.s2 * (xn * a.c2 - xw);
            r[4] = -(a.s2 * (xn * a.sn2));
        }
        r[REC - 1] = xn - xw;
    }
}

// One slide of B bins' trackers: T_f <- omega_f (T_f + u_m); the mean path's running sum of x - L.
template <int B, int NF, int DETREND>
__device__ __forceinline__ void slide_step(d2 (&tr)[B][NF], const d2 (&om)[B][NF], const double *r, double &sum) {
    const double u0 = r[0];
#pragma unroll
    for (int b = 0; b < B; ++b) tr[b][0] = cmul(om[b][0], d2{tr[b][0].x + u0, tr[b][0].y});
    if constexpr (NF >= 3) {
        const double u1r = r[1], u1i = r[2];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            tr[b][1] = cmul(om[b][1], tr[b][1] + d2{u1r, u1i});
            tr[b][2] = cmul(om[b][2], tr[b][2] + d2{u1r, -u1i});
        }
    }
    if constexpr (NF >= 5) {
        const double u2r = r[3], u2i = r[4];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            tr[b][3] = cmul(om[b][3], tr[b][3] + d2{u2r, u2i});
            tr[b][4] = cmul(om[b][4], tr[b][4] + d2{u2r, -u2i});
        }
    }
    if constexpr (DETREND == kDetrendMean) sum += r[Rec<NF>::n - 1];
}

// Workgroup -> (member, segment) of a grouped launch (SlideGroup): members own contiguous runs of
// workgroups.  Unrolled selects over the kernel-argument table (uniform scalar loads, no dynamic
// indexing of the argument struct).
struct SlideSeg {
    const void *series;
    void *out;
    int64_t w0, n_windows;
};
__device__ __forceinline__ SlideSeg slide_seg_of(const SlideGroup &g, int64_t seg) {
    const int64_t b = blockIdx.x;
    SlideSeg r{g.series[0], g.out[0], b * seg, g.n_windows[0]};
#pragma unroll
    for (int i = 1; i < kSlideGroupMax; ++i)
        if (i < g.n && b >= g.blk0[i]) r = SlideSeg{g.series[i], g.out[i], (b - g.blk0[i]) * seg, g.n_windows[i]};
    return r;
}

template <typename T, int LOG2N, int NF, int DETREND>
__global__ __launch_bounds__((1 << LOG2N) / (2 * slide_b<LOG2N>()),
                             slide_b<LOG2N>() == 2 ? 4 : (NF >= 5 ? 2 : (NF >= 3 ? (LOG2N == 12 && DETREND == kDetrendNone ? 4 : 3) : 4))) void slide_kernel(SlideArgs a,
                                                                                                              SlideGroup g) {
    constexpr int N = 1 << LOG2N, M = N / 2, B = slide_b<LOG2N>(), NT = M / B;
    constexpr int REC = Rec<NF>::n;
    const SlideSeg sg = slide_seg_of(g, a.seg);  // this workgroup's member (a single plan is a group of one)
    if (sg.w0 >= sg.n_windows) return;
    // per-step uniforms staged CH steps at a time: N/4 clamped to [128, 512], so that small windows keep
    // 4 single-/two-wave workgroups per SIMD (LDS: FFT buffer + quarter twiddles + uniforms)
    constexpr int CH = N / 4 < 128 ? 128 : (N / 4 > kSlideRMax ? kSlideRMax : N / 4);
    constexpr int LDS2 = (N > CH * REC / 2) ? N : CH * REC / 2;
    constexpr bool TWL = N <= 4096;  // the quarter twiddle table fits LDS beside the FFT buffer
    __shared__ d2 lds[LDS2];
    __shared__ d2 twq[TWL ? N / 4 : 1];

    const int t = threadIdx.x;
    auto kbin = [](int tt, int b) { return kbin_of<NT>(tt, b); };
    const int len = (int)((sg.n_windows - sg.w0) < a.seg ? (sg.n_windows - sg.w0) : a.seg);
    const T *__restrict__ x = static_cast<const T *>(sg.series) + sg.w0;  // the segment's first window
    const d2 *__restrict__ omega = static_cast<const d2 *>(a.omega);  // [NF][M]
    const d2 *__restrict__ hwin = omega + NF * M;                      // [M]
    // diagnostic timeline (wsp_plan_set_trace, scripts/slide_timeline.py): workgroup b writes {block | XCC << 32,
    // start, seeds done, end} at trace[4 b] while 4 b + 4 <= trace_cap; off (nullptr) by default
    long long *trc = (a.trace && 4 * (int64_t)blockIdx.x + 4 <= a.trace_cap && threadIdx.x == 0)
                         ? a.trace + 4 * (int64_t)blockIdx.x : nullptr;
    if (trc) {
        unsigned xcc = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        trc[0] = (long long)blockIdx.x | ((long long)(xcc & 15) << 32);
        trc[1] = wall_clock64();
    }

    d2 om[B][NF], tr[B][NF];
    // mean detrend: the trackers follow x - L, L = the segment's first sample, and the output subtracts
    // (mean - L) H_k: X_w - mean_w H = X(x - L) - (mean_w - L) H.  Centring keeps the ~N x price level
    // out of the trackers near DC (20x smaller rounding at bins 0-2, tests/test_slide_model.py).
    const double lvl = DETREND == kDetrendMean ? (double)x[0] : 0.0;

    double sum0 = 0.0;
    seed_ffts<T, LOG2N, NF, DETREND, NT>(a, x, lvl, lds, twq, [&](int m, double s, const d2 *y) {
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int k = kbin(t, b);
            if (m == 0) {
                tr[b][0] = s * y[k];
            } else {
                const d2 yp = y[k], ym = y[(N - k) & (N - 1)];
                tr[b][2 * m - 1] = s * yp;
                tr[b][2 * m] = s * d2{ym.x, -ym.y};
            }
        }
        if (DETREND == kDetrendMean && m == 0) sum0 = y[0].x;  // broadcast read: sum of x - L
    });

    if (trc) trc[2] = wall_clock64();
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
        for (int f = 0; f < NF; ++f) om[b][f] = omega[f * M + kbin(t, b)];
    d2 hk[B];
    double sum = 0.0;
    if constexpr (DETREND == kDetrendMean) {
#pragma unroll
        for (int b = 0; b < B; ++b) hk[b] = hwin[kbin(t, b)];
        sum = sum0;
    }

    T *__restrict__ out = static_cast<T *>(sg.out) + sg.w0 * M + 2 * t;
    // a.store_wt: sc1 buffer stores (written through to memory: no dirty rows left in the XCDs' L2s for the writeback
    // at the kernel's end), the descriptor at the segment's first row, offsets within the segment
    const bool wt = a.store_wt != 0;
    const __amdgpu_buffer_rsrc_t orc =
        __builtin_amdgcn_make_buffer_rsrc(static_cast<T *>(sg.out) + sg.w0 * M, (short)0, 0x7fffffff, 0x00020000);
    uint32_t ob = (uint32_t)(2 * t * (int)sizeof(T));
    double *u = reinterpret_cast<double *>(lds);
    for (int c0 = 0; c0 < len; c0 += CH) {
        const int clen = len - c0 < CH ? len - c0 : CH;
        if (c0) __syncthreads();  // the previous chunk's reads are done
        stage_uniforms<T, NF, N>(a, x, lvl, c0, clen, len, u, t, NT);
        __syncthreads();

        // ---- slide
#pragma unroll 1
        for (int st = 0; st < clen; ++st) {
            double mw = 0.0;
            if constexpr (DETREND == kDetrendMean) mw = sum * a.inv_n;
            double p[B];
#pragma unroll
            for (int b = 0; b < B; ++b) {
                d2 X = tr[b][0];
#pragma unroll
                for (int f = 1; f < NF; ++f) X += tr[b][f];
                if constexpr (DETREND == kDetrendMean) X -= mw * hk[b];
                p[b] = X.x * X.x + X.y * X.y;
            }
            // bins 2(t + NT q) and 2(t + NT q) + 1: one 16-B (fp64) / 8-B (fp32) store per pair; plain
            // stores: a pure write stream runs at 5.75 TB/s plain vs 5.5 non-temporal
            // (tools/write_probe.hip, profiles/r02/slide/write_probe.log)
#pragma unroll
            for (int q = 0; q < B / 2; ++q) {
                typedef T v2t __attribute__((ext_vector_type(2)));
                const v2t pv = v2t{(T)p[2 * q], (T)p[2 * q + 1]};
                if (wt) {
                    const int qo = (int)(ob + 2 * NT * q * sizeof(T));
                    if constexpr (sizeof(T) == 8) {
                        typedef unsigned u4 __attribute__((ext_vector_type(4)));
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, pv), orc, qo, 0, 16);
                    } else {
                        typedef unsigned u2 __attribute__((ext_vector_type(2)));
                        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, pv), orc, qo, 0, 16);
                    }
                } else {
                    *reinterpret_cast<v2t *>(out + 2 * NT * q) = pv;
                }
            }
            out += M;
            ob += M * sizeof(T);
            if (c0 + st + 1 < len) slide_step<B, NF, DETREND>(tr, om, u + st * REC, sum);
        }
    }
    if (trc) trc[3] = wall_clock64();
}

// Workgroups: each slides a segment of consecutive windows (seeded once, per-step uniforms staged CH
// steps at a time); segment length from the residency (occupancy API, once per instantiation).
// ---- hop = 1 top-k records (MTB_OUT_TOPK): only the band's bins are tracked.
// Seeds of every segment into the workspace: [NF][span] trackers of bins kmin .. kmin + span - 1, then
// {sum of x - L (mean path), L}; one workgroup per segment, the same in-LDS FFTs as slide_kernel.
// threads of the seed pass: N/4 (one radix-4 butterfly per thread and stage), at most 1024
template <int LOG2N> constexpr int seed_nt() { return (1 << LOG2N) / 4 < 1024 ? (1 << LOG2N) / 4 : 1024; }

template <typename T, int LOG2N, int NF, int DETREND>
__global__ __launch_bounds__(seed_nt<LOG2N>()) void slide_seed_kernel(SlideArgs a) {
    constexpr int N = 1 << LOG2N, NT = seed_nt<LOG2N>();
    constexpr bool TWL = N <= 4096;
    __shared__ d2 lds[N];
    __shared__ d2 twq[TWL ? N / 4 : 1];
    const int t = threadIdx.x;
    const int64_t w0 = (int64_t)blockIdx.x * a.seg;
    if (w0 >= a.n_windows) return;
    const T *__restrict__ x = static_cast<const T *>(a.series) + w0;
    const double lvl = DETREND == kDetrendMean ? (double)x[0] : 0.0;
    d2 *__restrict__ ws = static_cast<d2 *>(a.ws) + blockIdx.x * slide_topk_seed_stride(NF, a.span);
    const int span = a.span, kmin = a.kmin;
    seed_ffts<T, LOG2N, NF, DETREND, NT>(a, x, lvl, lds, twq, [&](int m, double s, const d2 *y) {
        for (int j = t; j < span; j += NT) {
            const int k = kmin + j;
            if (m == 0) {
                ws[j] = s * y[k];
            } else {
                const d2 ym = y[(N - k) & (N - 1)];
                ws[(2 * m - 1) * span + j] = s * y[k];
                ws[(2 * m) * span + j] = s * d2{ym.x, -ym.y};
            }
        }
        if (m == 0 && t == 0) ws[NF * span] = d2{y[0].x, lvl};
    });
}

// The same seeds by the register-resident workgroup FFT (wg::wg_fft: N/16 threads, 16 points each, radix-16
// Stockham passes with LDS only between passes -- 2 exchanges at N = 2048 / 4096 against 6 / 7 LDS round trips
// of fft_lds at N/4 threads), one transform m at a time, every output in natural order to LDS and the band read
// back: Y_m = FFT_N((x[w0 + i] - L) e^{-j m th i}) as slide_seed_kernel (N >= 1024).
//
// Seed chains (round 5, wsp_plan_set_variant 6 -- an ablation, slower than the default one FFT seed per segment:
// the chain's slide steps are serial, r05g): a workgroup seeds G = a.seed_chain consecutive segments -- the first by the FFTs, each next one
// by sliding the band's trackers a.seg windows on from the previous (slide_step, the uniforms of stage_uniforms: the
// same operations the scan kernel applies, so a chained seed is exactly what the scan wave of the previous segment
// holds after sliding across the seam, as if the segments were one).  The segment count of the scan (one wave per
// segment, a full round of resident waves) no longer sets the number of FFT seeds: a one-eighth C4 shard has 2048
// segments of 64 windows and seeded every one by two 2048-point FFTs, a fixed ~44 us beside a ~45 us scan
// (profiles/r04/shards.json: C4 top-8 3.7x at 8 ranks).  Chains are at most 256 windows long (as the rounding of a
// 256-window segment); the workgroup's threads keep their bins' trackers (j = t + TP i < span) in registers.
template <int LOG2N, int NF, int DETREND, int JB>
__global__ __launch_bounds__((1 << LOG2N) / 16) void slide_seed_r_kernel(SlideArgs a) {
    using G = wg::LGeo<LOG2N>;
    constexpr int N = 1 << LOG2N, M = N / 2, TP = G::TP, NM = (NF - 1) / 2, R = wg::last_radix<LOG2N>();
    constexpr int REC = Rec<NF>::n;  // JB: band bins per thread, span <= JB TP (launch_topk_t)
    __shared__ core::cpx<double> lds[G::SLOT];
    const int t = threadIdx.x;
    const int chain = a.seed_chain > 1 ? a.seed_chain : 1;
    const int64_t sg0 = (int64_t)blockIdx.x * chain;  // this workgroup's first segment
    const int64_t w0 = sg0 * a.seg;
    if (w0 >= a.n_windows) return;
    // diagnostic timeline (wsp_plan_set_trace): [workgroup | XCC << 32, start, FFT 0 done, seeds done, chain done, end]
    long long *trc = a.trace && 6 * ((int64_t)blockIdx.x + 1) <= a.trace_cap / 2 && t == 0 ? a.trace + 6 * (int64_t)blockIdx.x : nullptr;
    if (trc) {
        unsigned xcc = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        trc[0] = (long long)blockIdx.x | ((long long)(xcc & 15) << 32);
        trc[1] = wall_clock64();
    }
    const double *__restrict__ x = static_cast<const double *>(a.series) + w0;
    const core::cpx<double> *__restrict__ tw = static_cast<const core::cpx<double> *>(a.twiddle);
    const d2 *__restrict__ mod = static_cast<const d2 *>(a.omega) + (NF + 1) * M;  // [NM][N] e^{-j m th i}
    const double lvl = DETREND == kDetrendMean ? x[0] : 0.0;
    const int64_t stride = slide_topk_seed_stride(NF, a.span);
    d2 *__restrict__ ws = static_cast<d2 *>(a.ws) + sg0 * stride;
    const int span = a.span, kmin = a.kmin;
    // seed records: agent-scope (write-through, sc1) stores -- every workgroup of a chain writes its later segments'
    // records at its end, and the dirty lines plain or non-temporal stores leave in the XCDs' L2s are written back at
    // the kernel boundary before the scan can start: 1/8 C4 top-8 0.0781 / 0.0784 ms (non-temporal), 0.0774 / 0.0785
    // (plain, variant 7), 0.0732 / 0.0733 (write-through), first scan workgroup 31.0 / 30.3 / 25.1 us after the first
    // seed workgroup's start (r05r, profiles/r05/timeline); the whole batch unchanged.  Variant 8 = non-temporal.
    const bool nts = a.variant == 8, wt = a.variant != 7 && a.variant != 8;
    auto wst = [&](d2 *p, d2 v) {
        typedef double v2d __attribute__((ext_vector_type(2)));
        if (wt) {
            double *q = reinterpret_cast<double *>(p);
            __hip_atomic_store(q, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(q + 1, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (nts) {
            __builtin_nontemporal_store(v2d{v.x, v.y}, reinterpret_cast<v2d *>(p));
        } else {
            *p = v;
        }
    };
    d2 trk[JB][NF];  // the chain's trackers of bins kmin + t + TP i
    double sum = 0.0;
    double xs[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) xs[r] = x[t + TP * r] - lvl;
#pragma unroll
    for (int m = 0; m <= NM; ++m) {
        core::cpx<double> v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (m == 0) {
                v[r] = core::cpx<double>{xs[r], 0.0};
            } else {
                const d2 e = mod[(m - 1) * N + t + TP * r];
                v[r] = core::cpx<double>{xs[r] * e.x, xs[r] * e.y};
            }
        }
        wg::wg_fft<double, LOG2N>(v, lds, t, tw, LOG2N);  // ends after a barrier: lds is free
        // v[q R + r] = Y[b + (N/R) r], b = t + TP q: natural order into lds
#pragma unroll
        for (int q = 0; q < 16 / R; ++q)
#pragma unroll
            for (int r = 0; r < R; ++r) lds[core::pad16(t + TP * q + (N / R) * r)] = v[q * R + r];
        __syncthreads();
        const double s = m == 0 ? a.s0 : (m == 1 ? a.s1 : a.s2);
#pragma unroll
        for (int i = 0; i < JB; ++i) {
            const int j = t + TP * i;
            if (j >= span) continue;
            const int k = kmin + j;
            const core::cpx<double> yp = lds[core::pad16(k)];
            if (m == 0) {
                trk[i][0] = s * d2{yp.re, yp.im};
                wst(ws + j, trk[i][0]);
            } else {
                const core::cpx<double> ym = lds[core::pad16((N - k) & (N - 1))];
                trk[i][2 * m - 1] = s * d2{yp.re, yp.im};
                trk[i][2 * m] = s * d2{ym.re, -ym.im};
                wst(ws + (2 * m - 1) * span + j, trk[i][2 * m - 1]);
                wst(ws + (2 * m) * span + j, trk[i][2 * m]);
            }
        }
        if (m == 0) {
            sum = lds[0].re;  // sum of x - L (mean path)
            if (t == 0) wst(ws + NF * span, d2{sum, lvl});  // and L
        }
        __syncthreads();  // the band reads before the next transform's exchanges
        if (trc) trc[2 + (m > 0)] = wall_clock64();
    }
    if (chain == 1) {
        if (trc) trc[4] = trc[5] = wall_clock64();
        return;
    }
    d2 om[JB][NF];
    const d2 *__restrict__ omega = static_cast<const d2 *>(a.omega);
#pragma unroll
    for (int i = 0; i < JB; ++i) {
        const int j = t + TP * i;
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            om[i][f] = j < span ? omega[f * M + kmin + j] : d2{1.0, 0.0};
            if (j >= span) trk[i][f] = d2{0.0, 0.0};
        }
    }
    // the chain's per-step uniforms, all at once into LDS (stage_uniforms: every thread a share of the steps), then
    // the sequential slide reads them by broadcast -- loading x[w], x[w + N] inside the dependent loop put a global
    // load latency on every step (C4 top-8 0.355 -> 0.440 ms in the first version, r05f)
    const int64_t seg = a.seg;
    const int64_t last = a.n_windows - 1 - w0;  // no step past the batch's last window
    const int nsteps = (int)((chain - 1) * seg < last ? (chain - 1) * seg : last);
    double *u = reinterpret_cast<double *>(lds);
    static_assert(256 * REC <= G::SLOT * 2, "a chain's uniforms fit the FFT's LDS");
    stage_uniforms<double, NF, N>(a, x, lvl, 0, nsteps, nsteps + 1, u, t, TP);
    __syncthreads();
    auto put = [&](int g) {
        d2 *__restrict__ wsg = ws + g * stride;
#pragma unroll
        for (int i = 0; i < JB; ++i) {
            const int j = t + TP * i;
            if (j >= span) continue;
#pragma unroll
            for (int f = 0; f < NF; ++f) wst(wsg + f * span + j, trk[i][f]);
        }
        if (t == 0) wst(wsg + NF * span, d2{sum, lvl});  // the chain's level L (the scan's uniforms follow x - L)
    };
    for (int g = 1; g < chain; ++g) {
        const int64_t wsg0 = g * seg;  // this segment's first window, relative to w0
        if (wsg0 > nsteps) break;
        // unrolled: the LDS reads of 8 steps' uniforms issue together, ahead of the dependent tracker updates
        // (one read + wait per step put the LDS latency on every step of the serial chain)
        const int st1 = (int)wsg0;
#pragma unroll 8
        for (int st = st1 - (int)seg; st < st1; ++st) slide_step<JB, NF, DETREND>(trk, om, u + st * REC, sum);
        put(g);
    }
    if (trc) trc[4] = trc[5] = wall_clock64();
}

// One wave per segment: lane l tracks bins kmin + l + 64 b (b < NB), stages each window's band X in LDS
// and runs the FFT kernel's one-wave scan (core::topk_wave64: power desc, bin asc, as the reference's
// strict-'>' insertion, L/WaveSpecZZ_1.0.3-pla-kalman-fast-gpuopt-nodetrend.mq5:536-554), which writes the
// window's record row.
template <int LOG2N, int NF, int DETREND, int NB>
__global__ __launch_bounds__(64) void slide_topk_kernel(SlideArgs a) {
    constexpr int N = 1 << LOG2N, M = N / 2, REC = Rec<NF>::n, CHT = 128;
    __shared__ double u[CHT * REC];
    __shared__ core::cpx<double> xb[64 * NB];
    const int l = threadIdx.x;
    const int64_t w0 = (int64_t)blockIdx.x * a.seg;
    if (w0 >= a.n_windows) return;
    const int len = (int)((a.n_windows - w0) < a.seg ? (a.n_windows - w0) : a.seg);
    const double *__restrict__ x = static_cast<const double *>(a.series) + w0;
    const d2 *__restrict__ omega = static_cast<const d2 *>(a.omega);
    const d2 *__restrict__ hwin = omega + NF * M;
    const d2 *__restrict__ ws = static_cast<const d2 *>(a.ws) + blockIdx.x * slide_topk_seed_stride(NF, a.span);
    const int span = a.span, kmin = a.kmin;
    d2 tr[NB][NF], om[NB][NF], hk[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int j = l + 64 * b;
        const bool ok = j < span;
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            tr[b][f] = ok ? ws[f * span + j] : d2{0.0, 0.0};
            om[b][f] = ok ? omega[f * M + kmin + j] : d2{1.0, 0.0};
        }
        hk[b] = (DETREND == kDetrendMean && ok) ? hwin[kmin + j] : d2{0.0, 0.0};
    }
    const d2 sl = ws[NF * span];
    double sum = sl.x;
    const double lvl = sl.y;
    double *__restrict__ rec = static_cast<double *>(a.out) + w0 * (int64_t)(4 * a.topk);
    for (int c0 = 0; c0 < len; c0 += CHT) {
        const int clen = len - c0 < CHT ? len - c0 : CHT;
        if (c0) __syncthreads();
        stage_uniforms<double, NF, N>(a, x, lvl, c0, clen, len, u, l, 64);
        __syncthreads();
#pragma unroll 1
        for (int st = 0; st < clen; ++st) {
            const double mw = DETREND == kDetrendMean ? sum * a.inv_n : 0.0;
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                d2 X = tr[b][0];
#pragma unroll
                for (int f = 1; f < NF; ++f) X += tr[b][f];
                if constexpr (DETREND == kDetrendMean) X -= mw * hk[b];
                xb[l + 64 * b] = core::cpx<double>{X.x, X.y};
            }
            __syncthreads();  // one wave: orders the band's LDS writes before the scan's reads
            core::topk_wave64<NB, double>(xb, kmin, span, a.topk, l, rec, true);
            __syncthreads();  // the scan's reads before the next window's writes
            rec += 4 * a.topk;
            if (c0 + st + 1 < len) slide_step<NB, NF, DETREND>(tr, om, u + st * REC, sum);
        }
    }
}

// ---- the same records by a transposed scan (k <= 8): lane per window instead of a wave per window.
// The wave slides its band's trackers as slide_topk_kernel does (lane l: bins kmin + l + 64 b) and
// stages WB consecutive windows' band X in LDS ([window][bin], odd row stride: the scan's 16-byte
// reads of 16 rows are conflict-free).  Then the lanes turn to the windows: lane l scans window
// l % WB over the quarter (LPW = 64 / WB parts) l / WB of the band with the reference's 8-slot
// insertion in registers (strict '>' against slots sorted by power: an equal power goes after the
// earlier, lower bin -- L/WaveSpecZZ_1.0.3-pla-kalman-fast-gpuopt-nodetrend.mq5:536-554), and the
// LPW partial lists of a window are merged across lanes (log2 LPW rounds: exchange with the partner
// lane, keep the best 8 of the two by a bitonic merge under the key (power desc, bin asc)).  Every
// lane of a window then holds its top 8; lane part q writes slots 2q, 2q + 1 (Re / Im from LDS).
// Against one wave-wide max + ballot per slot and window (topk_wave64: 8 dependent reduction rounds
// per window), the scan is ~90 independent VALU operations per window and lane group.
constexpr int kTopkT = 8;  // slots of the transposed scan (the reference's top 8); larger k: slide_topk_kernel

__device__ __forceinline__ bool kbetter(double pa, int ba, double pb, int bb) { return pa > pb || (pa == pb && ba < bb); }

// the reference's insertion (gpuopt-nodetrend.mq5:545-552): the first slot s with p > tp[s] takes (p, j),
// the slots after it shift down one; branch-free over the sorted register list
template <int K> __device__ __forceinline__ void topk_insert(double (&tp)[K], int (&tb)[K], double p, int j) {
    bool c[K];
#pragma unroll
    for (int s = 0; s < K; ++s) c[s] = p > tp[s];
#pragma unroll
    for (int s = K - 1; s > 0; --s) {
        tp[s] = c[s] ? (c[s - 1] ? tp[s - 1] : p) : tp[s];
        tb[s] = c[s] ? (c[s - 1] ? tb[s - 1] : j) : tb[s];
    }
    tp[0] = c[0] ? p : tp[0];
    tb[0] = c[0] ? j : tb[0];
}
// Merge the LPW sorted partial lists (power desc, index asc) of a window held by lanes mw + WB q: log2 LPW
// rounds of exchange with the partner lane, each keeping the best K of the two lists by a bitonic merge
// (best of mine[s] and the partner's [K-1-s] is the union's top K in bitonic order; half-cleaners sort it).
// Every lane of the window ends with the same sorted top K.
template <int K, int WB, int LPW> __device__ __forceinline__ void merge_parts(double (&tp)[K], int (&tb)[K]) {
#pragma unroll
    for (int r = 1; r < LPW; r <<= 1) {
        double op[K];
        int ob[K];
#pragma unroll
        for (int s = 0; s < K; ++s) {
            op[s] = __shfl_xor(tp[s], WB * r, 64);
            ob[s] = __shfl_xor(tb[s], WB * r, 64);
        }
#pragma unroll
        for (int s = 0; s < K; ++s) {
            const bool t = kbetter(op[K - 1 - s], ob[K - 1 - s], tp[s], tb[s]);
            tp[s] = t ? op[K - 1 - s] : tp[s];
            tb[s] = t ? ob[K - 1 - s] : tb[s];
        }
#pragma unroll
        for (int h = K / 2; h > 0; h >>= 1)
#pragma unroll
            for (int i = 0; i < K; ++i)
                if ((i & h) == 0) {
                    const bool t = kbetter(tp[i + h], tb[i + h], tp[i], tb[i]);
                    const double pa = tp[i], pb = tp[i + h];
                    const int ba = tb[i], bb = tb[i + h];
                    tp[i] = t ? pb : pa;
                    tp[i + h] = t ? pa : pb;
                    tb[i] = t ? bb : ba;
                    tb[i + h] = t ? ba : bb;
                }
    }
}

constexpr int kCand = 8;  // candidate list entries per lane of the transposed scan (+1 scratch slot)

template <int LOG2N, int NF, int DETREND, int NB, int WB>
__global__ __launch_bounds__(64) void slide_topk_t_kernel(SlideArgs a) {
    constexpr int N = 1 << LOG2N, M = N / 2, REC = Rec<NF>::n, CHT = 128, LPW = 64 / WB, K = kTopkT;
    constexpr int kEmpty = 0x7fffffff;  // bin of an empty slot: sorts after every real bin
    __shared__ double u[CHT * REC];
    extern __shared__ d2 xs[];  // [WB][span | 1], sized at launch: the LDS a wave holds sets the occupancy
    const int l = threadIdx.x;
    const int64_t w0 = (int64_t)blockIdx.x * a.seg;
    if (w0 >= a.n_windows) return;
    const int len = (int)((a.n_windows - w0) < a.seg ? (a.n_windows - w0) : a.seg);
    const double *__restrict__ x = static_cast<const double *>(a.series) + w0;
    const d2 *__restrict__ omega = static_cast<const d2 *>(a.omega);
    const d2 *__restrict__ hwin = omega + NF * M;
    const d2 *__restrict__ ws = static_cast<const d2 *>(a.ws) + blockIdx.x * slide_topk_seed_stride(NF, a.span);
    const int span = a.span, kmin = a.kmin, sp = span | 1;
    d2 tr[NB][NF], om[NB][NF], hk[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int j = l + 64 * b;
        const bool ok = j < span;
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            tr[b][f] = ok ? ws[f * span + j] : d2{0.0, 0.0};
            om[b][f] = ok ? omega[f * M + kmin + j] : d2{1.0, 0.0};
        }
        hk[b] = (DETREND == kDetrendMean && ok) ? hwin[kmin + j] : d2{0.0, 0.0};
    }
    const d2 sl = ws[NF * span];
    double sum = sl.x;
    const double lvl = sl.y;
    // the scan's lane roles: window mw of the staged batch, band part mq: bins mq, mq + LPW, ...
    const int mw = l % WB, mq = l / WB;
    double *__restrict__ rec = static_cast<double *>(a.out) + w0 * (int64_t)(4 * a.topk);
    const int kk = a.topk;
    double tp[K];
    int tb[K], pb[K];
    bool have_prev = false;
    double *cp = reinterpret_cast<double *>(xs + WB * sp);  // candidate lists [kCand + 1][64] powers, bins
    int *cj = reinterpret_cast<int *>(cp + (kCand + 1) * 64);
    for (int c0 = 0; c0 < len; c0 += CHT) {
        const int clen = len - c0 < CHT ? len - c0 : CHT;
        if (c0) __syncthreads();
        stage_uniforms<double, NF, N>(a, x, lvl, c0, clen, len, u, l, 64);
        __syncthreads();
#pragma unroll 1
        for (int st = 0; st < clen; ++st) {
            const int wi = c0 + st, slot = wi % WB;
            const double mwv = DETREND == kDetrendMean ? sum * a.inv_n : 0.0;
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                d2 X = tr[b][0];
#pragma unroll
                for (int f = 1; f < NF; ++f) X += tr[b][f];
                if constexpr (DETREND == kDetrendMean) X -= mwv * hk[b];
                const int j = l + 64 * b;
                if (j < span) xs[slot * sp + j] = X;
            }
            if (wi + 1 < len) slide_step<NB, NF, DETREND>(tr, om, u + st * REC, sum);
            if (slot != WB - 1 && wi + 1 < len) continue;
            // ---- scan the staged batch: windows wi - slot .. wi
            __syncthreads();
            const bool wok = mw <= slot;
            const d2 *row = xs + mw * sp;
            // Threshold: the powers, in THIS window, of the 8 bins that won this lane's window slot in the
            // previous batch (window - WB).  They are 8 distinct bins of this window, so their minimum is
            // at most its 8th largest power: every bin of its top 8 -- ties at the 8th included -- has
            // p >= tau.  Only those candidates take the 8-slot insertion; the rest cost a compare.
            double tau = -1.0;
            if (have_prev && wok) {
                tau = __builtin_inf();
#pragma unroll
                for (int s = 0; s < K; ++s) {
                    const d2 X = row[pb[s] != kEmpty ? pb[s] : 0];
                    tau = fmin(tau, pb[s] != kEmpty ? X.x * X.x + X.y * X.y : -1.0);
                }
            }
            // candidates of this lane's part (bins mq, mq + LPW, ...: ascending, interleaved so that the
            // strong low bins spread over the parts) into the lane's LDS list [C + 1][64]
            int cnt = 0;
            if (wok) {
                for (int j = mq; j < span; j += 4 * LPW) {
                    double pw[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int jj = j + i * LPW;
                        const d2 X = row[jj < span ? jj : mq];
                        pw[i] = jj < span ? X.x * X.x + X.y * X.y : -1.0;
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int at = cnt < kCand ? cnt : kCand;  // slot kCand: scratch for overflow
                        cp[at * 64 + l] = pw[i];
                        cj[at * 64 + l] = j + i * LPW;
                        cnt += pw[i] >= tau ? 1 : 0;
                    }
                }
            }
#pragma unroll
            for (int s = 0; s < K; ++s) tp[s] = -1.0, tb[s] = kEmpty;
            if (__ballot(cnt > kCand) == 0) {
                for (int i = 0; __ballot(i < cnt) != 0; ++i) {  // the candidates, in ascending bin order
                    const bool on = i < cnt;
                    topk_insert<K>(tp, tb, on ? cp[i * 64 + l] : -1.0, on ? cj[i * 64 + l] : kEmpty);
                }
            } else if (wok) {  // a part with more candidates than the list holds (first batch of a segment): all bins
                for (int j = mq; j < span; j += 4 * LPW) {
                    double pw[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int jj = j + i * LPW;
                        const d2 X = row[jj < span ? jj : mq];
                        pw[i] = jj < span ? X.x * X.x + X.y * X.y : -1.0;
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) topk_insert<K>(tp, tb, pw[i], j + i * LPW);
                }
            }
            merge_parts<K, WB, LPW>(tp, tb);  // the LPW partial lists of a window (lanes mw + WB q)
#pragma unroll
            for (int s = 0; s < K; ++s) pb[s] = tb[s];  // this slot's winners: the next batch's threshold bins
            have_prev = true;
            // records of window (wi - slot + mw): part mq writes slots mq * K / LPW ..
            if (wok) {
                double *o = rec + (int64_t)(wi - slot + mw) * (4 * kk);
                constexpr int PER = K / LPW > 0 ? K / LPW : 1;
#pragma unroll
                for (int e = 0; e < PER; ++e) {
                    const int s = mq * PER + e;
                    // slot s of the lists by selects (register arrays are indexed at compile time only)
                    double ps = tp[0];
                    int bs = tb[0];
#pragma unroll
                    for (int i = 1; i < K; ++i) {
                        ps = s == i ? tp[i] : ps;
                        bs = s == i ? tb[i] : bs;
                    }
                    if (s < K && s < kk) {
                        const bool real = bs != kEmpty;
                        d2 X = d2{0.0, 0.0};
                        if (real) X = xs[mw * sp + bs];
                        typedef double d4 __attribute__((ext_vector_type(4)));
                        *reinterpret_cast<d4 *>(o + 4 * s) =
                            real ? d4{(double)(kmin + bs), ps, X.x, X.y} : d4{-1.0, -1.0, 0.0, 0.0};
                    }
                }
            }
            __syncthreads();  // the scan's reads before the next batch's writes
        }
    }
}

// ---- the same records by a probe threshold (default for k <= 8 and bands <= 256 bins).
// The wave slides its band's trackers bin-major (lane l: bins kmin + l + 64 b) and, per window, keeps
// only the bins that can be in the top k: tau = the smallest power, in THIS window, of the k bins that won
// the same slot of the previous batch (WB windows earlier; the segment's first window seeds every slot).
// Those are k distinct bins of this window, so tau is at most its k-th largest power and every member of
// its top k -- ties at the k-th included -- has p >= tau (compared on the high words: a superset).  The
// probes live in registers, one bit per slot in the owner lane's mask, so tau is one 32-bit wave min.
// The candidates (8.4 per window on average at C4, 11 at the 99th percentile) go to the slot's list in LDS
// in ascending bin order (ballot + mbcnt); after WB windows each lane takes one window and runs the
// reference's k-slot insertion (strict '>', gpuopt-nodetrend.mq5:545-552) over its list only.  A window
// with more than kPCand candidates, or the segment's first, is scanned exactly by the one-wave reduction
// (core::topk_wave64), whose winners then probe that slot.
constexpr int kPCand = 16;  // candidate list entries per window (default form)

// The LDS a wave holds sets the occupancy (one wave per workgroup): WB windows per batch x C candidates
// (20 B each) + CHT staged steps of uniforms + the fallback's band.
template <int LOG2N, int NF, int DETREND, int NB, int WB, int C = 16, int CHT = 128, int LB = 1>
__global__ __launch_bounds__(64, (NB > 2 && LB > 2) ? 2 : LB) void slide_topk_p_kernel(SlideArgs a) {
    constexpr int N = 1 << LOG2N, M = N / 2, REC = Rec<NF>::n, K = kTopkT;
    constexpr int kEmpty = 0x7fffffff;
    static_assert(WB <= 32 && CHT % WB == 0, "one lane and one mask bit per window of a batch");
    __shared__ double u[CHT * REC];
    __shared__ core::cpx<double> xb[64 * NB];  // the fallback's band
    __shared__ int win[K];                     // the fallback's winners (band index, -1 empty)
    __shared__ unsigned nm[64 * NB];           // next batch's probe bits per band bin
    __shared__ int cnt[WB];                    // candidates per slot, -1: the fallback wrote the record
    __shared__ d2 cx[WB * C];                  // candidates' X, per slot in ascending bin order
    __shared__ int cb[WB * C];                 // candidates' band indices
    const int l = threadIdx.x;
    const int64_t w0 = (int64_t)blockIdx.x * a.seg;
    if (w0 >= a.n_windows) return;
    // diagnostic timeline (wsp_plan_set_trace): [start, end] of this workgroup
    long long *trs = a.trace && a.trace_cap / 2 + 2 * ((int64_t)blockIdx.x + 1) <= a.trace_cap && l == 0
                         ? a.trace + a.trace_cap / 2 + 2 * (int64_t)blockIdx.x
                         : nullptr;
    if (trs) trs[0] = wall_clock64();
    const int len = (int)((a.n_windows - w0) < a.seg ? (a.n_windows - w0) : a.seg);
    const double *__restrict__ x = static_cast<const double *>(a.series) + w0;
    const d2 *__restrict__ omega = static_cast<const d2 *>(a.omega);
    const d2 *__restrict__ hwin = omega + NF * M;
    const d2 *__restrict__ ws = static_cast<const d2 *>(a.ws) + blockIdx.x * slide_topk_seed_stride(NF, a.span);
    const int span = a.span, kmin = a.kmin;
    d2 tr[NB][NF], om[NB][NF], hk[NB];
    unsigned mask[NB];  // bit s: this lane's bin of slot b is one of slot s's probes
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int j = l + 64 * b;
        const bool ok = j < span;
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            tr[b][f] = ok ? ws[f * span + j] : d2{0.0, 0.0};
            om[b][f] = ok ? omega[f * M + kmin + j] : d2{1.0, 0.0};
        }
        hk[b] = (DETREND == kDetrendMean && ok) ? hwin[kmin + j] : d2{0.0, 0.0};
        mask[b] = 0u;
        nm[j] = 0u;
    }
    const d2 sl = ws[NF * span];
    double sum = sl.x;
    const double lvl = sl.y;
    double *__restrict__ rec = static_cast<double *>(a.out) + w0 * (int64_t)(4 * a.topk);
    const int kk = a.topk;
    const bool probes = span >= kk;  // every window's winners are min(k, span) real bins
    for (int c0 = 0; c0 < len; c0 += CHT) {
        const int clen = len - c0 < CHT ? len - c0 : CHT;
        __syncthreads();
        stage_uniforms<double, NF, N>(a, x, lvl, c0, clen, len, u, l, 64);
        __syncthreads();
#pragma unroll 1
        for (int st = 0; st < clen; ++st) {
            const int wi = c0 + st, slot = wi % WB;
            // this step's uniforms into registers first: the LDS latency then overlaps the window's scan instead of
            // sitting in front of the slide (the last window's are never used)
            double ur[REC];
#pragma unroll
            for (int i = 0; i < REC; ++i) ur[i] = u[st * REC + i];
            const double mwv = DETREND == kDetrendMean ? sum * a.inv_n : 0.0;
            d2 X[NB];
            int ph[NB];  // high words of the powers (non-negative doubles order as their bits); INT_MIN outside
            int mh = 0x7fffffff;
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                d2 v = tr[b][0];
#pragma unroll
                for (int f = 1; f < NF; ++f) v += tr[b][f];
                if constexpr (DETREND == kDetrendMean) v -= mwv * hk[b];
                X[b] = v;
                const double p = v.x * v.x + v.y * v.y;
                ph[b] = l + 64 * b < span ? (int)(__builtin_bit_cast(unsigned long long, p) >> 32) : INT_MIN;
                if ((mask[b] >> slot) & 1u) mh = min(mh, ph[b]);
            }
            const int th = (wi > 0 && probes) ? core::wave_min64(mh) : 0;
            unsigned long long bal[NB];
            int total = 0;
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                bal[b] = __ballot(ph[b] >= th - 1);  // one high-word step of slack: any contraction of |X|^2
                total += __popcll(bal[b]);
            }
            if (wi > 0 && total <= C) {
                int base = 0;
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    if ((bal[b] >> l) & 1) {
                        const int pos = slot * C + base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal[b] >> 32),
                                                                                       __builtin_amdgcn_mbcnt_lo((unsigned)bal[b], 0u));
                        cx[pos] = X[b];
                        cb[pos] = l + 64 * b;
                    }
                    base += __popcll(bal[b]);
                }
                if (l == 0) cnt[slot] = total;
                if (a.flags && l == 0) a.flags[w0 + wi] = 0;
            } else {  // exact one-wave scan of this window; its winners probe the slot from now on
#pragma unroll
                for (int b = 0; b < NB; ++b) xb[l + 64 * b] = core::cpx<double>{X[b].x, X[b].y};
                __syncthreads();
                core::topk_wave64<NB, double>(xb, kmin, span, kk, l, rec + (int64_t)wi * (4 * kk), true, win);
                if (l == 0) cnt[slot] = -1;
                if (a.flags && l == 0) a.flags[w0 + wi] = wi == 0 ? 1 : 2;
                __syncthreads();
                if (l < kk && win[l] >= 0) atomicOr(&nm[win[l]], 1u << slot);
                __syncthreads();
                if (wi == 0) {  // the segment's first window probes every slot of the first batch
#pragma unroll
                    for (int b = 0; b < NB; ++b) mask[b] = nm[l + 64 * b] ? 0xffffffffu : 0u;
                }
            }
            if (wi + 1 < len) slide_step<NB, NF, DETREND>(tr, om, ur, sum);
            if (slot != WB - 1 && wi + 1 < len) continue;
            // ---- the staged batch: windows wi - slot .. wi, LPW = 64 / WB lanes per window (lane l: window
            // mw = l % WB, candidates q, q + LPW, ... of it, q = l / WB), merged across the window's lanes
            __syncthreads();
            constexpr int LPW = 64 / WB;
            const int mw = l % WB, q = l / WB;
            const int n = mw <= slot ? cnt[mw] : -1;
            double tp[K];
            int tb[K];
#pragma unroll
            for (int s = 0; s < K; ++s) tp[s] = -1.0, tb[s] = kEmpty;
            for (int i = q; __ballot(i < n) != 0; i += LPW) {
                const bool on = i < n;
                const d2 v = cx[mw * C + (on ? i : 0)];
                topk_insert<K>(tp, tb, on ? v.x * v.x + v.y * v.y : -1.0, on ? i : kEmpty);  // i: ascending bins
            }
            merge_parts<K, WB, LPW>(tp, tb);  // (power desc, index asc): the sequential insertion's order
            if (n >= 0 && q == 0) {
                double *o = rec + (int64_t)(wi - slot + mw) * (4 * kk);
                typedef double d4 __attribute__((ext_vector_type(4)));
#pragma unroll
                for (int s = 0; s < K; ++s) {
                    if (s < kk) {
                        const bool real = tb[s] != kEmpty;
                        const int ci = real ? mw * C + tb[s] : 0;
                        const d2 v = cx[ci];
                        const int bj = cb[ci];
                        // (plain stores: written through to memory -- agent-scope sc1, 32 B per slot, a partial line
                        // each -- the whole batch took 0.769 ms against 0.361 and a 1/8 shard 0.093 against 0.074, r05s)
                        *reinterpret_cast<d4 *>(o + 4 * s) = real ? d4{(double)(kmin + bj), tp[s], v.x, v.y} : d4{-1.0, -1.0, 0.0, 0.0};
                        if (real) atomicOr(&nm[bj], 1u << mw);
                    }
                }
            }
            __syncthreads();
#pragma unroll
            for (int b = 0; b < NB; ++b) {  // the batch's winners become the next batch's probes
                mask[b] = nm[l + 64 * b];
                nm[l + 64 * b] = 0u;
            }
        }
    }
    if (trs) trs[1] = wall_clock64();
}

template <int LOG2N, int NF, int DETREND> hipError_t launch_topk_t(const SlideArgs &a, hipStream_t s) {
    const int64_t grid = (a.n_windows + a.seg - 1) / a.seg;
    if constexpr (LOG2N >= 10) {
        const int chain = a.seed_chain > 1 ? a.seed_chain : 1;
        constexpr int TP = (1 << LOG2N) / 16;
        const dim3 sg((unsigned)((grid + chain - 1) / chain)), sb(TP);
        if (a.span <= TP) hipLaunchKernelGGL((slide_seed_r_kernel<LOG2N, NF, DETREND, 1>), sg, sb, 0, s, a);
        else if (a.span <= 2 * TP) hipLaunchKernelGGL((slide_seed_r_kernel<LOG2N, NF, DETREND, 2>), sg, sb, 0, s, a);
        else if (a.span <= 4 * TP) hipLaunchKernelGGL((slide_seed_r_kernel<LOG2N, NF, DETREND, 4>), sg, sb, 0, s, a);
        else hipLaunchKernelGGL((slide_seed_r_kernel<LOG2N, NF, DETREND, (kSlideTopkMaxSpan + TP - 1) / TP>), sg, sb, 0, s, a);
    } else {
        hipLaunchKernelGGL((slide_seed_kernel<double, LOG2N, NF, DETREND>), dim3((unsigned)grid), dim3(seed_nt<LOG2N>()), 0,
                           s, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int nb = (a.span + 63) / 64;
    // transposed scan for k <= 8 and bands of <= 256 bins (staged batch: WB windows x <= 64 NB bins); the
    // 512-bin form (NB = 8: 80 tracker registers per lane) stays on the one-wave scan.  WB: 16 windows per
    // staged batch (4 lanes per window, 2 merge rounds) while the batch takes <= 16 KiB of LDS, else 8
    // (variant 2 / 3 force 16 / 8: ablations)
    const size_t row = (size_t)(a.span | 1) * 2 * sizeof(double);
    const int wb = a.variant == 2 ? 16 : (a.variant == 3 ? 8 : (16 * row <= (16u << 10) ? 16 : 8));
    static_assert(kCand >= 1, "candidate list");
    if (a.topk <= kTopkT && (a.variant == 0 || a.variant >= 4) && nb <= 4) {  // probe threshold
#define PROBE(...)                                                                                                       \
    do {                                                                                                                 \
        if (nb <= 1) hipLaunchKernelGGL((slide_topk_p_kernel<LOG2N, NF, DETREND, 1, __VA_ARGS__>), dim3((unsigned)grid), dim3(64), 0, s, a); \
        else if (nb <= 2) hipLaunchKernelGGL((slide_topk_p_kernel<LOG2N, NF, DETREND, 2, __VA_ARGS__>), dim3((unsigned)grid), dim3(64), 0, s, a); \
        else hipLaunchKernelGGL((slide_topk_p_kernel<LOG2N, NF, DETREND, 4, __VA_ARGS__>), dim3((unsigned)grid), dim3(64), 0, s, a); \
    } while (0)
        // the LDS per wave sets the occupancy: 16 windows per batch x 16 candidates + 64 staged steps = 9.8 KiB and
        // <= 128 VGPRs: 4 waves per SIMD (C4 top-8 0.389 ms; 32 windows x 16 candidates + 128 steps = 17 KiB:
        // 2.25 waves per SIMD, 0.449 ms; 32 x 12 + 64 steps = 12 KiB: 3 waves, 0.433 ms -- profiles/r03/s2)
        if (a.variant == 4) PROBE(32, kPCand, 128, 1);
        else if (a.variant == 5) PROBE(32, 12, 64, 3);
        else PROBE(16, kPCand, 64, 4);
#undef PROBE
        return hipGetLastError();
    }
    if (a.topk <= kTopkT && a.variant != 1 && nb <= 4) {
        const size_t lds = (size_t)wb * row + (size_t)(kCand + 1) * 64 * (sizeof(double) + sizeof(int));
        if (wb == 16) {
            if (nb <= 1) hipLaunchKernelGGL((slide_topk_t_kernel<LOG2N, NF, DETREND, 1, 16>), dim3((unsigned)grid), dim3(64), lds, s, a);
            else if (nb <= 2) hipLaunchKernelGGL((slide_topk_t_kernel<LOG2N, NF, DETREND, 2, 16>), dim3((unsigned)grid), dim3(64), lds, s, a);
            else hipLaunchKernelGGL((slide_topk_t_kernel<LOG2N, NF, DETREND, 4, 16>), dim3((unsigned)grid), dim3(64), lds, s, a);
        } else {
            if (nb <= 1) hipLaunchKernelGGL((slide_topk_t_kernel<LOG2N, NF, DETREND, 1, 8>), dim3((unsigned)grid), dim3(64), lds, s, a);
            else if (nb <= 2) hipLaunchKernelGGL((slide_topk_t_kernel<LOG2N, NF, DETREND, 2, 8>), dim3((unsigned)grid), dim3(64), lds, s, a);
            else hipLaunchKernelGGL((slide_topk_t_kernel<LOG2N, NF, DETREND, 4, 8>), dim3((unsigned)grid), dim3(64), lds, s, a);
        }
        return hipGetLastError();
    }
    if (nb <= 1) hipLaunchKernelGGL((slide_topk_kernel<LOG2N, NF, DETREND, 1>), dim3((unsigned)grid), dim3(64), 0, s, a);
    else if (nb <= 2) hipLaunchKernelGGL((slide_topk_kernel<LOG2N, NF, DETREND, 2>), dim3((unsigned)grid), dim3(64), 0, s, a);
    else if (nb <= 4) hipLaunchKernelGGL((slide_topk_kernel<LOG2N, NF, DETREND, 4>), dim3((unsigned)grid), dim3(64), 0, s, a);
    else hipLaunchKernelGGL((slide_topk_kernel<LOG2N, NF, DETREND, 8>), dim3((unsigned)grid), dim3(64), 0, s, a);
    return hipGetLastError();
}

template <int LOG2N, int NF> hipError_t topk_by_detrend(const SlideArgs &a, hipStream_t s) {
    return a.detrend == kDetrendMean ? launch_topk_t<LOG2N, NF, kDetrendMean>(a, s)
                                     : launch_topk_t<LOG2N, NF, kDetrendNone>(a, s);
}

template <int LOG2N> hipError_t topk_by_nf(const SlideArgs &a, hipStream_t s) {
    switch (a.nf) {
    case 1: return topk_by_detrend<LOG2N, 1>(a, s);
    case 3: return topk_by_detrend<LOG2N, 3>(a, s);
    case 5: return topk_by_detrend<LOG2N, 5>(a, s);
    default: return hipErrorInvalidValue;
    }
}

// One launch over every member of the group: segment length from the residency (occupancy API, once
// per instantiation) and the members' total window count, so that a multi-symbol batch gets the same
// segments as one long series would (C5: 7 symbols of ~19k windows each seed 4-8x fewer times than
// as separate launches).
template <typename T, int LOG2N, int NF, int DETREND>
hipError_t launch_t(const SlideArgs &a0, const SlideGroup &g0, hipStream_t s) {
    constexpr int NT = (1 << LOG2N) / (2 * slide_b<LOG2N>());
    static std::atomic<int> resident{0};
    int res = resident.load(std::memory_order_relaxed);
    if (res == 0) {
        int per_cu = 0, dev = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, slide_kernel<T, LOG2N, NF, DETREND>, NT, 0) !=
                hipSuccess ||
            hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return hipErrorInvalidValue;
        res = per_cu * cus > 0 ? per_cu * cus : 256;
        resident.store(res, std::memory_order_relaxed);
    }
    SlideArgs a = a0;
    SlideGroup g = g0;
    int64_t total = 0;
    for (int m = 0; m < g.n; ++m) total += g.n_windows[m];
    if (a.seg <= 0) {
        // Round 6 (profiles/r06/c4_seg): 128-window segments from four rounds of them on, 64-window
        // segments from one round of those on, below that one round of resident workgroups (>= 32 windows each).
        // The round-2..5 policy -- one round of resident workgroups, at most 256 windows -- left a one-round launch
        // (a 1/8 C4 shard: 767 workgroups of 171 windows) waiting for its slowest workgroups: workgroups with equal
        // work ended between 107 and 222 us (slide_timeline, the older workgroups of a CU run ahead and the last one
        // finishes alone).  With several rounds of shorter segments a CU whose workgroups finish early takes new
        // ones.  Measured on C4 (N = 2048, Hann, 768 slots): whole batch 1.570 -> 1.482-1.520 ms at 128 (64: 1.527,
        // 96-160: 1.57-1.63), 1/2 shard 0.797 -> 0.744 at 128, 1/4 0.408 -> 0.384 at 64, 1/8 0.220 -> 0.196-0.201 at
        // 64 (48-144: 0.209-0.233).
        const int64_t slots = a.share > 1.0 ? (int64_t)((double)res / a.share) + 1 : (int64_t)res;
        if (total >= 4 * slots * 128) {
            a.seg = 128;
        } else if (total >= slots * 64) {
            a.seg = 64;
        } else {
            a.seg = (total + slots - 1) / slots;
            a.seg = a.seg < 32 ? 32 : a.seg;
        }
    }
    g.blk0[0] = 0;
    for (int m = 0; m < g.n; ++m) g.blk0[m + 1] = g.blk0[m] + (g.n_windows[m] + a.seg - 1) / a.seg;
    const int64_t grid = g.blk0[g.n];
    if (grid <= 0) return hipSuccess;
    hipLaunchKernelGGL((slide_kernel<T, LOG2N, NF, DETREND>), dim3((unsigned)grid), dim3(NT), 0, s, a, g);
    return hipGetLastError();
}

template <typename T, int LOG2N, int NF> hipError_t by_detrend(const SlideArgs &a, const SlideGroup &g, hipStream_t s) {
    return a.detrend == kDetrendMean ? launch_t<T, LOG2N, NF, kDetrendMean>(a, g, s)
                                     : launch_t<T, LOG2N, NF, kDetrendNone>(a, g, s);
}

template <typename T, int LOG2N> hipError_t by_nf(const SlideArgs &a, const SlideGroup &g, hipStream_t s) {
    switch (a.nf) {
    case 1: return by_detrend<T, LOG2N, 1>(a, g, s);
    case 3: return by_detrend<T, LOG2N, 3>(a, g, s);
    case 5: return by_detrend<T, LOG2N, 5>(a, g, s);
    default: return hipErrorInvalidValue;
    }
}

template <typename T> hipError_t by_n(const SlideArgs &a, const SlideGroup &g, hipStream_t s) {
    switch (a.log2n) {
    case 9: return by_nf<T, 9>(a, g, s);
    case 10: return by_nf<T, 10>(a, g, s);
    case 11: return by_nf<T, 11>(a, g, s);
    case 12: return by_nf<T, 12>(a, g, s);
    case 13: return by_nf<T, 13>(a, g, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

// top-k launchers, one translation unit per window length (slide_topk_l<LOG2N>.hip)
hipError_t launch_slide_topk_l9(const SlideArgs &a, hipStream_t s);
hipError_t launch_slide_topk_l10(const SlideArgs &a, hipStream_t s);
hipError_t launch_slide_topk_l11(const SlideArgs &a, hipStream_t s);
hipError_t launch_slide_topk_l12(const SlideArgs &a, hipStream_t s);
hipError_t launch_slide_topk_l13(const SlideArgs &a, hipStream_t s);
// power rows, one translation unit per element type (slide_power_f32.hip / sliding_dft.hip)
hipError_t launch_slide_group_f32(const SlideArgs &a, const SlideGroup &g, hipStream_t s);
hipError_t launch_slide_group_f64(const SlideArgs &a, const SlideGroup &g, hipStream_t s);

}  // namespace wsp
