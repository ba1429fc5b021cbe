// large_fft.hip -- windows of N = 32768 .. 262144 samples (SURVEY 8f rank 4:
// the legacy InpFFTWindow menu up to 262144, default 65536 in
// L/WaveSpecZZ_1.0.4-new.mq5:657).
//
// One window no longer fits a workgroup (M = N/2 complex points = 256 KiB ..
// 2 MiB), so the M-point complex FFT of z[n] = x[2n] + i x[2n+1] runs as a
// four-step transform, M = M1 x M2, n = n1 + M1 n2, k = k2 + M2 k1:
//
//   col_kernel  per window and block of CB consecutive n1: gather the column
//               z[n1 + M1 n2] (CB x 16 B contiguous per row), detrend (mean)
//               + window on load, M2-point FFT over n2, twiddle W_M^(n1 k2),
//               store Y[k2][n1] (rows of M1 complex).
//   row_kernel  per window and block of RB rows k2 plus their mirror rows
//               M2 - k2: M1-point FFT of each row -> Z[k2 + M2 k1]; the real
//               post-processing pairs Z[k] with Z[M - k], which sits in the
//               mirror row of the same workgroup (row 0 and row M2/2 pair
//               with themselves); |X_k|^2 or the packed (Re, Im) layout,
//               staged through LDS so that each row block leaves as runs of
//               RB consecutive bins.
//
// Y for a chunk of windows (about 192 MiB: the measured optimum between
// launch count and Infinity-Cache residency) is written and read back right
// away.  Each workgroup walks several windows of the chunk with a register
// prefetch of the next window's slice.  Both kernels share one workgroup FFT: 16
// complex points per thread, L/16 threads per transform, Stockham passes
// of radix 16 (and one of 2/4/8), LDS between passes (+1 pad per 16), and
// the twiddles of every pass from the W_N table.
//
// Detrend: mean by a per-window reduction pre-pass (mean_kernel), IIR trend
// by a per-window scan pre-pass (iir_kernel, restarts per window as
// L/WaveSpecZZ_1.0.2.mq5:3040-3053), Kalman by the common pre-pass; the
// latter two write detrended windows that the column pass reads with hop = N.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>

#include "spectrum_dispatch.h"
#include "wg_fft.h"

namespace wsp {
namespace large {

using core::cadd;
using core::cconj;
using core::cmul;
using core::cpx;
using core::csub;
using core::dft;
using core::pad16;

using wg::LGeo;
using wg::last_radix;
using wg::wg_fft;

struct ColArgs {
    const void *series;  // window w at series + w*hop
    void *y;             // chunk rows: Y[wc][k2][n1]
    const void *tw;      // W_N^k, k < N
    const double *means; // per window (mean detrend) or null
    int64_t hop, w0, nwin;  // windows w0 .. w0 + nwin - 1 of this chunk
    int log2n, vec;
    double a0, a1, a2, cd, sd, c1, s1, inv_theta, inv_nm1;  // window: rotation by th*2*M1*TP per r, th per odd sample
};

constexpr int kCB = 16;  // columns per workgroup in col_kernel (CB: 8 for fp64 M2 = 512, see col_cb)

template <typename T, int LOG2M1, int LOG2M2, int WCLASS, bool MEAN, int CB = kCB>
__global__ __launch_bounds__(CB *(1 << LOG2M2) / 16) void col_kernel(ColArgs a) {
    using G = LGeo<LOG2M2>;
    constexpr int M1 = 1 << LOG2M1, M2 = G::L, TP = G::TP, NB1 = M1 / CB;
    constexpr bool kCos = WCLASS == core::kWinCos || WCLASS == core::kWinCos2;
    // the CB column transforms interleaved element by element (wg_fft stride S = CB, round 6): with one contiguous
    // slot per column (SLOT = M2 + M2/16 complex = a multiple of 32 dwords) the 8 lanes of a ds_write_b128 group and
    // the 16 of a ds_read_b128 group, which hold adjacent columns, all hit the same banks (8-way conflicts on every
    // exchange); one element of padding per column still left 2-3-way read conflicts at CB = 8 / 16 (SQ pass r06s:
    // 0.40 of the col_kernel's LDS cycles at N = 262144)
    __shared__ cpx<T> lds[CB * G::SLOT];
    const int tid = threadIdx.x, c = tid % CB, t = tid / CB;
    const int beta = blockIdx.x % NB1;
    const int n1 = beta * CB + c;
    const T *__restrict__ series = static_cast<const T *>(a.series);
    const cpx<T> *__restrict__ tw = static_cast<const cpx<T> *>(a.tw);
    cpx<T> *__restrict__ y = static_cast<cpx<T> *>(a.y);
    const int N = 1 << a.log2n;
    // window angle of sample 2n at r = 0: th * 2 (n1 + M1 t); per r: + th * 2 M1 TP
    double cw0 = 1.0, sw0 = 0.0;
    if constexpr (kCos) sincos(a.inv_theta * (double)(2 * (n1 + M1 * t)), &sw0, &cw0);
    using v2 = typename core::V2<T>::t;
    v2 raw[16];
    auto load = [&](int64_t wc) {  // the 16 sample pairs of this thread's column slice of window w0 + wc
        const T *__restrict__ xw = series + (a.w0 + wc) * a.hop;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int n = n1 + M1 * (t + TP * r);
            if (a.vec) {
                raw[r] = __builtin_nontemporal_load(reinterpret_cast<const v2 *>(xw + 2 * n));
            } else {
                raw[r].x = xw[2 * n];
                raw[r].y = xw[2 * n + 1];
            }
        }
    };
    // register prefetch of the next window (64 VGPRs in fp64) except at fp64 M2 = 512, whose FFT leaves no room
    // for it within 256 VGPRs (the 8-column form overlaps loads and FFTs by running two workgroups per CU instead)
    constexpr bool kPrefetch = LOG2M2 < 9 || sizeof(T) == 4;
    const int64_t wstep = gridDim.x / NB1;
    int64_t wc = blockIdx.x / NB1;
    if (kPrefetch && wc < a.nwin) load(wc);
    for (; wc < a.nwin; wc += wstep) {
        if (!kPrefetch) load(wc);
        const double mean = MEAN ? a.means[a.w0 + wc] : 0.0;
        cpx<T> v[16];
        double cw = cw0, sw = sw0;
        if constexpr (kCos) asm volatile("" : "+v"(cw), "+v"(sw));
        int nb = n1 + M1 * t;  // sample pair index of r = 0, advanced per r (pinned: no 16-value hoist)
        if constexpr (WCLASS == core::kWinBartlett) asm volatile("" : "+v"(nb));
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int n = nb + M1 * TP * r;
            double xa = (double)raw[r].x, xb = (double)raw[r].y;
            if constexpr (MEAN) {
                xa -= mean;
                xb -= mean;
            }
            if constexpr (kCos) {
                const double co = cw * a.c1 - sw * a.s1;  // odd sample: th + th1
                if constexpr (WCLASS == core::kWinCos2) {
                    xa *= a.a0 + a.a1 * cw + a.a2 * (2.0 * cw * cw - 1.0);
                    xb *= a.a0 + a.a1 * co + a.a2 * (2.0 * co * co - 1.0);
                } else {
                    xa *= a.a0 + a.a1 * cw;
                    xb *= a.a0 + a.a1 * co;
                }
                const double cn = cw * a.cd - sw * a.sd;
                sw = sw * a.cd + cw * a.sd;
                cw = cn;
            } else if constexpr (WCLASS == core::kWinBartlett) {  // L/WaveSpecZZ_1.0.2.mq5:918-922
                xa *= 1.0 - fabs((2.0 * (2 * n) - N + 1) * a.inv_nm1);
                xb *= 1.0 - fabs((2.0 * (2 * n + 1) - N + 1) * a.inv_nm1);
            }
            v[r] = {(T)xa, (T)xb};
        }
        if (kPrefetch && wc + wstep < a.nwin) load(wc + wstep);  // next window's samples in flight during this FFT
        wg_fft<T, LOG2M2, 1, CB>(v, lds + c, t, tw, a.log2n);
        // v[q R + r] = X[k2], k2 = t + TP q + (M2/R) r; twiddle W_M^(n1 k2) = W_N^(2 n1 k2)
        constexpr int R = last_radix<LOG2M2>();
        cpx<T> *__restrict__ yw = y + wc * (int64_t)M2 * M1;
        const cpx<T> wstep_r = tw[(2 * n1 * (M2 / R)) & (N - 1)];
#pragma unroll
        for (int q = 0; q < 16 / R; ++q) {
            cpx<T> wr = tw[(2 * n1 * (t + TP * q)) & (N - 1)];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int k2 = t + TP * q + (M2 / R) * r;
                yw[(int64_t)k2 * M1 + n1] = cmul(v[q * R + r], wr);
                if (r + 1 < R) wr = cmul(wr, wstep_r);
            }
        }
    }
}

struct RowArgs {
    const void *y;   // Y[wc][k2][n1]
    void *out;       // window w's record at out + w * record
    const void *tw;  // W_N^k
    int64_t w0, nwin;
    int log2n;
    int packed;      // 0: |X_k|^2 (N/2 per window); 1: out[2k] = Re X_k, out[2k+1] = Im X_k (N per window)
    long long *trace;  // fused kernel diagnostic timeline (wsp_plan_set_trace), nullptr = off
    int64_t trace_cap;
};

template <int LOG2M1> struct RowGeo {
    static constexpr int RB = LOG2M1 >= 8 ? 8 : 16;  // rows (and mirror rows) per workgroup
};

template <typename T, int LOG2M1, int LOG2M2, bool PACKED, bool XCD = true>
__global__ __launch_bounds__(2 * RowGeo<LOG2M1>::RB *(1 << LOG2M1) / 16) void row_kernel(RowArgs a) {
    using G = LGeo<LOG2M1>;
    constexpr int RB = RowGeo<LOG2M1>::RB;
    constexpr int M1 = G::L, M2 = 1 << LOG2M2, TP = G::TP, NB2 = (M2 / 2) / RB;
    constexpr int64_t M = (int64_t)M1 * M2;
    __shared__ cpx<T> lds[2 * RB * G::SLOT];
    const int tid = threadIdx.x, rho = tid / TP, t = tid % TP;
    // XCD-aware block order: blocks b and b + 8 share an XCD (round-robin dealing, MI355X_MICROARCH.md), so
    // virtual block (b % 8) * (grid / 8) + b / 8 puts row blocks beta and beta + 1 -- each writes runs of RB
    // consecutive bins, the two halves of the same output lines at RB = 8 in fp64 -- on one XCD's L2
    const int vb = XCD && gridDim.x % 8 == 0 ? (int)(blockIdx.x % 8) * (int)(gridDim.x / 8) + (int)(blockIdx.x / 8)
                                             : (int)blockIdx.x;
    const int beta = vb % NB2;
    // slot rho < RB: row beta*RB + rho; slot RB + i: row M2 - (beta*RB + i), or M2/2 for i = 0 of block 0
    auto row_of = [&](int s) {
        const int i = s < RB ? s : s - RB, lo = beta * RB + i;
        return s < RB ? lo : (lo == 0 ? M2 / 2 : M2 - lo);
    };
    const int row = row_of(rho);
    const cpx<T> *__restrict__ tw = static_cast<const cpx<T> *>(a.tw);
    const int N = 1 << a.log2n;
    cpx<T> *slot = lds + rho * G::SLOT;
    const int64_t wstep = gridDim.x / NB2;
    int64_t wc = vb / NB2;
    cpx<T> nxt[16];
    auto load = [&](int64_t w) {
        const cpx<T> *__restrict__ yr = static_cast<const cpx<T> *>(a.y) + (w * M2 + row) * (int64_t)M1;
#pragma unroll
        for (int r = 0; r < 16; ++r) nxt[r] = yr[t + TP * r];
    };
    if (wc < a.nwin) load(wc);
    for (; wc < a.nwin; wc += wstep) {
        cpx<T> v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = nxt[r];
        if (wc + wstep < a.nwin) load(wc + wstep);  // next window's rows in flight during this one
        // the row's TP threads are lanes of one wave and its slot is theirs: wave-local exchanges (round 6; N = 131072
        // 1.378 -> 1.353-1.368 ms, 262144 1.641 -> 1.633, r06x same box)
        static_assert(TP <= 64 && 64 % TP == 0, "a row's threads in one wave");
        wg_fft<T, LOG2M1, 1, 1, true>(v, slot, t, tw, a.log2n);
        // Z[row + M2 k1] in v[q R + r], k1 = t + TP q + (M1/R) r: to LDS in natural order
        constexpr int R = last_radix<LOG2M1>();
#pragma unroll
        for (int q = 0; q < 16 / R; ++q)
#pragma unroll
            for (int r = 0; r < R; ++r) slot[pad16(t + TP * q + (M1 / R) * r)] = v[q * R + r];
        __syncthreads();
        // X[k] = E + W_N^k O, E = (Z_k + conj Z_{M-k})/2, O = (Z_k - conj Z_{M-k})/(2i)
        const bool self = row == 0 || row == M2 / 2;
        const cpx<T> *pslot = lds + (self ? rho : (rho < RB ? rho + RB : rho - RB)) * G::SLOT;
        T res[16][PACKED ? 2 : 1];
        const cpx<T> wstep_r = tw[(M2 * (M1 / R)) & (N - 1)];  // W_N^k along r: k += M2 M1/R
#pragma unroll
        for (int q = 0; q < 16 / R; ++q) {
            cpx<T> wk = tw[(row + M2 * (t + TP * q)) & (N - 1)];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int k1 = t + TP * q + (M1 / R) * r;
                const int pk1 = row == 0 ? ((M1 - k1) & (M1 - 1)) : (M1 - 1 - k1);
                const cpx<T> z = v[q * R + r], zp = cconj(pslot[pad16(pk1)]);
                const cpx<T> e = {T(0.5) * (z.re + zp.re), T(0.5) * (z.im + zp.im)};
                const cpx<T> d = {T(0.5) * (z.re - zp.re), T(0.5) * (z.im - zp.im)};
                const cpx<T> o = {d.im, -d.re};  // d / i
                const cpx<T> x = cadd(e, cmul(wk, o));
                if (r + 1 < R) wk = cmul(wk, wstep_r);
                if constexpr (PACKED) {
                    res[q * R + r][0] = x.re;
                    res[q * R + r][1] = x.im;
                } else {
                    res[q * R + r][0] = x.re * x.re + x.im * x.im;
                }
            }
        }
        __syncthreads();  // partner reads done: the LDS becomes the output stage [k1][slot]
        constexpr int E = PACKED ? 2 : 1;
        T *stage = reinterpret_cast<T *>(lds);  // (M1 x 2RB) records of E values
#pragma unroll
        for (int q = 0; q < 16 / R; ++q)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int k1 = t + TP * q + (M1 / R) * r;
#pragma unroll
                for (int e = 0; e < E; ++e) stage[(k1 * (2 * RB + 1) + rho) * E + e] = res[q * R + r][e];
            }
        __syncthreads();
        // runs of RB consecutive bins per (k1, half): lanes over slots
        T *__restrict__ ow = static_cast<T *>(a.out) + (a.w0 + wc) * (int64_t)(PACKED ? 2 * M : M);
        constexpr int NT = 2 * RB * TP;
        for (int i = tid; i < M1 * 2 * RB; i += NT) {
            const int s = i % (2 * RB), k1 = i / (2 * RB);
            const int64_t k = row_of(s) + (int64_t)M2 * k1;
#pragma unroll
            for (int e = 0; e < E; ++e) ow[k * E + e] = stage[(k1 * (2 * RB + 1) + s) * E + e];
        }
        __syncthreads();  // stage reads done before the next window's FFT
    }
}

// ---------------------------------------------------------------- fused form
// One workgroup per window at a time (persistent: workgroup g takes windows g, g + grid, ...): the
// column pass and the row pass of the same window back to back, the column results Y in a slot of
// the workgroup's own (M complex) that the next window reuses.  With one workgroup per CU the slots
// in flight are 256 x 512 KiB = 128 MiB at N = 65536, inside the 256 MiB Infinity Cache, so the Y round
// trip is served from cache instead of HBM (two-pass form: the whole chunk's Y goes through HBM, PMC
// 2.38x the algorithmic bytes).  The probe that priced this (tools/mall_probe.hip,
// profiles/r02/large_slot_probe.log): the algorithmic bytes alone 620-665 us, + ~330 us for the
// recycled-slot round trip.  Same arithmetic as col_kernel / row_kernel (same wg_fft, twiddles and
// post-processing).  The workgroup's own stores of Y are visible to its loads after __syncthreads
// (workgroup-scope release / acquire; one CU, one L1).
template <typename T, int LOG2M1, int LOG2M2, int WCLASS, bool MEAN, bool PACKED, int NT = 256, bool PF = true,
          bool NTS = false, bool TR = false>
__global__ __launch_bounds__(NT) void fused_kernel(ColArgs a, RowArgs ra) {
    using GC = LGeo<LOG2M2>;
    using GR = LGeo<LOG2M1>;
    constexpr int M1 = GR::L, M2 = GC::L, TPC = GC::TP, TPR = GR::TP;
    // NT threads: CB columns per column block, RB rows (+ RB mirror rows) per row block; both fill the
    // LDS (CB x SLOT or 2 RB x SLOT complex: 70 KiB at NT = 256; at 512 threads the FFT's ~250 VGPRs
    // spill 350 B/lane), one workgroup per CU
    constexpr int CB = NT / TPC, RB = NT / (2 * TPR), NB1 = M1 / CB, NB2 = (M2 / 2) / RB;
    static_assert(CB * TPC == NT && 2 * RB * TPR == NT && NB1 >= 1 && NB2 >= 1, "thread geometry");
    constexpr int64_t M = (int64_t)M1 * M2;
    constexpr bool kCos = WCLASS == core::kWinCos || WCLASS == core::kWinCos2;
    // column transforms interleaved element by element (wg_fft stride S = CB; col_kernel): adjacent columns (adjacent
    // lanes) in different LDS banks -- the column FFT took 8.5 of a column block's 13 us with contiguous per-column
    // slots (r06o timeline), 4.3-4.7 with one element of padding per column (r06p)
    constexpr int LDS_C = CB * GC::SLOT, LDS_R = 2 * RB * GR::SLOT;
    __shared__ cpx<T> lds[LDS_C > LDS_R ? LDS_C : LDS_R];
    const int tid = threadIdx.x;
    const T *__restrict__ series = static_cast<const T *>(a.series);
    const cpx<T> *__restrict__ tw = static_cast<const cpx<T> *>(a.tw);
    cpx<T> *__restrict__ y = static_cast<cpx<T> *>(a.y) + (int64_t)blockIdx.x * M;  // this workgroup's slot
    const int N = 1 << a.log2n;
    using v2 = typename core::V2<T>::t;
    // column pass geometry (col_kernel): column c of the block, transform thread t
    const int cc = tid % CB, ct = tid / CB;
    // row pass geometry (row_kernel): slot rho, transform thread t
    const int rho = tid / TPR, rt = tid % TPR;
    v2 raw[16];
    auto load_cols = [&](int64_t w, int beta) {  // 16 sample pairs of column beta * CB + cc
        const T *__restrict__ xw = series + w * a.hop;
        const int n1 = beta * CB + cc;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int n = n1 + M1 * (ct + TPC * r);
            if (a.vec) {
                raw[r] = __builtin_nontemporal_load(reinterpret_cast<const v2 *>(xw + 2 * n));
            } else {
                raw[r].x = xw[2 * n];
                raw[r].y = xw[2 * n + 1];
            }
        }
    };
    cpx<T> nxt[16];
    auto load_rows = [&](int beta2) {
        const int i = rho < RB ? rho : rho - RB, lo = beta2 * RB + i;
        const int row = rho < RB ? lo : (lo == 0 ? M2 / 2 : M2 - lo);
        const cpx<T> *__restrict__ yr = y + (int64_t)row * M1;
#pragma unroll
        for (int r = 0; r < 16; ++r) nxt[r] = yr[rt + TPR * r];
    };
    // window angle of this thread's first sample pair in column block 0 (th * 2 (cc + M1 ct)), and the
    // rotation by th * 2 CB from one column block to the next (<= NB1 - 1 steps): no sincos in the loop
    double cw00 = 1.0, sw00 = 0.0, cbd = 1.0, sbd = 0.0;
    if constexpr (kCos) {
        sincos(a.inv_theta * (double)(2 * (cc + M1 * ct)), &sw00, &cw00);
        sincos(a.inv_theta * (double)(2 * CB), &sbd, &cbd);
    }
    // diagnostic timeline (wsp_plan_set_trace, scripts/large_timeline.py): thread 0 of workgroup b records, for its
    // first window only, 4 ticks per block -- start, samples / rows in registers (loads done), FFT done, block done --
    // for the NB1 column blocks then the NB2 row blocks, at trace[32 b + 4 i] (NB1 + NB2 <= 8 blocks)
    // (TR: a separate instantiation, so that the default kernel carries none of it)
    long long *trc = (TR && ra.trace && threadIdx.x == 0 && 32 * (int64_t)blockIdx.x + 32 <= ra.trace_cap)
                         ? ra.trace + 32 * (int64_t)blockIdx.x : nullptr;
    for (int64_t w = blockIdx.x; w < a.nwin; w += gridDim.x) {
        if (w != blockIdx.x) trc = nullptr;
        // ---- column pass: NB1 blocks of CB columns
        if (PF) load_cols(w, 0);
        const double mean = MEAN ? a.means[w] : 0.0;
        double cwb = cw00, swb = sw00;  // angle of column block beta
        for (int beta = 0; beta < NB1; ++beta) {
            if (trc && beta < 8) trc[4 * beta] = wall_clock64();
            if (!PF) load_cols(w, beta);
            const int n1 = beta * CB + cc;
            double cw = cwb, sw = swb;
            if constexpr (kCos) {
                const double cn = cwb * cbd - swb * sbd;
                swb = swb * cbd + cwb * sbd;
                cwb = cn;
            }
            int nb = n1 + M1 * ct;
            if constexpr (WCLASS == core::kWinBartlett) asm volatile("" : "+v"(nb));
            cpx<T> v[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = nb + M1 * TPC * r;
                double xa = (double)raw[r].x, xb = (double)raw[r].y;
                if constexpr (MEAN) {
                    xa -= mean;
                    xb -= mean;
                }
                if constexpr (kCos) {
                    const double co = cw * a.c1 - sw * a.s1;
                    if constexpr (WCLASS == core::kWinCos2) {
                        xa *= a.a0 + a.a1 * cw + a.a2 * (2.0 * cw * cw - 1.0);
                        xb *= a.a0 + a.a1 * co + a.a2 * (2.0 * co * co - 1.0);
                    } else {
                        xa *= a.a0 + a.a1 * cw;
                        xb *= a.a0 + a.a1 * co;
                    }
                    const double cn = cw * a.cd - sw * a.sd;
                    sw = sw * a.cd + cw * a.sd;
                    cw = cn;
                } else if constexpr (WCLASS == core::kWinBartlett) {  // L/WaveSpecZZ_1.0.2.mq5:918-922
                    xa *= 1.0 - fabs((2.0 * (2 * n) - N + 1) * a.inv_nm1);
                    xb *= 1.0 - fabs((2.0 * (2 * n + 1) - N + 1) * a.inv_nm1);
                }
                v[r] = {(T)xa, (T)xb};
            }
            if (trc && beta < 8) {  // samples consumed: loads done
                asm volatile("" ::"v"(v[15].re));
                trc[4 * beta + 1] = wall_clock64();
            }
            // next block's samples in flight during this FFT (not across the row pass: registers)
            if (PF && beta + 1 < NB1) load_cols(w, beta + 1);
            wg_fft<T, LOG2M2, 1, CB>(v, lds + cc, ct, tw, a.log2n);
            if (trc && beta < 8) {
                asm volatile("" ::"v"(v[15].re));
                trc[4 * beta + 2] = wall_clock64();
            }
            constexpr int R = last_radix<LOG2M2>();
            const cpx<T> wstep_r = tw[(2 * n1 * (M2 / R)) & (N - 1)];
#pragma unroll
            for (int q = 0; q < 16 / R; ++q) {
                cpx<T> wr = tw[(2 * n1 * (ct + TPC * q)) & (N - 1)];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int k2 = ct + TPC * q + (M2 / R) * r;
                    y[(int64_t)k2 * M1 + n1] = cmul(v[q * R + r], wr);
                    if (r + 1 < R) wr = cmul(wr, wstep_r);
                }
            }
            if (trc && beta < 8) trc[4 * beta + 3] = wall_clock64();
        }
        __syncthreads();  // Y of this window complete and visible to the workgroup
        // ---- row pass: NB2 blocks of RB rows + their mirror rows
        if (PF) load_rows(0);
        for (int beta2 = 0; beta2 < NB2; ++beta2) {
            const int ti = 4 * (NB1 + beta2);
            if (trc && ti + 3 < 32) trc[ti] = wall_clock64();
            if (!PF) load_rows(beta2);
            const int i = rho < RB ? rho : rho - RB, lo = beta2 * RB + i;
            const int row = rho < RB ? lo : (lo == 0 ? M2 / 2 : M2 - lo);
            cpx<T> *slot = lds + rho * GR::SLOT;
            cpx<T> v[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = nxt[r];
            if (trc && ti + 3 < 32) {
                asm volatile("" ::"v"(v[15].re));  // the rows are in registers
                trc[ti + 1] = wall_clock64();
            }
            if (PF && beta2 + 1 < NB2) load_rows(beta2 + 1);
            // (workgroup barriers: the wave-local exchanges that the two-pass row kernel takes measured 1.186 -> 1.200
            // ms here, r06x; profiles/r06/large/r06x_ab_wave_local_rows.log)
            wg_fft<T, LOG2M1>(v, slot, rt, tw, a.log2n);
            if (trc && ti + 3 < 32) {
                asm volatile("" ::"v"(v[15].re));
                trc[ti + 2] = wall_clock64();
            }
            constexpr int R = last_radix<LOG2M1>();
            // the R2C step's twiddles, loaded before the barrier (round 6: behind it their L2 latency was exposed)
            cpx<T> wk0[16 / R];
#pragma unroll
            for (int q = 0; q < 16 / R; ++q) wk0[q] = tw[(row + M2 * (rt + TPR * q)) & (N - 1)];
#pragma unroll
            for (int q = 0; q < 16 / R; ++q)
#pragma unroll
                for (int r = 0; r < R; ++r) slot[pad16(rt + TPR * q + (M1 / R) * r)] = v[q * R + r];
            __syncthreads();
            const bool self = row == 0 || row == M2 / 2;
            const cpx<T> *pslot = lds + (self ? rho : (rho < RB ? rho + RB : rho - RB)) * GR::SLOT;
            T res[16][PACKED ? 2 : 1];
            const cpx<T> wstep_r = tw[(M2 * (M1 / R)) & (N - 1)];
#pragma unroll
            for (int q = 0; q < 16 / R; ++q) {
                cpx<T> wk = wk0[q];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int k1 = rt + TPR * q + (M1 / R) * r;
                    const int pk1 = row == 0 ? ((M1 - k1) & (M1 - 1)) : (M1 - 1 - k1);
                    const cpx<T> z = v[q * R + r], zp = cconj(pslot[pad16(pk1)]);
                    const cpx<T> e = {T(0.5) * (z.re + zp.re), T(0.5) * (z.im + zp.im)};
                    const cpx<T> d = {T(0.5) * (z.re - zp.re), T(0.5) * (z.im - zp.im)};
                    const cpx<T> o = {d.im, -d.re};
                    const cpx<T> x = cadd(e, cmul(wk, o));
                    if (r + 1 < R) wk = cmul(wk, wstep_r);
                    if constexpr (PACKED) {
                        res[q * R + r][0] = x.re;
                        res[q * R + r][1] = x.im;
                    } else {
                        res[q * R + r][0] = x.re * x.re + x.im * x.im;
                    }
                }
            }
            __syncthreads();
            constexpr int E = PACKED ? 2 : 1;
            T *stage = reinterpret_cast<T *>(lds);
#pragma unroll
            for (int q = 0; q < 16 / R; ++q)
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int k1 = rt + TPR * q + (M1 / R) * r;
#pragma unroll
                    for (int e = 0; e < E; ++e) stage[(k1 * (2 * RB + 1) + rho) * E + e] = res[q * R + r][e];
                }
            __syncthreads();
            T *__restrict__ ow = static_cast<T *>(ra.out) + w * (int64_t)(PACKED ? 2 * M : M);
            for (int ii = tid; ii < M1 * 2 * RB; ii += NT) {
                const int sl = ii % (2 * RB), k1 = ii / (2 * RB);
                const int il = sl < RB ? sl : sl - RB, l2 = beta2 * RB + il;
                const int64_t k = (sl < RB ? l2 : (l2 == 0 ? M2 / 2 : M2 - l2)) + (int64_t)M2 * k1;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const T o = stage[(k1 * (2 * RB + 1) + sl) * E + e];
                    if constexpr (NTS) __builtin_nontemporal_store(o, ow + k * E + e);  // keep the slots in the MALL
                    else ow[k * E + e] = o;
                }
            }
            __syncthreads();
            if (trc && ti + 3 < 32) trc[ti + 3] = wall_clock64();
        }
    }
}

// ---------------------------------------------------------------- pre-passes

// Per-window mean (L/WaveSpecZZ_gpu_wip.mq5:940-950) for the column pass.
template <typename T>
__global__ __launch_bounds__(256) void mean_kernel(const T *__restrict__ series, int64_t hop, int64_t n_windows, int n,
                                                   double *__restrict__ means) {
    __shared__ double red[4];
    for (int64_t w = blockIdx.x; w < n_windows; w += gridDim.x) {
        const T *__restrict__ xw = series + w * hop;
        double s = 0.0;
        for (int i = threadIdx.x; i < n; i += 256) s += (double)xw[i];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) means[w] = (red[0] + red[1] + red[2] + red[3]) / (double)n;
        __syncthreads();
    }
}

// Per-window IIR trend detrend (L/WaveSpecZZ_1.0.2.mq5:3040-3053, restarting
// at every window): t0 = c (x0 + x0), tj = c (xj + x(j-1)) + alpha t(j-1),
// d = x - t.  1024 threads per window, C = N/1024 consecutive samples each:
// local filter from a zero state, affine carry scan across threads
// (multipliers apow[j] = alpha^(C 2^j)), then the chunk again with its carry.
struct IirPow {
    double alpha, c;
    double apow[8];  // alpha^(C 2^j), C = N/1024 samples per thread
};

template <typename T>
__global__ __launch_bounds__(1024) void iir_kernel(const T *__restrict__ series, int64_t hop, int64_t n_windows, int n,
                                                  IirPow ip, T *__restrict__ dout) {
    __shared__ double wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const double alpha = ip.alpha, c = ip.c;
    const double *apow = ip.apow;
    const int C = n / 1024;
    for (int64_t w = blockIdx.x; w < n_windows; w += gridDim.x) {
        const T *__restrict__ xw = series + w * hop;
        const int j0 = tid * C;
        double prev = (double)xw[j0 == 0 ? 0 : j0 - 1];
        double tr = 0.0;
        for (int j = 0; j < C; ++j) {
            const double x = (double)xw[j0 + j];
            tr = c * (x + prev) + alpha * tr;
            prev = x;
        }
        // inclusive scan of (A = alpha^C, tr) within the wave, then across the 16 waves
        double v = tr;
#pragma unroll
        for (int k = 0, d = 1; d < 64; ++k, d <<= 1) {
            const double up = __shfl_up(v, d, 64);
            if (lane >= d) v = apow[k] * up + v;
        }
        if (lane == 63) wsum[wv] = v;
        __syncthreads();
        double G = 0.0;  // state entering this wave: sum over earlier waves, apow[6] = alpha^(64 C)
        for (int i = 0; i < wv; ++i) G = apow[6] * G + wsum[i];
        // carry into this thread = state after the previous chunk
        double carry = __shfl_up(v, 1, 64);
        double p = 1.0;  // alpha^(C lane)
#pragma unroll
        for (int k = 0; k < 6; ++k)
            if ((lane >> k) & 1) p *= apow[k];
        carry = lane == 0 ? G : carry + p * G;
        if (tid == 0) carry = 0.0;
        __syncthreads();  // wsum reuse
        tr = carry;
        prev = (double)xw[j0 == 0 ? 0 : j0 - 1];
        T *__restrict__ dw = dout + w * (int64_t)n;
        for (int j = 0; j < C; ++j) {
            const double x = (double)xw[j0 + j];
            tr = c * (x + prev) + alpha * tr;
            prev = x;
            dw[j0 + j] = (T)(x - tr);
        }
    }
}

}  // namespace large

// ------------------------------------------------------------------- launch
namespace {

int cu_count() {
    static const int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 256;
        return n > 0 ? n : 256;
    }();
    return cus;
}

// windows in flight: enough workgroups for every CU's LDS (two per CU at
// 70 KiB), each walking several windows of the chunk with a prefetch
int64_t windows_in_flight(int64_t nwin, int blocks_per_window, size_t lds_bytes) {
    const int64_t per_cu = std::max<int64_t>(1, (160 * 1024) / (int64_t)lds_bytes);
    const int64_t slots = per_cu * cu_count();
    return std::max<int64_t>(1, std::min<int64_t>(nwin, slots / blocks_per_window));
}

template <typename T, int LM1, int LM2, int WC, bool MEAN, int CB = large::kCB>
hipError_t col_launch_cb(const large::ColArgs &a, hipStream_t s) {
    constexpr int NB1 = (1 << LM1) / CB;
    const int64_t g = windows_in_flight(a.nwin, NB1, CB * large::LGeo<LM2>::SLOT * sizeof(core::cpx<T>)) * NB1;
    hipLaunchKernelGGL((large::col_kernel<T, LM1, LM2, WC, MEAN, CB>), dim3((unsigned)g), dim3(CB * (1 << LM2) / 16), 0,
                       s, a);
    return hipGetLastError();
}

// fp64 M2 = 512 (N = 262144): 8 columns per workgroup by default -- 256 threads and 70 KiB of LDS, so two
// independent workgroups per CU whose loads, FFTs and stores overlap, against one 512-thread workgroup per CU
// (16 columns, 139 KiB: loads, FFT and stores back to back); variant 6 keeps the 16-column form (A/B)
template <typename T, int LM1, int LM2, int WC, bool MEAN>
hipError_t col_launch(const large::ColArgs &a, int variant, hipStream_t s) {
    if constexpr (LM2 == 9 && sizeof(T) == 8)
        if (variant != 6) return col_launch_cb<T, LM1, LM2, WC, MEAN, 8>(a, s);
    if constexpr (LM2 == 8 && sizeof(T) == 8)  // variant 8: the same 8-column form at M2 = 256 (N = 65536, two passes)
        if (variant == 8) return col_launch_cb<T, LM1, LM2, WC, MEAN, 8>(a, s);
    return col_launch_cb<T, LM1, LM2, WC, MEAN>(a, s);
}

// variant 7: the row pass in plain block order (A/B of the XCD-aware order)
template <typename T, int LM1, int LM2, bool PACKED>
hipError_t row_launch(const large::RowArgs &a, int variant, hipStream_t s) {
    constexpr int RB = large::RowGeo<LM1>::RB, NB2 = ((1 << LM2) / 2) / RB;
    const int64_t g = windows_in_flight(a.nwin, NB2, 2 * RB * large::LGeo<LM1>::SLOT * sizeof(core::cpx<T>)) * NB2;
    if (variant == 7)
        hipLaunchKernelGGL((large::row_kernel<T, LM1, LM2, PACKED, false>), dim3((unsigned)g), dim3(2 * RB * (1 << LM1) / 16), 0, s, a);
    else
        hipLaunchKernelGGL((large::row_kernel<T, LM1, LM2, PACKED>), dim3((unsigned)g), dim3(2 * RB * (1 << LM1) / 16), 0, s, a);
    return hipGetLastError();
}

template <typename T, int LM1, int LM2> hipError_t chunk_launch(const LargeLaunch &L, const large::ColArgs &ca,
                                                                const large::RowArgs &ra, int wclass, bool mean,
                                                                hipStream_t s) {
    hipError_t e;
    using namespace core;
#define COL(WC)                                                                            \
    e = mean ? col_launch<T, LM1, LM2, WC, true>(ca, L.variant, s) : col_launch<T, LM1, LM2, WC, false>(ca, L.variant, s)
    switch (wclass) {
    case kWinCos: COL(kWinCos); break;
    case kWinCos2: COL(kWinCos2); break;
    case kWinBartlett: COL(kWinBartlett); break;
    default: COL(kWinNone); break;
    }
#undef COL
    if (e != hipSuccess) return e;
    return L.packed ? row_launch<T, LM1, LM2, true>(ra, L.variant, s) : row_launch<T, LM1, LM2, false>(ra, L.variant, s);
}

// the fused form for M2 = 256 (N = 65536, 131072): one launch over every window (ablations: variant 3 =
// 512 threads without register prefetch, two waves per SIMD; variant 4 = 256 threads with prefetch)
template <typename T, int LM1, int NT, bool PF, bool NTS = false>
hipError_t fused_launch(const LargeLaunch &L, const large::ColArgs &ca0, const large::RowArgs &ra, int wclass, bool mean,
                        hipStream_t s) {
    large::ColArgs ca = ca0;
    ca.w0 = 0;
    ca.nwin = L.n_windows;
    // workgroups in flight: one per CU (the slots stay in the Infinity Cache; two per CU measured 1.90 ms
    // against 1.51), never more slots than the plan workspace holds (a chunk of windows)
    const int per_cu = 1;
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>({L.n_windows, L.chunk, (int64_t)per_cu * cu_count()}));
    using namespace core;
    if constexpr (sizeof(T) == 8 && NT == 512 && !PF && NTS) {  // diagnostic timeline of the default form (Hann, power)
        if (ra.trace && !mean && !L.packed && wclass == kWinCos) {
            hipLaunchKernelGGL((large::fused_kernel<T, LM1, 8, kWinCos, false, false, NT, PF, NTS, true>), dim3((unsigned)grid),
                               dim3(NT), 0, s, ca, ra);
            return hipGetLastError();
        }
    }
#define FUSED(WC)                                                                                                          \
    if (mean) {                                                                                                            \
        if (L.packed) hipLaunchKernelGGL((large::fused_kernel<T, LM1, 8, WC, true, true, NT, PF, NTS>), dim3((unsigned)grid), dim3(NT), 0, s, ca, ra); \
        else hipLaunchKernelGGL((large::fused_kernel<T, LM1, 8, WC, true, false, NT, PF, NTS>), dim3((unsigned)grid), dim3(NT), 0, s, ca, ra); \
    } else {                                                                                                               \
        if (L.packed) hipLaunchKernelGGL((large::fused_kernel<T, LM1, 8, WC, false, true, NT, PF, NTS>), dim3((unsigned)grid), dim3(NT), 0, s, ca, ra); \
        else hipLaunchKernelGGL((large::fused_kernel<T, LM1, 8, WC, false, false, NT, PF, NTS>), dim3((unsigned)grid), dim3(NT), 0, s, ca, ra); \
    }
    switch (wclass) {
    case kWinCos: FUSED(kWinCos); break;
    case kWinCos2: FUSED(kWinCos2); break;
    case kWinBartlett: FUSED(kWinBartlett); break;
    default: FUSED(kWinNone); break;
    }
#undef FUSED
    return hipGetLastError();
}

hipError_t chunk_dispatch(int log2m, const LargeLaunch &L, const large::ColArgs &ca, const large::RowArgs &ra,
                          int wclass, bool mean, hipStream_t s, bool f32);

// two internal streams per device for the pipelined ablation (created once, never destroyed)
hipStream_t aux_stream(int i) {
    static std::mutex mu;
    static std::map<int, std::array<hipStream_t, 2>> streams;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    auto it = streams.find(dev);
    if (it == streams.end()) {
        std::array<hipStream_t, 2> a{};
        for (auto &x : a)
            if (hipStreamCreateWithFlags(&x, hipStreamNonBlocking) != hipSuccess) return nullptr;
        it = streams.emplace(dev, a).first;
    }
    return it->second[i];
}

template <typename T>
hipError_t pipelined_t(const LargeLaunch &L, large::ColArgs ca, large::RowArgs ra, int wclass, bool mean, int log2m,
                       hipStream_t s) {
    const int64_t chunk = std::max<int64_t>(1, L.chunk / 4);
    hipStream_t st[2] = {aux_stream(0), aux_stream(1)};
    if (!st[0] || !st[1]) return hipErrorInvalidValue;
    hipEvent_t fork, join[2];
    hipError_t e = hipEventCreateWithFlags(&fork, hipEventDisableTiming);
    if (e != hipSuccess) return e;
    for (auto &j : join)
        if ((e = hipEventCreateWithFlags(&j, hipEventDisableTiming)) != hipSuccess) return e;
    (void)hipEventRecord(fork, s);
    for (auto x : st) (void)hipStreamWaitEvent(x, fork, 0);
    const size_t ybytes = (size_t)chunk * ((size_t)1 << log2m) * sizeof(core::cpx<T>);
    int64_t i = 0;
    for (int64_t w0 = 0; w0 < L.n_windows; w0 += chunk, ++i) {
        ca.w0 = ra.w0 = w0;
        ca.nwin = ra.nwin = std::min<int64_t>(chunk, L.n_windows - w0);
        ca.y = static_cast<char *>(L.y) + (i % 2) * ybytes;  // two Y buffers (the workspace holds 4 chunks)
        ra.y = ca.y;
        if ((e = chunk_dispatch(log2m, L, ca, ra, wclass, mean, st[i % 2], sizeof(T) == 4)) != hipSuccess) return e;
    }
    for (int k = 0; k < 2; ++k) {
        (void)hipEventRecord(join[k], st[k]);
        (void)hipStreamWaitEvent(s, join[k], 0);
    }
    (void)hipEventDestroy(fork);
    for (auto j : join) (void)hipEventDestroy(j);
    return hipGetLastError();
}

template <typename T> hipError_t launch_t(const LargeLaunch &L, hipStream_t s) {
    const int log2m = L.log2n - 1;
    const int n = 1 << L.log2n;
    // pre-passes
    const void *src = L.series;
    int64_t hop = L.hop;
    const double *means = nullptr;
    if (L.detrend == kDetrendMean) {
        hipLaunchKernelGGL(large::mean_kernel<T>, dim3((unsigned)std::min<int64_t>(L.n_windows, 4096)), dim3(256), 0, s,
                           static_cast<const T *>(L.series), L.hop, L.n_windows, n, L.means);
        means = L.means;
    } else if (L.detrend == kDetrendIir) {
        large::IirPow ip{};
        ip.alpha = L.iir_alpha;
        ip.c = L.iir_c;
        long double pw = powl((long double)L.iir_alpha, (long double)(n / 1024));
        for (int j = 0; j < 8; ++j) {
            ip.apow[j] = (double)pw;
            pw = pw * pw;
        }
        hipLaunchKernelGGL(large::iir_kernel<T>, dim3((unsigned)std::min<int64_t>(L.n_windows, 1024)), dim3(1024), 0, s,
                           static_cast<const T *>(L.series), L.hop, L.n_windows, n, ip, static_cast<T *>(L.detrended));
        src = L.detrended;
        hop = n;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    large::ColArgs ca{};
    ca.series = src;
    ca.y = L.y;
    ca.tw = L.twiddle;
    ca.means = means;
    ca.hop = hop;
    ca.log2n = L.log2n;
    ca.vec = (hop % 2 == 0) && (reinterpret_cast<uintptr_t>(src) % (2 * sizeof(T)) == 0);
    const int wclass = core::window_class(L.window, &ca.a0, &ca.a1, &ca.a2);
    const int lm1 = log2m / 2, lm2 = log2m - lm1;  // M1 <= M2: the column pass takes the longer transform
    const long double two_pi = 6.283185307179586476925286766559005768L;
    const long double th = two_pi / (long double)(n - 1);
    ca.inv_theta = (double)th;
    ca.inv_nm1 = 1.0 / (double)(n - 1);
    const long double dstep = th * 2.0L * (long double)(1 << lm1) * (long double)((1 << lm2) / 16);
    ca.cd = (double)cosl(dstep);
    ca.sd = (double)sinl(dstep);
    ca.c1 = (double)cosl(th);
    ca.s1 = (double)sinl(th);
    large::RowArgs ra{};
    ra.y = L.y;
    ra.out = L.out;
    ra.tw = L.twiddle;
    ra.log2n = L.log2n;
    ra.packed = L.packed;
    ra.w0 = 0;
    ra.nwin = L.n_windows;
    ra.trace = L.trace;
    ra.trace_cap = L.trace_cap;
    // The fused one-workgroup-per-window form (fused_kernel, 512 threads, no register prefetch) is the default
    // for fp64 N = 65536, the legacy default window (4096 x 65536: 1.387 ms against 1.444 for the two-pass form,
    // profiles/r03/s2); N = 131072 would hold 192 slots of 1 MiB at most (a quarter of the CUs idle) and stays
    // two-pass, like fp32 (unmeasured fused).  Ablations (wsp_plan_set_variant): 1 = two-pass forced, 2 = two-pass
    // over quarter chunks on two internal streams, 3 = fused (N = 65536 / 131072), 4 = the 256-thread fused form
    // with register prefetch (1.516 ms: one wave per SIMD cannot hide the FFT's latencies).
    const bool fused_default = L.variant == 0 && log2m == 15 && sizeof(T) == 8;
    // (non-temporal output stores: the streamed spectra do not evict the slots from the Infinity Cache --
    // 1.376 -> 1.346 ms; variant 5 keeps plain stores)
    if ((L.variant == 3 || fused_default) && (log2m == 15 || log2m == 16))
        return log2m == 15 ? fused_launch<T, 7, 512, false, true>(L, ca, ra, wclass, means != nullptr, s)
                           : fused_launch<T, 8, 512, false, true>(L, ca, ra, wclass, means != nullptr, s);
    if (L.variant == 5 && log2m == 15)  // ablation: the fused form with plain output stores
        return fused_launch<T, 7, 512, false, false>(L, ca, ra, wclass, means != nullptr, s);
    if (L.variant == 4 && (log2m == 15 || log2m == 16))
        return log2m == 15 ? fused_launch<T, 7, 256, true>(L, ca, ra, wclass, means != nullptr, s)
                           : fused_launch<T, 8, 256, true>(L, ca, ra, wclass, means != nullptr, s);
    // the pipelined form alternates two Y buffers of max(1, chunk / 4) windows: it needs the workspace to hold
    // two of them, which a one-window chunk (wsp_plan_set_chunk(plan, 1)) does not -- that plan runs the
    // plain chunk loop below instead of writing a second buffer past its workspace
    if (L.variant == 2 && L.chunk >= 2) return pipelined_t<T>(L, ca, ra, wclass, means != nullptr, log2m, s);
    for (int64_t w0 = 0; w0 < L.n_windows; w0 += L.chunk) {
        ca.w0 = ra.w0 = w0;
        ca.nwin = ra.nwin = std::min<int64_t>(L.chunk, L.n_windows - w0);
        switch (log2m) {
        case 14: e = chunk_launch<T, 7, 7>(L, ca, ra, wclass, means != nullptr, s); break;
        case 15: e = chunk_launch<T, 7, 8>(L, ca, ra, wclass, means != nullptr, s); break;
        case 16: e = chunk_launch<T, 8, 8>(L, ca, ra, wclass, means != nullptr, s); break;
        case 17: e = chunk_launch<T, 8, 9>(L, ca, ra, wclass, means != nullptr, s); break;
        default: return hipErrorInvalidValue;
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t chunk_dispatch(int log2m, const LargeLaunch &L, const large::ColArgs &ca, const large::RowArgs &ra,
                          int wclass, bool mean, hipStream_t s, bool f32) {
    if (f32) {
        switch (log2m) {
        case 14: return chunk_launch<float, 7, 7>(L, ca, ra, wclass, mean, s);
        case 15: return chunk_launch<float, 7, 8>(L, ca, ra, wclass, mean, s);
        case 16: return chunk_launch<float, 8, 8>(L, ca, ra, wclass, mean, s);
        case 17: return chunk_launch<float, 8, 9>(L, ca, ra, wclass, mean, s);
        default: return hipErrorInvalidValue;
        }
    }
    switch (log2m) {
    case 14: return chunk_launch<double, 7, 7>(L, ca, ra, wclass, mean, s);
    case 15: return chunk_launch<double, 7, 8>(L, ca, ra, wclass, mean, s);
    case 16: return chunk_launch<double, 8, 8>(L, ca, ra, wclass, mean, s);
    case 17: return chunk_launch<double, 8, 9>(L, ca, ra, wclass, mean, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

int64_t large_chunk(int log2n, bool f32) {
    constexpr int64_t mb = 192;  // measured best of 16..2048 MiB (profiles/r01/large_chunk_sweep.log)
    const int64_t per = (int64_t(1) << (log2n - 1)) * (f32 ? 8 : 16);
    const int64_t c = (mb << 20) / per;
    return c < 1 ? 1 : c;
}

hipError_t launch_large(const LargeLaunch &L, hipStream_t stream) {
    if (L.n_windows <= 0) return hipSuccess;
    return L.f32 ? launch_t<float>(L, stream) : launch_t<double>(L, stream);
}

}  // namespace wsp
