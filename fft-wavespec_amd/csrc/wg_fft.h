// wg_fft.h -- one complex FFT of L = 64 .. 8192 points held by L/16 threads of a workgroup, 16 points
// per thread in registers: Stockham passes of radix 16 (and one last pass of radix 2 / 4 / 8), the
// in-register DFTs with compile-time constants (core::dft), LDS only between passes (+1 element pad
// per 16: conflict-free strided writes), twiddles from the W_N table (one entry per butterfly, powers
// by products along r).  Used by the four-step large-N transform (large_fft.hip: column and row
// FFTs) and by the sliding DFT's segment seeds (sliding_core.h).
#pragma once
#include "spectrum_core.h"

namespace wsp {
namespace wg {

using core::cmul;
using core::cpx;
using core::dft;
using core::pad16;

template <int LOG2L> struct LGeo {
    static constexpr int L = 1 << LOG2L;
    static constexpr int TP = L / 16;                         // threads per transform
    static constexpr int NP = LOG2L / 4 + (LOG2L % 4 ? 1 : 0);  // passes
    static constexpr int radix(int p) { return p < LOG2L / 4 ? 16 : (1 << (LOG2L % 4)); }
    static constexpr int ns(int p) {
        int s = 1;
        for (int i = 0; i < p; ++i) s *= radix(i);
        return s;
    }
    static constexpr int SLOT = L + L / 16;  // padded LDS elements per transform
    static_assert(LOG2L >= 6 && LOG2L <= 13, "transform length 64 .. 8192");
};

// L-point forward FFT of one transform held by TP threads (16 points each:
// v[r] = x[t + TP r] on entry).  On exit v[q R + r] = X[b + (L/R) r] with
// b = t + TP q and R the last pass's radix.  `slot` is this transform's LDS
// region (SLOT elements); tw = W_N^j, j < N, of a table of period N (twN).
// S: element stride of the transform in LDS (round 6).  S = 1: the transform owns SLOT consecutive elements.  S = CB > 1:
// CB transforms interleaved element by element (element e of transform c at slot_base[c + CB pad16(e)], the caller
// passing slot = base + c): the lanes of one LDS instruction, which hold adjacent transforms at nearby elements, then
// fall on distinct banks for every pass (the column passes of large_fft.hip; contiguous per-column slots a multiple
// of 32 dwords apart made them 8-way conflicts, and a one-element pad still left 2-3-way read conflicts at 8 or 16
// columns per workgroup).
// WL (round 6): the transform's TP threads are lanes of one wave and its slot is private to them (the row transforms
// of large_fft.hip: 8 / 16 threads per row), so the exchanges only need the wave's own LDS ordering -- LDS executes a
// wave's instructions in order; the wait and the memory clobber keep the compiler from moving the reads above the
// writes -- instead of workgroup barriers that wait for every other wave.
template <bool WL> __device__ __forceinline__ void wg_sync() {
    if constexpr (WL) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    } else {
        __syncthreads();
    }
}

template <typename T, int LOG2L, int PASS = 1, int S = 1, bool WL = false>
__device__ __forceinline__ void wg_fft(cpx<T> (&v)[16], cpx<T> *slot, int t, const cpx<T> *__restrict__ tw, int log2tw) {
    using G = LGeo<LOG2L>;
    constexpr int L = G::L, TP = G::TP;
    if constexpr (PASS == 1) dft<T, 16>(v);  // pass 0: radix 16 over r, no twiddles (Ns = 1)
    if constexpr (PASS < G::NP) {
        // write the previous pass's outputs: butterfly b (Ns = ns(PASS-1), R = radix(PASS-1))
        constexpr int Rp = G::radix(PASS - 1), Nsp = G::ns(PASS - 1);
        constexpr int R = G::radix(PASS), Ns = G::ns(PASS);
        // twiddle W_{Ns R}^{j r} = W_N^{j r N/(Ns R)}: one table entry per butterfly, powers by products (<= 15
        // steps: ~15 ulp).  Loaded before the exchange's barrier (round 6): behind it the table read's L2 latency
        // was exposed on every pass (the barrier also orders global loads).
        cpx<T> w1s[16 / R];
#pragma unroll
        for (int q = 0; q < 16 / R; ++q) w1s[q] = tw[(((t + TP * q) % Ns) << log2tw) / (Ns * R)];
#pragma unroll
        for (int q = 0; q < 16 / Rp; ++q) {
            const int b = t + TP * q, j = b % Nsp, base = (b / Nsp) * Nsp * Rp + j;
#pragma unroll
            for (int r = 0; r < Rp; ++r) slot[S * pad16(base + Nsp * r)] = v[q * Rp + r];
        }
        wg_sync<WL>();
#pragma unroll
        for (int q = 0; q < 16 / R; ++q) {
            const int b = t + TP * q;
#pragma unroll
            for (int r = 0; r < R; ++r) v[q * R + r] = slot[S * pad16(b + (L / R) * r)];
            const cpx<T> w1 = w1s[q];
            cpx<T> wr = w1;
#pragma unroll
            for (int r = 1; r < R; ++r) {
                v[q * R + r] = cmul(v[q * R + r], wr);
                if (r + 1 < R) wr = cmul(wr, w1);
            }
            dft<T, R>(v + q * R);
        }
        wg_sync<WL>();  // slot reuse by the caller / next pass
        wg_fft<T, LOG2L, PASS + 1, S, WL>(v, slot, t, tw, log2tw);
    }
}

template <int LOG2L> __device__ __forceinline__ constexpr int last_radix() { return LGeo<LOG2L>::radix(LGeo<LOG2L>::NP - 1); }

}  // namespace wg
}  // namespace wsp
