// slide_mixed.hip -- a multi-symbol, mixed-length hop = 1 batch (C5: 28 symbols x N in {512, 1024, 2048,
// 4096}, the WaveCyclesBatchFetcher shape, WaveCyclesBatchFetcher.mq5:106-133) in ONE persistent launch of
// the seeded sliding DFT (sliding_core.h: the same seeds, slide steps, uniforms and stores as slide_kernel).
//
// Why one launch: as one launch per window length, every launch starts with all of its workgroups seeding at
// once (in-LDS FFTs, no writes in flight) and ends with a drain, and small batches (a strong-scaled shard of
// C5) pay both per length.  Here 512-thread workgroups, resident two per CU, pull tasks from a device counter:
// task = one segment of a 4096-pt member, or two 2048 / two 1024 / four 512 segments side by side (sub-
// workgroups of N/(2B) threads, wave-aligned, so the workgroup barriers of the seed FFTs line up: every
// sub-workgroup of a task has the same N).  Tasks are ordered longest windows first and each costs about the
// same (S windows x 2048 bins, half that for N <= 1024), so after the first task the workgroups' seed phases
// fall at different times and overlap the others' write streams, and the last tasks are the short ones.
//
// LDS: 4096 complex for the FFT buffers / staged uniforms of the sub-workgroups (P x N <= 4096) + the W_4096
// quarter table (W_N^k = W_4096^(k 4096/N)) = 80 KiB: two workgroups per CU, 4 waves per SIMD at <= 128 VGPRs.
// The task index is broadcast through the first LDS word between two barriers; the counter slot is reset by
// the last workgroup to leave, so the next execute on the slot starts from zero (mtbridge.cpp rings 256 slots).
#include "sliding_core.h"

namespace wsp {
namespace {

// In-place natural-order complex FFT of N points in LDS by the NT threads of a sub-workgroup (thread t): fft_lds
// with the twiddles read from the W_4096 quarter table at stride 4096 / N.  Barriers are workgroup-wide: every
// sub-workgroup of the workgroup runs the same N.
template <int LOG2N, int NT> __device__ __forceinline__ void fft_lds_sub(d2 *buf, const d2 *twq, int t) {
    constexpr int N = 1 << LOG2N, H = N / 2, N4 = N / 4, TS = 4096 / N;
    int ns = 1;
    if constexpr (LOG2N & 1) {
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
        const int tws = N / (4 * ns) * TS;
        d2 v[Q][4], w1[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int j = t + NT * q;
            w1[q] = twq[(j & (ns - 1)) * tws];
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
            const d2 t3 = d2{d.y, -d.x};
            const int o = ((j - k) << 2) + k;
            buf[o] = t0 + t2;
            buf[o + ns] = t1 + t3;
            buf[o + 2 * ns] = t0 - t2;
            buf[o + 3 * ns] = t1 - t3;
        }
        __syncthreads();
    }
}

// The kernel argument is read in place through the kernarg segment pointer (address space 4: scalar loads, any
// index).  Passing the struct by reference to the device functions made the compiler copy its 1.4 KiB to scratch.
typedef const __attribute__((address_space(4))) SlideMix *MixP;

// series / output and first window of class-c segment s (members of class c: [mem0[c], mem0[c + 1]), segments
// from sg0); false when s is past the class's last segment.  Unrolled selects over the kernel-argument table
// (no dynamic indexing of the argument struct).
__device__ __forceinline__ bool mix_seg(MixP m, int c, int64_t s, const void *&ser, void *&outp, int64_t &w0,
                                        int &len) {
    int lo = m->mem0[0], hi = m->mem0[1], nseg = m->nseg[0], seg = m->seg[0];
#pragma unroll
    for (int i = 1; i < kMixClass; ++i)
        if (c == i) lo = m->mem0[i], hi = m->mem0[i + 1], nseg = m->nseg[i], seg = m->seg[i];
    if (s >= nseg) return false;
    int64_t base = m->sg0[0], nw = m->n_windows[0];
    ser = m->series[0];
    outp = m->out[0];
#pragma unroll
    for (int i = 0; i < kMixMax; ++i)
        if (i >= lo && i < hi && s >= m->sg0[i]) base = m->sg0[i], nw = m->n_windows[i], ser = m->series[i], outp = m->out[i];
    w0 = (s - base) * seg;
    len = (int)(nw - w0 < seg ? nw - w0 : seg);
    return true;
}

template <typename T, int LOG2N, int NF, int DETREND, int BS, int SR>
__device__ __forceinline__ void mix_task(MixP m, int c, int64_t task, d2 *lds, const d2 *twq, long long *trace) {
    // BS: bins per thread for N <= 1024 (2 by default, the per-length launches' geometry: 0.737 against 0.777 ms
    // for C5 at 4, which holds 4 / 8 segments side by side; profiles/r04/ab).  One-wave 512-point sub-workgroups
    // with wave fences instead of lockstep barriers lost too (0.812 against 0.735 ms: the N = 512 tail then has
    // half the tasks, tools/ablations/c5_mixed_one_wave_512.patch)
    constexpr int N = 1 << LOG2N, M = N / 2, B = LOG2N <= 10 ? BS : 4, NT = M / B, P = kMixNT / NT, REC = Rec<NF>::n,
                  NM = (NF - 1) / 2;
    constexpr int CH = N / 4 < 128 ? 128 : (N / 4 > kSlideRMax ? kSlideRMax : N / 4);
    static_assert(P * N <= 4096 && CH * REC / 2 <= N && P * NT == kMixNT, "sub-workgroup geometry");
    // sub-workgroups are whole waves: the index (and the segment lookups below) are wave-uniform
    const int sub = __builtin_amdgcn_readfirstlane(threadIdx.x / NT);
    int t = threadIdx.x % NT;
    asm volatile("" : "+v"(t));  // per task: the bin addresses are not hoisted out of the task loop (and spilled)
    d2 *buf = lds + sub * N;
    // this sub-workgroup's segment, and the longest segment of the task (the trip count every sub-workgroup runs)
    int len = 0, maxlen = 0;
    int64_t w0 = 0;
    const void *ser = m->series[0];
    void *outp = m->out[0];
    const bool on = mix_seg(m, c, task * P + sub, ser, outp, w0, len);
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const void *ps;
        void *po;
        int pl = 0;
        int64_t pw;
        if (mix_seg(m, c, task * P + p, ps, po, pw, pl)) maxlen = pl > maxlen ? pl : maxlen;
    }
    const d2 *__restrict__ omega = static_cast<const d2 *>(m->omega[0]);
    double c1 = m->c1[0], sn1 = m->sn1[0], c2 = m->c2[0], sn2 = m->sn2[0], inv_n = m->inv_n[0];
#pragma unroll
    for (int i = 1; i < kMixClass; ++i)
        if (c == i) {
            omega = static_cast<const d2 *>(m->omega[i]);
            c1 = m->c1[i], sn1 = m->sn1[i], c2 = m->c2[i], sn2 = m->sn2[i], inv_n = m->inv_n[i];
        }
    const T *__restrict__ x = static_cast<const T *>(ser) + w0;
    const d2 *__restrict__ hwin = omega + NF * M;
    const d2 *__restrict__ mod = omega + (NF + 1) * M;  // [NM][N] e^{-j m th i}
    const double lvl = (DETREND == kDetrendMean && on) ? (double)x[0] : 0.0;

    // ---- seeds: Y_m = FFT_N((x[w0 + i] - L) e^{-j m th i}) (seed_ffts), trackers of this thread's bins
    d2 om[B][NF], tr[B][NF];
    double sum = 0.0;
#pragma unroll
    for (int mm = 0; mm <= NM; ++mm) {
        if constexpr (SR) {  // register passes (default): the inputs straight from global memory into registers
            d2 a[N / NT];
#pragma unroll
            for (int r = 0; r < N / NT; ++r) {
                const int i = t + NT * r;
                const double xi = on ? (double)x[i] - lvl : 0.0;
                a[r] = mm == 0 ? d2{xi, 0.0} : xi * mod[(mm - 1) * N + i];
            }
            fft_reg_sub<LOG2N, NT, 4096 / N>(a, buf, twq, t);
        } else {  // mode 5 (ablation): the round-4 form, inputs staged in LDS and radix-4 passes through LDS
            for (int i = t; i < N; i += NT) {
                const double xi = on ? (double)x[i] - lvl : 0.0;
                buf[i] = mm == 0 ? d2{xi, 0.0} : xi * mod[(mm - 1) * N + i];
            }
            __syncthreads();
            fft_lds_sub<LOG2N, NT>(buf, twq, t);
        }
        const double s = mm == 0 ? m->s0 : (mm == 1 ? m->s1 : m->s2);
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int k = kbin_of<NT>(t, b);
            if (mm == 0) {
                tr[b][0] = s * buf[k];
            } else {
                const d2 yp = buf[k], ym = buf[(N - k) & (N - 1)];
                tr[b][2 * mm - 1] = s * yp;
                tr[b][2 * mm] = s * d2{ym.x, -ym.y};
            }
        }
        if (DETREND == kDetrendMean && mm == 0) sum = buf[0].x;  // sum of x - L
        __syncthreads();
    }
    if (trace && threadIdx.x == 0) trace[2] = wall_clock64();  // diagnostic timeline: seeds done
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
        for (int f = 0; f < NF; ++f) om[b][f] = omega[f * M + kbin_of<NT>(t, b)];
    d2 hk[B];
    if constexpr (DETREND == kDetrendMean) {
#pragma unroll
        for (int b = 0; b < B; ++b) hk[b] = hwin[kbin_of<NT>(t, b)];
    }

    // ---- slide (slide_kernel's loop; a sub-workgroup past its segment's end only keeps the barriers)
    SlideArgs ua{};
    ua.s0 = m->s0, ua.s1 = m->s1, ua.s2 = m->s2, ua.c1 = c1, ua.sn1 = sn1, ua.c2 = c2, ua.sn2 = sn2;
    T *__restrict__ out = static_cast<T *>(outp) + w0 * M + 2 * t;
    // write-through form (m->wt, the default): buffer stores with the sc1 policy, so no dirty output lines wait in the
    // XCDs' L2s for the writeback at the end of the launch; the descriptor is based at the segment's first row (uniform
    // per sub-workgroup), the offsets stay within the segment (<= 2048 rows x 2048 bins x 8 B)
    const bool wt = m->wt != 0;
    const __amdgpu_buffer_rsrc_t orc =
        __builtin_amdgcn_make_buffer_rsrc(static_cast<T *>(outp) + w0 * M, (short)0, 0x7fffffff, 0x00020000);
    uint32_t ob = (uint32_t)(2 * t * (int)sizeof(T));
    double *u = reinterpret_cast<double *>(buf);
    for (int c0 = 0; c0 < maxlen; c0 += CH) {
        const int clen = maxlen - c0 < CH ? maxlen - c0 : CH;
        if (c0) __syncthreads();
        stage_uniforms<T, NF, N>(ua, x, lvl, c0, clen < len - c0 ? clen : len - c0, len, u, t, NT);
        __syncthreads();
        const int act = len - c0 < clen ? (len - c0 > 0 ? len - c0 : 0) : clen;  // this sub-workgroup's windows
#pragma unroll 1
        for (int st = 0; st < act; ++st) {
            double mw = 0.0;
            if constexpr (DETREND == kDetrendMean) mw = sum * inv_n;
            double pw[B];
#pragma unroll
            for (int b = 0; b < B; ++b) {
                d2 X = tr[b][0];
#pragma unroll
                for (int f = 1; f < NF; ++f) X += tr[b][f];
                if constexpr (DETREND == kDetrendMean) X -= mw * hk[b];
                pw[b] = X.x * X.x + X.y * X.y;
            }
#pragma unroll
            for (int q = 0; q < B / 2; ++q) {
                typedef T v2t __attribute__((ext_vector_type(2)));
                const v2t pv = v2t{(T)pw[2 * q], (T)pw[2 * q + 1]};
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
    __syncthreads();  // the staged uniforms' reads before the next task's writes
}

template <typename T, int NF, int DETREND, int BS, int SR>
__global__ __launch_bounds__(kMixNT, 4) void slide_mixed_kernel(SlideMix) {
    const MixP m = (MixP)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ d2 lds[4096];
    __shared__ d2 twq[1024];
    const int tid = threadIdx.x;
    const d2 *__restrict__ tw = static_cast<const d2 *>(m->tw4096);
    for (int i = tid; i < 1024; i += kMixNT) twq[i] = tw[i];
    int *ldsi = reinterpret_cast<int *>(lds);
    for (;;) {
        if (tid == 0) ldsi[0] = atomicAdd(m->counter, 1);
        __syncthreads();
        const int task = __builtin_amdgcn_readfirstlane(ldsi[0]);  // uniform: the task's scalars stay in SGPRs
        __syncthreads();
        if (task >= m->n_tasks) break;  // every workgroup leaves on its first failed grab: the grid drains
        int c = 0;
#pragma unroll
        for (int i = 1; i < kMixClass; ++i)
            if (i < m->nclass && task >= m->task0[i]) c = i;
        int t0 = m->task0[0], l2 = m->log2n[0];
#pragma unroll
        for (int i = 1; i < kMixClass; ++i)
            if (c == i) t0 = m->task0[i], l2 = m->log2n[i];
        const int64_t local = task - t0;
        long long *tr = m->trace ? m->trace + 4 * (int64_t)task : nullptr;  // diagnostic timeline, off by default
        if (tr && tid == 0) {
            unsigned xcc = 0;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            tr[0] = (long long)blockIdx.x | ((long long)(xcc & 15) << 32);
            tr[1] = wall_clock64();
        }
        switch (l2) {
        case 12: mix_task<T, 12, NF, DETREND, BS, SR>(m, c, local, lds, twq, tr); break;
        case 11: mix_task<T, 11, NF, DETREND, BS, SR>(m, c, local, lds, twq, tr); break;
        case 10: mix_task<T, 10, NF, DETREND, BS, SR>(m, c, local, lds, twq, tr); break;
        default: mix_task<T, 9, NF, DETREND, BS, SR>(m, c, local, lds, twq, tr); break;
        }
        if (tr && tid == 0) tr[3] = wall_clock64();
    }
    if (tid == 0) {  // the last workgroup out resets this execute's counter slot
        __threadfence();
        if (atomicAdd(m->done, 1) == (int)gridDim.x - 1) {
            atomicExch(m->counter, 0);
            atomicExch(m->done, 0);
        }
    }
}

template <typename T, int NF, int DETREND, int BS> int resident_t(int dev) {
    static std::atomic<int> per_cu{0};
    int pc = per_cu.load(std::memory_order_relaxed);
    if (pc == 0) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, slide_mixed_kernel<T, NF, DETREND, BS, 1>, kMixNT, 0) !=
                hipSuccess ||
            pc <= 0)
            pc = 1;
        per_cu.store(pc, std::memory_order_relaxed);
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    return pc * cus;
}

template <typename T, int BS> int resident_nf(int nf, int detrend, int dev) {
    const bool mean = detrend == kDetrendMean;
    if (nf == 1) return mean ? resident_t<T, 1, kDetrendMean, BS>(dev) : resident_t<T, 1, kDetrendNone, BS>(dev);
    return mean ? resident_t<T, 3, kDetrendMean, BS>(dev) : resident_t<T, 3, kDetrendNone, BS>(dev);
}

template <typename T, int BS, int SR> hipError_t launch_nf(const SlideMix &m, int nf, int detrend, int grid, hipStream_t s) {
    const bool mean = detrend == kDetrendMean;
#define MIX(NF_, D_) hipLaunchKernelGGL((slide_mixed_kernel<T, NF_, D_, BS, SR>), dim3((unsigned)grid), dim3(kMixNT), 0, s, m)
    if (nf == 1) {
        if (mean) MIX(1, kDetrendMean);
        else MIX(1, kDetrendNone);
    } else {
        if (mean) MIX(3, kDetrendMean);
        else MIX(3, kDetrendNone);
    }
#undef MIX
    return hipGetLastError();
}
template <typename T, int BS> hipError_t launch_sr(const SlideMix &m, int nf, int detrend, int grid, hipStream_t s) {
    return m.seed_lds ? launch_nf<T, BS, 0>(m, nf, detrend, grid, s) : launch_nf<T, BS, 1>(m, nf, detrend, grid, s);
}

}  // namespace

int slide_mix_resident(int nf, int detrend, bool f32, int bsmall, int dev) {
    if (bsmall == 2) return f32 ? resident_nf<float, 2>(nf, detrend, dev) : resident_nf<double, 2>(nf, detrend, dev);
    return f32 ? resident_nf<float, 4>(nf, detrend, dev) : resident_nf<double, 4>(nf, detrend, dev);
}

hipError_t launch_slide_mix(const SlideMix &m, int nf, int detrend, bool f32, int grid, hipStream_t s) {
    if ((nf != 1 && nf != 3) || grid < 1 || m.nclass < 1 || m.nclass > kMixClass || m.n_tasks < 1 || !m.counter ||
        !m.done || !m.tw4096 || (m.bsmall != 2 && m.bsmall != 4))
        return hipErrorInvalidValue;
    for (int c = 0; c < m.nclass; ++c)
        if (m.log2n[c] < 9 || m.log2n[c] > 12 || m.seg[c] < 1 || !m.omega[c]) return hipErrorInvalidValue;
    if (m.bsmall == 2) return f32 ? launch_sr<float, 2>(m, nf, detrend, grid, s) : launch_sr<double, 2>(m, nf, detrend, grid, s);
    return f32 ? launch_sr<float, 4>(m, nf, detrend, grid, s) : launch_sr<double, 4>(m, nf, detrend, grid, s);
}

}  // namespace wsp
