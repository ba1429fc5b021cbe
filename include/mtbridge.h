/*
 * mtbridge.h -- C ABI of libmtbridge.so, the MI355X-native drop-in for the
 * `mt-bridge.dll` that WaveSpecZZ binds with `#import "mt-bridge.dll"`
 * (reference Include/imports.mqh:4-20).
 *
 * Type mapping (MQL5 -> C):
 *   int -> int32_t, long -> int64_t (NOT C long), double&[] -> double*,
 *   int& -> int32_t*, long& -> int64_t*, ushort&[] -> uint16_t* (UTF-16).
 * Arrays are passed as raw pointers with explicit sizes.  All buffers are
 * caller-owned; the library never keeps a caller pointer past return.
 * Every entry point is thread-safe (MT5 runs different charts on different
 * threads of one process).
 *
 * Status codes follow L/WaveSpecZZ_gpu_wip.mq5:263-269 and
 * WaveCyclesBatchFetcher.mq5:14-22.
 */
#ifndef MTBRIDGE_H
#define MTBRIDGE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTB_API __attribute__((visibility("default")))

/* ---- status codes (ALGLIB_STATUS_*) ---------------------------------- */
#define MTB_OK 0
#define MTB_BAD_ARGS (-1)
#define MTB_BACKEND_UNAVAILABLE (-2)
#define MTB_TIMEOUT (-3)
#define MTB_INTERNAL_ERROR (-4)
#define MTB_NOT_READY (-5)
#define MTB_NO_MEM (-6)

/* ---- enums of the spectrum batch API -------------------------------- */
/* detrend: none (1.1.0:1239), mean (L/WaveSpecZZ_gpu_wip.mq5:940-950),
 * IIR trend (L/WaveSpecZZ_1.0.2.mq5:3040-3053), per-window Kalman 4D
 * (L/WaveSpecZZ_1.0.3-pla-kalman-fast.mq5:2015-2125, reset per window). */
#define MTB_DETREND_NONE 0
#define MTB_DETREND_MEAN 1
#define MTB_DETREND_IIR 2
#define MTB_DETREND_KALMAN 3
/* window: enum WINDOW_TYPE, L/WaveSpecZZ_1.0.2.mq5:626-632 */
#define MTB_WINDOW_NONE 0
#define MTB_WINDOW_HANN 1
#define MTB_WINDOW_HAMMING 2
#define MTB_WINDOW_BLACKMAN 3
#define MTB_WINDOW_BARTLETT 4
/* arithmetic precision of the device path */
#define MTB_PREC_F64 0
#define MTB_PREC_F32 1
/* output: |X_k|^2 for k < N/2 (FftProcessor::Run 1.1.0:529-530), or the
 * packed gpu_fft_real_forward layout out[2k]=Re X_k, out[2k+1]=Im X_k
 * (1.1.0:522-528). */
#define MTB_OUT_POWER 0
#define MTB_OUT_PACKED 1
/* top-k bin scan records (L/WaveSpecZZ_1.0.3-pla-kalman-fast-gpuopt-nodetrend.mq5:536-554):
 * top_k slots of [bin, power, Re X_bin, Im X_bin], power-descending (ties: lower bin first),
 * bins in [ceil(N/max_period), floor(N/min_period)] clamped to N/2-1, empty slots
 * [-1, -1, 0, 0]. */
#define MTB_OUT_TOPK 2
/* phase outputs (fp64 only), CalculateFFTPhase / UnwrapPhase /
 * CalculateGroupDelay of L/WaveSpecZZ_1.0.4-new.mq5:1040-1120 run at :3225-3227
 * over n = N entries (X_k for k < N/2, zero above: the GPU unpack :3183-3196):
 *   MTB_OUT_PHASE      record of 3*(N/2) doubles [P_k | unwrapped phase_k |
 *                      group delay_k (clamped to +-100)], k < N/2;
 *   MTB_OUT_TOPK_PHASE top_k slots of [bin, power, Re, Im, unwrapped phase,
 *                      group delay] (the values the ETA estimators read at the
 *                      dominant bin, :1165 and :1239); empty [-1, -1, 0, 0, 0, 0]. */
#define MTB_OUT_PHASE 3
#define MTB_OUT_TOPK_PHASE 4

/* =====================================================================
 * 1. Reference surface -- Include/imports.mqh:5-19 (exact signatures)
 * ===================================================================== */

/* imports.mqh:5.  Opens (first call) or joins the process-wide session on
 * `device_index` (0-based HIP device; -1 = every visible GPU, windows of
 * batch calls are sharded across them).  `stream_count` HIP streams per
 * device (caller clamps 16..512, 1.1.0:729).  Every successful call adds one
 * reference to the session and one to the calling thread's count (MT5 runs
 * each chart on its own thread and each chart calls gpu_init once, EnsureGpu
 * 1.1.0:722-751; a chart retries it every bar until it succeeds).  Returns
 * MTB_OK, MTB_BACKEND_UNAVAILABLE (no usable device), or MTB_BAD_ARGS when a
 * session is already open on a different device (it is not replaced). */
MTB_API int32_t gpu_init(int32_t device_index, int32_t stream_count);

/* imports.mqh:6 (OnDeinit 1.1.0:706-716).  Drops one reference taken by
 * gpu_init.  When the calling thread's own count reaches zero, the jobs that
 * thread submitted are released (other charts' jobs are untouched); when the
 * session's count reaches zero, every remaining job is released and the
 * streams, pooled buffers and host registrations are freed once calls still
 * in flight on other threads have returned.  Without an open session it is a
 * no-op. */
MTB_API void gpu_shutdown(void);

/* imports.mqh:7; caller FftProcessor::Run 1.1.0:518-531.  Real forward DFT
 * (unnormalised, e^{-2 pi i k n/N}) of in[0..len) into out[0..len):
 * out[2k] = Re X_k, out[2k+1] = Im X_k for k < len/2.  len: power of two,
 * 32..262144 (the legacy InpFFTWindow menu, L/WaveSpecZZ_1.0.4-new.mq5:657).
 * Synchronous. */
MTB_API int32_t gpu_fft_real_forward(const double *in, int32_t len, double *out);

/* imports.mqh:8-19: MUSIC/ESPRIT cycle extraction lives outside the
 * spectrum hot path.  These return
 * MTB_BACKEND_UNAVAILABLE and set the last error. */
MTB_API int32_t gpu_extract_cycles(const double *series, int32_t len, int32_t top_k, double min_period,
                                   double max_period, double sample_rate_seconds, int32_t method,
                                   int32_t ar_order, double *out, int32_t out_stride, int32_t out_capacity,
                                   int32_t *out_len);
MTB_API int32_t gpu_submit_extract_cycles(const double *series, int32_t len, int32_t top_k, double min_period,
                                          double max_period, double sample_rate_seconds, int32_t method,
                                          int32_t ar_order, int64_t *job_id);
MTB_API int32_t gpu_try_get_cycles(int64_t job_id, double *out, int32_t out_stride, int32_t out_capacity,
                                   int32_t *out_len, int32_t *ready);
MTB_API int32_t gpu_submit_extract_cycles_batch(const double *series, int32_t series_len, int32_t window_len,
                                                int32_t hop, int32_t top_k, double min_period, double max_period,
                                                double sample_rate_seconds, int32_t method, int32_t ar_order,
                                                int32_t stride, int64_t *job_id);
MTB_API int32_t gpu_try_get_cycles_batch(int64_t job_id, double *out, int32_t out_cap, int32_t *out_len,
                                         int32_t *ready);

/* imports.mqh:18.  Releases a job of any kind (callers always free after a
 * result or an error: 1.1.0:1040, 1277). Unknown id -> MTB_BAD_ARGS. */
MTB_API int32_t gpu_free_job(int64_t job_id);

/* imports.mqh:19.  Copies the calling thread's last error as UTF-16 into
 * buf (at most buf_len units, NUL-terminated) and returns the number of
 * units written INCLUDING the terminator (caller: ShortArrayToString(buf,
 * 0, n-1), 1.1.0:742-744).  0 when there is no error text. */
MTB_API int32_t gpu_get_last_error_w(uint16_t *buf, int32_t buf_len);

/* =====================================================================
 * 2. Batch FFT declared by the legacy indicators
 *    (L/WaveSpecZZ_1.0.3-pla-batch.mq5:29, L/WaveSpecZZ_gpu_cycles.mq5:14)
 * ===================================================================== */

/* n_windows pre-materialised windows in[w*window_len + j] -> packed spectra
 * out[w*window_len + 2k (+1)], same per-window layout as
 * gpu_fft_real_forward. */
MTB_API int32_t gpu_fft_real_forward_batch(const double *in, int32_t window_len, int32_t n_windows, double *out);

/* Inverse of gpu_fft_real_forward (declared L/WaveSpecZZ_1.0.4-core.mq5:65;
 * called at :426 on the forward output of :344 after the spectral stages, the
 * result goes back into the time-domain pipeline at :432).  The DLL's own
 * numerics are unpinned (no CPU counterpart in the reference); defined here
 * as the exact inverse of the packed layout: in[2k] + i in[2k+1] = X_k for
 * 0 < k < len/2, X_0 = in[0] (in[1], Im X_0 of a real signal, is ignored),
 * X_{len/2} = 0 (no slot in the layout), out[n] = (1/len) sum_k X_k
 * e^{+2 pi i k n/len}.  inverse(forward(x)) == x for x without a Nyquist
 * component.  len: power of two, 32..16384.  Synchronous. */
MTB_API int32_t gpu_fft_real_inverse(const double *in_spec, int32_t len, double *out);

/* Batch form: n_windows packed spectra in[w*window_len ...] -> samples. */
MTB_API int32_t gpu_fft_real_inverse_batch(const double *in, int32_t window_len, int32_t n_windows, double *out);

/* L/WaveSpecZZ_1.0.4-core.mq5:72 (called at :416 on the packed forward
 * output).  spectrum: spectrum_len doubles = spectrum_len/2 packed bins (any
 * even length >= 2); bins from spectrum_len/2 up are the zeroed upper half of
 * the reference's arrays.  method 0: unwrapped phase, 1: wrapped phase
 * atan2(Im, Re), 2: group delay (clamped +-100); out[k] for k <
 * spectrum_len/2 (out_len >= spectrum_len/2).  Method numbering is
 * build-defined (the DLL is unpinned).  Synchronous. */
MTB_API int32_t gpu_spectral_phase_unwrap(const double *spectrum, int32_t spectrum_len, int32_t method, double *out,
                                          int32_t out_len);

/* =====================================================================
 * 3. Hot path: batched sliding-window power spectrum over a series
 *    (shape of gpu_submit_extract_cycles_batch, imports.mqh:14-16;
 *    nwin = 1 + (series_len - window_len)/hop as at 1.1.0:1016)
 * ===================================================================== */

/* Window w covers series[w*hop .. w*hop+window_len) of a CHRONOLOGICAL
 * series (physical memory of an MQL as-series array).  Per window:
 * detrend -> window -> real FFT -> output.  `out` receives nwin records of
 * window_len/2 doubles (MTB_OUT_POWER) or window_len doubles
 * (MTB_OUT_PACKED); only min(nwin, out_cap/record) records are written and
 * *out_len = records written.  trend_period: InpTrendPeriod (int > 0) for
 * MTB_DETREND_IIR.  precision: MTB_PREC_F64 or MTB_PREC_F32 (the f32 device
 * path converts the series to float on the host and results back).
 * window_len: power of two, 32..262144; above 16384 the outputs are
 * MTB_OUT_POWER and MTB_OUT_PACKED (four-step transform).  Synchronous. */
MTB_API int32_t gpu_spectrum_batch(const double *series, int32_t series_len, int32_t window_len, int32_t hop,
                                   int32_t detrend, int32_t window, int32_t trend_period, int32_t precision,
                                   int32_t output, double *out, int32_t out_cap, int32_t *out_len);

/* Asynchronous form.  Copies `series` before returning (1.1.0:1316 reuses
 * its buffer right after submit).  *job_id = 0 on failure. */
MTB_API int32_t gpu_submit_spectrum_batch(const double *series, int32_t series_len, int32_t window_len,
                                          int32_t hop, int32_t detrend, int32_t window, int32_t trend_period,
                                          int32_t precision, int32_t output, int64_t *job_id);

/* Poll: MTB_OK + *ready=0 while pending; MTB_OK + *ready=1 when the records
 * are copied to out.  The pending status is the one WaveCyclesBatchFetcher's
 * unchanged loop needs (WaveCyclesBatchFetcher.mq5:127-131 sleeps only on
 * OK && ready == 0 and re-polls at once on any other status, so a NOT_READY
 * convention would spend its 4000 tries in microseconds); the indicator's
 * warm-up loop (1.1.0:1029-1039) accepts it as well.  Any other status is an
 * error (unknown job, device error, out_cap below one record).  The caller
 * frees the job.  (The reference's single-job cycles poll, 1.1.0:1274, uses
 * NOT_READY; the cycle functions are out of scope here and return
 * MTB_BACKEND_UNAVAILABLE.) */
MTB_API int32_t gpu_try_get_spectrum_batch(int64_t job_id, double *out, int32_t out_cap, int32_t *out_len,
                                           int32_t *ready);

/* The spectrum's immediate consumer fused into the same launch: only
 * 4*top_k doubles per window leave the device instead of N/2 (MTB_OUT_TOPK
 * record layout).  top_k in 1..64 (the reference uses 8); periods in bars. */
MTB_API int32_t gpu_spectrum_topk_batch(const double *series, int32_t series_len, int32_t window_len, int32_t hop,
                                        int32_t detrend, int32_t window, int32_t trend_period, int32_t precision,
                                        int32_t top_k, double min_period, double max_period, double *out,
                                        int32_t out_cap, int32_t *out_len);

/* gpu_spectrum_topk_batch with MTB_OUT_TOPK_PHASE records (6*top_k doubles
 * per window: bin, power, Re, Im, unwrapped phase, group delay).  fp64. */
MTB_API int32_t gpu_spectrum_topk_phase_batch(const double *series, int32_t series_len, int32_t window_len,
                                              int32_t hop, int32_t detrend, int32_t window, int32_t trend_period,
                                              int32_t top_k, double min_period, double max_period, double *out,
                                              int32_t out_cap, int32_t *out_len);

/* Kalman 4D parameters for MTB_DETREND_KALMAN, in the order of the inputs
 * at L/WaveSpecZZ_1.0.3-pla-kalman-fast.mq5:886-901: follow_strength,
 * q_pos, q_vel, q_acc, q_jerk, adapt_gain, meas_noise, init_var_pos,
 * init_var_vel, init_var_acc, init_var_jerk, init_vel, init_acc, init_jerk,
 * clip_std, ema_blend_period.  n must be 16.  Process-wide. */
MTB_API int32_t gpu_set_kalman_params(const double *params, int32_t n);

/* Pinned feed staging (north star: "FeedCache.mqh rewired to stage price bars
 * into pinned host buffers for hipMemcpyAsync"; replaces the plain-host-memory
 * use of the FeedCache close history, Include/FeedCache.mqh:36-115,
 * `struct FeedCache`).  Every batch call stages the caller's series through
 * the library's own pinned (hipHostMalloc) buffers, chunk by chunk, while
 * earlier chunks' H2D copies and kernels run; a synchronous call's records come
 * back through a ring of four pinned slots that the host drains into the
 * caller's array while the next chunks are copied off the device (so an
 * output-dominated call overlaps its host copy-out with PCIe).
 *
 * gpu_register_host records [ptr, ptr + count) with the session: it refuses
 * ranges overlapping another registration, and registrations end with the
 * session (last gpu_shutdown).  It does NOT page-lock the caller's memory
 * (round 6): hipHostRegister of caller arrays was withdrawn because, after a
 * locked array was unregistered and freed, a later pageable copy into memory
 * reused from its pages could fault inside the HIP runtime.
 * No call of this library page-locks, maps or DMAs caller memory, so freeing,
 * moving (ArrayResize) or unregistering a buffer has no device-side hazard; a
 * buffer must still not be freed while a call reading it runs.
 * MTB_OK; MTB_BAD_ARGS for null/empty ranges, ranges overlapping another
 * registration (register) or an unknown base pointer (unregister);
 * MTB_BACKEND_UNAVAILABLE without a session. */
MTB_API int32_t gpu_register_host(const double *ptr, int64_t count);
MTB_API int32_t gpu_unregister_host(const double *ptr);
/* Round 5 made page-locking of registered caller memory opt-in (mode 1);
 * round 6 withdrew it.  Mode 0 (record the range, stage through
 * the library's pinned buffers) is the only mode: 0 returns 0, 1 returns
 * MTB_BAD_ARGS with a last-error text saying so, any other mode MTB_BAD_ARGS. */
MTB_API int32_t gpu_set_host_locking(int32_t mode);
/* The current session's identity: a number > 0 that changes whenever the
 * session is torn down (last gpu_shutdown) and a new one opened; 0 without a
 * session.  Registrations belong to one session: a caller that registered a
 * buffer under session id s and finds another id has nothing to unregister. */
MTB_API int64_t gpu_session_id(void);

/* =====================================================================
 * 4. Device-resident plans: the same hot path on buffers already in HBM
 *    (multi-GPU shards, benchmarks, pipelines that keep data on device).
 * ===================================================================== */

/* Creates a plan on HIP device `device`.  Returns a handle > 0, or 0 on
 * error (see gpu_get_last_error_w).  n_windows windows of window_len
 * samples, window w at offset w*hop (elements) of the series. */
MTB_API int64_t wsp_plan_create(int32_t device, int32_t window_len, int64_t hop, int64_t n_windows,
                                int32_t detrend, int32_t window, int32_t trend_period, int32_t precision,
                                int32_t output);

/* Device-resident inverse plan (gpu_fft_real_inverse_batch on HBM buffers):
 * wsp_plan_execute reads n_windows packed spectra of window_len doubles and
 * writes n_windows rows of window_len samples. */
MTB_API int64_t wsp_plan_create_inverse(int32_t device, int32_t window_len, int64_t n_windows);

/* Enqueues the hot path on `hip_stream` (a hipStream_t; NULL = the null
 * stream) reading d_series (device pointer, double or float per the plan's
 * precision, >= (n_windows-1)*hop + window_len elements) and writing d_out
 * (n_windows * record elements).  Asynchronous; no allocation, no host
 * sync.  A plan with a device workspace (Kalman detrend, IIR above 16384,
 * window_len above 16384, hop = 1 top-k by the sliding DFT) orders its own
 * executes: one issued on a different stream than the previous execute waits
 * for it on the device (hipStreamWaitEvent), so such a plan may be executed
 * from several streams and threads but its executes never overlap; plans
 * without a workspace run concurrently on any number of streams.  A
 * workspace replaced by a reconfiguration is freed by the next configuration
 * call (create / set / destroy / gpu_shutdown), never inside an execute. */
MTB_API int32_t wsp_plan_execute(int64_t plan, const void *d_series, void *d_out, void *hip_stream);

/* Sets a top-k plan's scan: MTB_OUT_TOPK (4*top_k elements per window; a
 * power/packed plan switches to it) or MTB_OUT_TOPK_PHASE (6*top_k). */
MTB_API int32_t wsp_plan_set_topk(int64_t plan, int32_t top_k, double min_period, double max_period);

/* Algorithm for hop = 1 batches (an extension; the reference always runs an
 * FFT per window).  MTB_ALGO_AUTO (default): the seeded sliding DFT when the
 * plan is eligible -- hop = 1, window_len 512..8192, detrend none or mean,
 * Hann / Hamming / Blackman / no window, MTB_OUT_POWER or fp64 MTB_OUT_TOPK over
 * at most 512 bins -- and has at least 256
 * windows, otherwise the per-window FFT.  MTB_ALGO_FFT / MTB_ALGO_SLIDE force
 * one (MTB_BAD_ARGS if the plan is not eligible for the slide).  Both produce
 * the same spectra within the parity bars. */
#define MTB_ALGO_AUTO 0
#define MTB_ALGO_FFT 1
#define MTB_ALGO_SLIDE 2
MTB_API int32_t wsp_plan_set_algorithm(int64_t plan, int32_t algo);
/* Tuning: windows per sliding-DFT workgroup (each seeds its trackers once);
 * 0 = the library's policy (32..256).  A tracker's rounding grows with the
 * number of slides, so at most 2048 (the longest length the parity tests
 * cover); MTB_BAD_ARGS for an unknown plan or windows outside 0..2048. */
MTB_API int32_t wsp_plan_set_slide_segment(int64_t plan, int64_t windows);
/* Tuning (hop = 1 top-k records, N >= 1024): segments per seed workgroup.  The
 * first segment of a chain is seeded by the FFTs, each next one by sliding the
 * band's trackers on from the previous (the scan's own slide operations: the
 * records agree with FFT seeds within the parity bars); 1 = one FFT seed per
 * segment, 0 = the library's policy (chains of ~128 windows when the batch is
 * too small for 64-window segments to fill the GPU -- a strong-scaled shard --
 * and its segments drop to 32 windows, else 1).  Capped at 1 + 256 / segment
 * (a chain's steps are staged in LDS).
 * MTB_BAD_ARGS for an unknown plan or segments outside 0..16. */
MTB_API int32_t wsp_plan_set_seed_chain(int64_t plan, int32_t segments);
/* Diagnostic: a timeline of the hop = 1 sliding-DFT kernels of later executes into
 * d_trace, a device buffer of `capacity` int64 (wall-clock ticks, 100 MHz):
 * seed workgroup b writes [b | XCC << 32, start, FFT m = 0 done, seeds done,
 * chain done, end] at 6 b and scan workgroup b [start, end] at capacity / 2 +
 * 2 b, each while it fits; hop = 1 power slides (round 6): workgroup b writes
 * [b | XCC << 32, start, seeds done, end] at 4 b; the fused large-N kernel
 * (round 6: fp64 power with a Hann window, the N = 65536 default form) has
 * workgroup b write, for its first window, 4 ticks per column / row block
 * (start, loads done, FFT done, block done) at 32 b.  capacity = 0 turns it off
 * (the default).  MTB_BAD_ARGS for an unknown plan or a null buffer. */
MTB_API int32_t wsp_plan_set_trace(int64_t plan, void *d_trace, int64_t capacity);
/* Tuning / ablation: the kernel form, 0..8 (MTB_BAD_ARGS outside); 0 = the
 * library's choice (default).  Same records within the parity bars either way.
 *  - hop = 1 power rows by the sliding DFT: 7 = plain stores (the default
 *    writes the rows through to memory, agent-scope sc1 stores);
 *  - hop = 1 top-k records by the sliding DFT: 1 = one wave-wide reduction
 *    round per slot and window; 2 / 3 = the transposed lane-per-window scan
 *    (k <= 8, bands <= 256 bins) staging 16 / 8 windows per batch; 0 = the
 *    probe-threshold scan (16 windows per batch, 4 waves per SIMD), 4 / 5 = the
 *    same at 32 windows x 16 candidates / 32 x 12 (more LDS per wave); 6 =
 *    the default scan with seed chains of <= 256 windows at any segment
 *    length (one FFT seed per chain, the next segments' seeds by sliding the
 *    band on; slower on whole batches, round 5); 7 = plain stores of the seed
 *    records, 8 = non-temporal ones (the default writes them through to
 *    memory, agent scope);
 *  - N = 32768 .. 262144 (four-step transform): 1 = two passes over chunks of
 *    windows; 2 = the same pipelined over two internal streams (a one-window
 *    chunk runs the plain loop: its workspace holds one buffer); 3 = the fused
 *    one-workgroup-per-window kernel (N = 65536 / 131072; the default for fp64
 *    N = 65536); 4 = its 256-thread form with register prefetch; 5 = the fused
 *    kernel with plain (not non-temporal) output stores; 6 = fp64 N = 262144
 *    with 16-column column-pass workgroups (the default takes 8); 7 = the
 *    two-pass row kernel in plain block order (the default is XCD-aware);
 *    8 = two passes with 8-column column-pass workgroups at M2 = 256 (fp64
 *    N = 65536 / 131072);
 *  - fp32 Kalman pre-pass (spectrum plans, N <= 16384): 1 = single-wave
 *    workgroups of the one-lane filter, 2 = the sequential one-lane filter,
 *    7 = the packed two-segment filter in the original basis with its rows
 *    written through to memory (bit-identical to 8); 8 = the packed two-segment
 *    filter in the original basis with the reference's diagonal floors (the
 *    round-5 default; 0 steps in the Newton basis, see kalman_core.h); 9 = the
 *    default filter with the window applied by the spectrum kernel (0 has
 *    the two-segment filter multiply it into its rows at N <= 4096);
 *  - inverse plans (wsp_plan_create_inverse, N = 2048 .. 8192): 1 = the
 *    C2R pre-step through LDS (round-1 form), 2 = the pre-step in registers
 *    with the AoS exchange; 3 = 0 with the element loads in natural order
 *    (round 4); 4 = 0 with plain (not non-temporal) sample stores; 0 = the
 *    pre-step in registers, split exchange, each element's two reads (as X_k
 *    and as a mirror X_(M-k)) one load step apart;
 *  - MTB_OUT_PHASE records at N = 2048 / 4096 without IIR detrend: 2 = the
 *    split-exchange form (3 waves per SIMD; slower than the default AoS form);
 *  - MTB_OUT_TOPK_PHASE records (FFT kernel): 1 = the AoS form (two waves per
 *    SIMD, every thread's phase chunk) instead of the split-exchange one-wave
 *    scan + one-wave winners' phases. */
MTB_API int32_t wsp_plan_set_variant(int64_t plan, int32_t variant);
/* Diagnostics: d_flags (device, n_windows bytes, or NULL = off) receives, on
 * every execute of a hop = 1 top-k plan by the probe-threshold scan (variant
 * 0 / 4 / 5), the path each window took: 0 = the candidate list, 1 = the exact
 * one-wave scan at a segment's first window, 2 = the exact scan because more
 * candidates passed the threshold than the list holds.  Other plans leave it
 * untouched.  The records are the same either way. */
MTB_API int32_t wsp_plan_set_scan_flags(int64_t plan, void *d_flags);
/* Tuning: windows per chunk of the two-pass large-N path (N > 16384: column
 * results of one chunk of windows are written and read back per launch pair),
 * 0 = the library's ~192 MiB of column results; grows the plan workspace as
 * needed.  MTB_BAD_ARGS for an unknown plan or windows outside 0..2^20. */
MTB_API int32_t wsp_plan_set_chunk(int64_t plan, int64_t windows);
/* Tuning: workgroups of the per-window FFT kernel's launch (grid-stride over
 * window groups) and of the inverse plans' launch; 0 = the library's choice
 * (32768).  Applies to the FFT-kernel and inverse paths only (the sliding DFT,
 * Kalman pre-pass and large-N kernels size their own grids).  MTB_BAD_ARGS for
 * an unknown plan or workgroups outside 0..65536. */
MTB_API int32_t wsp_plan_set_grid(int64_t plan, int32_t workgroups);
/* MTB_ALGO_FFT or MTB_ALGO_SLIDE: what the next execute runs. */
MTB_API int32_t wsp_plan_get_algorithm(int64_t plan);

/* Bytes the plan's algorithm must move per execute: unique input samples
 * + output, for roofline accounting. */
MTB_API int64_t wsp_plan_algorithmic_bytes(int64_t plan);

/* Grouped hop = 1 plan: a multi-symbol batch in the WaveCyclesBatchFetcher
 * shape (one series per symbol, WaveCyclesBatchFetcher.mq5:112-118; C5 = 28
 * symbols x 4 window lengths) on device-resident buffers.  Member m: a series
 * of n_windows[m] + window_len[m] - 1 samples, every window of it (hop = 1),
 * MTB_OUT_POWER rows of window_len[m]/2 elements.  All members run in one
 * persistent sliding-DFT launch (wsp_group_set_mode), or the members of each
 * window length in one launch (longest windows first, up to 16 members per
 * launch), segmented over the length's total window count.
 * Members must be sliding-DFT batches: window_len 512..8192, detrend none or
 * mean, Hann / Hamming / Blackman / no window (Blackman up to 4096).  Returns
 * a handle > 0, or 0 (see gpu_get_last_error_w). */
MTB_API int64_t wsp_group_create(int32_t device, int32_t n_members, const int32_t *window_len,
                                 const int64_t *n_windows, int32_t detrend, int32_t window, int32_t precision);
/* Enqueues every member: d_series[m] / d_out[m] are device pointers (double
 * or float per the precision).  Asynchronous, no host sync.  The launches
 * start on `hip_stream` and, with more than one lane (wsp_group_set_streams),
 * fork onto the group's internal streams and join back into `hip_stream`
 * (events): work enqueued on `hip_stream` after the execute sees every
 * member's output.  The internal streams belong to the group and every execute
 * uses them, so executes of one group issued on different caller streams run
 * one after another, not concurrently (use one group per concurrent caller).
 * The mixed-length launch (the default mode) uses no internal streams and
 * ignores wsp_group_set_streams: it runs on `hip_stream` alone, so executes of
 * one group on different caller streams DO run concurrently -- each takes one
 * of 256 device task-counter slots in turn, and an execute whose slot's
 * previous user ran on another stream waits for it (an event) before reusing
 * the slot, so any number may be in flight. */
MTB_API int32_t wsp_group_execute(int64_t group, const void *const *d_series, void *const *d_out, void *hip_stream);
/* Algorithmic bytes of one execute (sum over members, as wsp_plan_algorithmic_bytes). */
MTB_API int64_t wsp_group_algorithmic_bytes(int64_t group);
/* Kernel launches one execute makes: 1 for the mixed-length launch, else one
 * per window length and 16 members. */
MTB_API int32_t wsp_group_launches(int64_t group);
/* Tuning: n_streams > 1 runs every execute's launches side by side on n
 * lanes -- the caller's stream and n - 1 internal streams forked from it and
 * joined back (events; no host sync) -- assigned greedily by output bytes,
 * each lane's launches sized for its share of the device's workgroup slots,
 * so one window length's seed phase and last workgroups overlap the others'.
 * Default (set by wsp_group_create): one lane per launch, at most 4 (the HIP
 * hardware queues of a process); 1 = everything on the caller's stream.
 * MTB_BAD_ARGS outside 1..8. */
MTB_API int32_t wsp_group_set_streams(int64_t group, int32_t n_streams);
/* Tuning: windows per sliding-DFT workgroup (0 = the launcher's policy over
 * each window length's total window count), at most 2048. */
MTB_API int32_t wsp_group_set_segment(int64_t group, int64_t windows);
/* Tuning / ablation: 0 (default) = the library's choice -- ONE persistent
 * launch over every member when all window lengths are 512..4096, the window
 * has at most three cosine terms (none / Hann / Hamming) and there are at
 * most 32 members (workgroups pull segments of all lengths from a device
 * counter, longest windows first); otherwise one launch per window length.
 * 1 = one launch per window length (lanes: wsp_group_set_streams); 2 = the
 * mixed launch with four bins per thread for N <= 1024 (ablation; the
 * default takes two there); 3 = the mixed launch with half-length segments
 * for the shortest window length, which drains the launch, at every batch
 * size (the default does so only when the batch is large enough that the
 * segment policy is above its floor of 128 windows); 4 = the mixed launch
 * with one segment length for every window length (ablation); 5 = the mixed
 * launch with the round-4 seed FFTs through LDS (ablation); 6 = the mixed
 * launch with plain output stores (the mixed launch writes its output rows
 * through to memory: agent-scope sc1 stores).  MTB_BAD_ARGS outside 0..6. */
MTB_API int32_t wsp_group_set_mode(int64_t group, int32_t mode);
/* Diagnostic: a per-task timeline of the mixed-length launch.  d_trace = a
 * device buffer of 4 x capacity_tasks int64: task t of each later execute
 * writes [workgroup | XCC << 32, start, seeds done, end] (wall-clock ticks,
 * 100 MHz) at 4 t when the execute has at most capacity_tasks tasks.
 * capacity_tasks = 0 turns it off (the default).  MTB_BAD_ARGS for an unknown
 * group or a null buffer. */
MTB_API int32_t wsp_group_set_trace(int64_t group, void *d_trace, int64_t capacity_tasks);
/* Tasks of the group's last mixed-length execute (0 before the first, -1 for
 * an unknown group). */
MTB_API int64_t wsp_group_last_tasks(int64_t group);
MTB_API int32_t wsp_group_destroy(int64_t group);

MTB_API int32_t wsp_plan_destroy(int64_t plan);

/* Version string "mtbridge-mi355x <semver> gfx950" (static storage). */
MTB_API const char *wsp_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MTBRIDGE_H */
