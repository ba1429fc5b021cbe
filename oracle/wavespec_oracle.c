/*
 * wavespec_oracle.c -- CPU restatement of WaveSpecZZ's spectrum hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker / the reported CPU baseline.  The product path (libmtbridge.so)
 * never links, loads or calls it.
 *
 * PARITY STATUS: "parity unpinned" with respect to the reference binary.
 *   The reference is MQL5 (needs MetaEditor, Windows-only) and its GPU
 *   arithmetic lives in the un-vendored mt-bridge.dll; it ships no tests,
 *   golden vectors or fixtures.  This file is a
 *   line-by-line restatement of the reference's own MQL5 CPU code, checked
 *   in tests/ against analytic known-answer tests (impulse, DC, cosine,
 *   Parseval) and against numpy.fft as an independent implementation.
 *
 * Every function cites the reference file:line it restates (paths relative
 * to the reference root; "1.1.0" = WaveSpecZZ_1.1.0-gpuopt.mq5,
 * "L/" = Legacy/).  MQL5 `double` = IEEE binary64, `int` = int32,
 * `long` = int64; MQL `cos/sin/MathSqrt` = libm.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

#ifdef _OPENMP
#include <omp.h>
#endif

#define ORA_EXPORT __attribute__((visibility("default")))

/* Thread count for ora_batch_spectrum (the CPU baseline reports it). */
ORA_EXPORT int ora_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

/* Detrend modes (builder-defined numbering, shared with include/mtbridge.h). */
enum { ORA_DETREND_NONE = 0, ORA_DETREND_MEAN = 1, ORA_DETREND_IIR = 2, ORA_DETREND_KALMAN = 3 };
/* enum WINDOW_TYPE, L/WaveSpecZZ_1.0.2.mq5:626-632 (used by ApplyWindow :925-935). */
enum { ORA_WIN_NONE = 0, ORA_WIN_HANN = 1, ORA_WIN_HAMMING = 2, ORA_WIN_BLACKMAN = 3, ORA_WIN_BARTLETT = 4 };

/* ------------------------------------------------------------------ gather */

/* BuildPlaPriceSeries / FeedBuilder::Build (1.1.0:765-769, 1.1.0:492-496):
 *   feed_data[j] = g_feed_cache.close[shift_end_feed + (N-1-j)]
 * `close_series` is newest-first (ArraySetAsSeries(cache.close,true),
 * Include/FeedCache.mqh:60,117), so the window comes out chronological. */
ORA_EXPORT void ora_gather_series(const double *close_series, int64_t shift_end_feed, int n,
                                  double *feed_data) {
    for (int j = 0; j < n; j++) feed_data[j] = close_series[shift_end_feed + (n - 1 - j)];
}

/* ----------------------------------------------------------------- detrend */

/* Mean removal, L/WaveSpecZZ_gpu_wip.mq5:940-950 (ApplyWindowTransform):
 * sequential sum, divide by window_len, subtract. */
ORA_EXPORT void ora_detrend_mean(const double *x, int n, double *d) {
    double mean = 0.0;
    for (int i = 0; i < n; ++i) mean += x[i];
    mean /= (double)n;
    for (int i = 0; i < n; ++i) d[i] = x[i] - mean;
}

/* IIR trend pre-filter, L/WaveSpecZZ_1.0.2.mq5:3040-3053 (guard
 * L/WaveSpecZZ_1.0.3-pla-batch.mq5:3256): restarts at every window.
 *   omega = 2*pi/P; alpha = (1-sin(omega))/cos(omega); c = (1-alpha)/2
 *   t0 = c*(x0+x0); tj = c*(xj + x(j-1)) + alpha*t(j-1); d = x - t        */
ORA_EXPORT void ora_iir_coeffs(int trend_period, double *alpha_out, double *c_out) {
    double omega = 2.0 * M_PI / trend_period;
    double alpha = (1.0 - sin(omega)) / cos(omega);
    double c = (1.0 - alpha) / 2.0;
    *alpha_out = alpha;
    *c_out = c;
}

ORA_EXPORT void ora_detrend_iir(const double *x, int n, int trend_period, double *d) {
    if (trend_period <= 0) { /* 1.0.3-pla-batch:3279-3281: filter skipped */
        memcpy(d, x, sizeof(double) * (size_t)n);
        return;
    }
    double alpha, c;
    ora_iir_coeffs(trend_period, &alpha, &c);
    double *t = (double *)malloc(sizeof(double) * (size_t)n);
    t[0] = c * (x[0] + x[0]);
    if (n > 1) t[1] = c * (x[1] + x[0]) + alpha * t[0];
    for (int j = 2; j < n; j++) t[j] = c * (x[j] + x[j - 1]) + alpha * t[j - 1];
    for (int j = 0; j < n; j++) d[j] = x[j] - t[j];
    free(t);
}

/* Kalman 4D (pos/vel/acc/jerk), L/WaveSpecZZ_1.0.3-pla-kalman-fast.mq5.
 * Parameters in the order of the inputs at :886-901. */
typedef struct {
    double follow_strength, q_pos, q_vel, q_acc, q_jerk, adapt_gain, meas_noise;
    double init_var_pos, init_var_vel, init_var_acc, init_var_jerk;
    double init_vel, init_acc, init_jerk, clip_std, ema_blend_period;
} ora_kalman_params;

/* Defaults of :886-901. */
ORA_EXPORT void ora_kalman_default_params(double *p16) {
    const double def[16] = {1.0, 0.01, 0.003, 0.0008, 0.0002, 0.8, 1.0, 16.0,
                            9.0, 4.0, 1.0, 0.0, 0.0, 0.0, 6.0, 0.0};
    memcpy(p16, def, sizeof(def));
}

typedef struct {
    double pos, vel, acc, jerk;
    double P[4][4];
    int ema_ready;
    double ema_prev;
} ora_kalman_state;

static double dmax(double a, double b) { return a > b ? a : b; }
static double dmin(double a, double b) { return a < b ? a : b; }

/* ResetKalmanState, :2015-2029 */
static void kalman_reset(ora_kalman_state *s, const ora_kalman_params *kp, double first_meas) {
    memset(s, 0, sizeof(*s));
    s->pos = first_meas;
    s->vel = kp->init_vel;
    s->acc = kp->init_acc;
    s->jerk = kp->init_jerk;
    s->P[0][0] = dmax(1e-9, kp->init_var_pos);
    s->P[1][1] = dmax(1e-9, kp->init_var_vel);
    s->P[2][2] = dmax(1e-9, kp->init_var_acc);
    s->P[3][3] = dmax(1e-9, kp->init_var_jerk);
    s->ema_ready = 0;
}

/* StepKalman4D, :2031-2125 -- same expression order as the MQL5 source. */
static double kalman_step(ora_kalman_state *s, const ora_kalman_params *kp, double z) {
    const double q_scale = dmax(0.05, kp->follow_strength);
    double Qp = dmax(1e-9, kp->q_pos * q_scale);
    double Qv = dmax(1e-9, kp->q_vel * q_scale);
    double Qa = dmax(1e-9, kp->q_acc * q_scale);
    double Qj = dmax(1e-9, kp->q_jerk * q_scale);
    double R = dmax(1e-9, kp->meas_noise);
    double(*P)[4] = s->P;

    double x0p = s->pos + s->vel + 0.5 * s->acc + (1.0 / 6.0) * s->jerk;
    double x1p = s->vel + s->acc + 0.5 * s->jerk;
    double x2p = s->acc + s->jerk;
    double x3p = s->jerk;

    double P00p = P[0][0] + P[0][1] + 0.5 * P[0][2] + (1.0 / 6.0) * P[0][3]
                + P[1][0] + P[1][1] + 0.5 * P[1][2] + (1.0 / 6.0) * P[1][3]
                + 0.5 * P[2][0] + 0.5 * P[2][1] + 0.25 * P[2][2] + (1.0 / 12.0) * P[2][3]
                + (1.0 / 6.0) * P[3][0] + (1.0 / 6.0) * P[3][1] + (1.0 / 12.0) * P[3][2] + (1.0 / 36.0) * P[3][3]
                + Qp;
    double P01p = P[0][1] + P[0][2] + 0.5 * P[0][3] + P[1][1] + P[1][2] + 0.5 * P[1][3] + 0.5 * P[2][1]
                + 0.5 * P[2][2] + 0.25 * P[2][3] + (1.0 / 6.0) * P[3][1] + (1.0 / 6.0) * P[3][2] + (1.0 / 12.0) * P[3][3];
    double P02p = P[0][2] + P[0][3] + P[1][2] + P[1][3] + 0.5 * P[2][2] + 0.5 * P[2][3] + (1.0 / 6.0) * P[3][2]
                + (1.0 / 6.0) * P[3][3];
    double P03p = P[0][3] + P[1][3] + 0.5 * P[2][3] + (1.0 / 6.0) * P[3][3];
    double P11p = P[1][1] + 2.0 * P[1][2] + P[1][3] + P[2][1] + 2.0 * P[2][2] + P[2][3] + 0.5 * P[3][1]
                + 0.5 * P[3][2] + 0.25 * P[3][3] + Qv;
    double P12p = P[1][2] + P[1][3] + P[2][2] + P[2][3] + 0.5 * P[3][2] + 0.5 * P[3][3];
    double P13p = P[1][3] + P[2][3] + 0.5 * P[3][3];
    double P22p = P[2][2] + 2.0 * P[2][3] + P[3][3] + Qa;
    double P23p = P[2][3] + P[3][3];
    double P33p = P[3][3] + Qj;
    double P10p = P01p, P20p = P02p, P30p = P03p;
    double P21p = P12p, P31p = P13p, P32p = P23p;

    double y = z - x0p;
    double S = P00p + R;
    if (kp->adapt_gain > 0.0) {
        double sigma = sqrt(S);
        double k = dmin(5.0, fabs(y) / sigma) * kp->adapt_gain;
        double boost = 1.0 + k;
        P00p += (boost - 1.0) * Qp;
        P11p += (boost - 1.0) * Qv;
        P22p += (boost - 1.0) * Qa;
        P33p += (boost - 1.0) * Qj;
        S = P00p + R;
    }
    if (kp->clip_std > 0.0) {
        double sigma = sqrt(S);
        double lim = kp->clip_std * sigma;
        if (y > lim) y = lim;
        if (y < -lim) y = -lim;
    }
    double K0 = P00p / S, K1 = P10p / S, K2 = P20p / S, K3 = P30p / S;

    s->pos = x0p + K0 * y;
    s->vel = x1p + K1 * y;
    s->acc = x2p + K2 * y;
    s->jerk = x3p + K3 * y;

    double P00n = (1.0 - K0) * P00p, P01n = (1.0 - K0) * P01p, P02n = (1.0 - K0) * P02p, P03n = (1.0 - K0) * P03p;
    double P10n = P10p - K1 * P00p, P11n = P11p - K1 * P01p, P12n = P12p - K1 * P02p, P13n = P13p - K1 * P03p;
    double P20n = P20p - K2 * P00p, P21n = P21p - K2 * P01p, P22n = P22p - K2 * P02p, P23n = P23p - K2 * P03p;
    double P30n = P30p - K3 * P00p, P31n = P31p - K3 * P01p, P32n = P32p - K3 * P02p, P33n = P33p - K3 * P03p;

    P[0][0] = dmax(1e-12, P00n); P[0][1] = P01n; P[0][2] = P02n; P[0][3] = P03n;
    P[1][0] = P10n; P[1][1] = dmax(1e-12, P11n); P[1][2] = P12n; P[1][3] = P13n;
    P[2][0] = P20n; P[2][1] = P21n; P[2][2] = dmax(1e-12, P22n); P[2][3] = P23n;
    P[3][0] = P30n; P[3][1] = P31n; P[3][2] = P32n; P[3][3] = dmax(1e-12, P33n);

    double out = s->pos;
    if (kp->ema_blend_period > 0.0) { /* :2117-2123 */
        double alpha = 2.0 / (kp->ema_blend_period + 1.0);
        if (!s->ema_ready) { s->ema_prev = out; s->ema_ready = 1; }
        s->ema_prev = alpha * out + (1.0 - alpha) * s->ema_prev;
        out = s->ema_prev;
    }
    return out;
}

/* Per-window Kalman detrend (north-star; builder-defined -- the reference
 * runs the filter once per bar on the newest sample, :3354-3360).  Same
 * call discipline as the reference call site: if not ready, Reset with the
 * first measurement, then Step on that same measurement.  Window-local:
 *   reset(x[0]); trend[j] = step(x[j]); d[j] = x[j] - trend[j].          */
ORA_EXPORT void ora_kalman_trend(const double *x, int n, const double *params16, double *trend) {
    ora_kalman_params kp;
    memcpy(&kp, params16, sizeof(kp));
    ora_kalman_state s;
    kalman_reset(&s, &kp, x[0]);
    for (int j = 0; j < n; j++) trend[j] = kalman_step(&s, &kp, x[j]);
}

ORA_EXPORT void ora_detrend_kalman(const double *x, int n, const double *params16, double *d) {
    double *t = (double *)malloc(sizeof(double) * (size_t)n);
    ora_kalman_trend(x, n, params16, t);
    for (int j = 0; j < n; j++) d[j] = x[j] - t[j];
    free(t);
}

/* ----------------------------------------------------------------- windows */

/* ApplyHann/Hamming/Blackman/BartlettWindow + ApplyWindow,
 * L/WaveSpecZZ_1.0.2.mq5:884-935.  Symmetric windows (denominator n-1). */
ORA_EXPORT double ora_window_value(int type, int i, int n) {
    switch (type) {
    case ORA_WIN_HANN: return 0.5 * (1.0 - cos(2.0 * M_PI * i / (n - 1)));
    case ORA_WIN_HAMMING: return 0.54 - 0.46 * cos(2.0 * M_PI * i / (n - 1));
    case ORA_WIN_BLACKMAN:
        return 0.42 - 0.5 * cos(2.0 * M_PI * i / (n - 1)) + 0.08 * cos(4.0 * M_PI * i / (n - 1));
    case ORA_WIN_BARTLETT: return 1.0 - fabs((2.0 * i - n + 1) / (n - 1));
    default: return 1.0;
    }
}

ORA_EXPORT void ora_apply_window(double *data, int n, int type) {
    if (type == ORA_WIN_NONE) return; /* :927-929 rectangular: no-op */
    for (int i = 0; i < n; i++) data[i] *= ora_window_value(type, i, n);
}

/* --------------------------------------------------------------------- FFT */

/* FourierTransformManual, L/WaveSpecZZ_1.0.2.mq5:938-974 (byte-identical in
 * L/WaveSpecZZ_1.0.4-new.mq5:998-1034): in-place iterative radix-2 DIT,
 * bit-reversal, twiddle recurrence w *= wlen, sign -2*pi/len. */
ORA_EXPORT void ora_fft_manual(const double *data, int n, double *fft_real, double *fft_imag) {
    if (n <= 1) return; /* :940 */
    double *temp = (double *)malloc(sizeof(double) * (size_t)n);
    memcpy(temp, data, sizeof(double) * (size_t)n);
    for (int i = 1, j = 0; i < n; i++) {
        int bit = n >> 1;
        for (; (j & bit) != 0; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) { double t = temp[i]; temp[i] = temp[j]; temp[j] = t; }
    }
    memcpy(fft_real, temp, sizeof(double) * (size_t)n);
    memset(fft_imag, 0, sizeof(double) * (size_t)n);
    free(temp);
    for (int len = 2; len <= n; len <<= 1) {
        double ang = -2 * M_PI / len;
        double wlen_real = cos(ang), wlen_imag = sin(ang);
        for (int i = 0; i < n; i += len) {
            double w_real = 1.0, w_imag = 0.0;
            for (int j = 0; j < len / 2; j++) {
                int idx1 = i + j, idx2 = i + j + len / 2;
                double t_real = fft_real[idx2] * w_real - fft_imag[idx2] * w_imag;
                double t_imag = fft_real[idx2] * w_imag + fft_imag[idx2] * w_real;
                fft_real[idx2] = fft_real[idx1] - t_real;
                fft_imag[idx2] = fft_imag[idx1] - t_imag;
                fft_real[idx1] += t_real;
                fft_imag[idx1] += t_imag;
                double w_temp = w_real;
                w_real = w_real * wlen_real - w_imag * wlen_imag;
                w_imag = w_temp * wlen_imag + w_imag * wlen_real;
            }
        }
    }
}

/* gpu_fft_real_forward output contract, inferred from its callers
 * (FftProcessor::Run 1.1.0:518-528; L/WaveSpecZZ_1.0.4-new.mq5:3183-3190):
 * out has `len` doubles, out[2k] = Re X_k, out[2k+1] = Im X_k, k < len/2. */
ORA_EXPORT void ora_pack_interleaved(const double *re, const double *im, int n, double *out) {
    for (int k = 0; k < n / 2; k++) { out[2 * k] = re[k]; out[2 * k + 1] = im[k]; }
}

/* spectrum[k] = re^2 + im^2 for k < N/2 (1.1.0:529-530;
 * L/WaveSpecZZ_1.0.2.mq5:3097-3101). */
ORA_EXPORT void ora_power(const double *re, const double *im, int n, double *spec) {
    for (int k = 0; k < n / 2; k++) spec[k] = re[k] * re[k] + im[k] * im[k];
}

/* ------------------------------------------------------------- top-k scan */

/* Top-k bin scan of L/WaveSpecZZ_1.0.3-pla-kalman-fast-gpuopt-nodetrend.mq5:536-554
 * (the immediate consumer of the spectrum in the 1.1.0 predecessor), with k
 * generalised from 8: bins in [ceil(N/MaxP), floor(N/MinP)] (max clamped to
 * bins-1), inserted in ascending bin order with a strict '>' (ties keep the
 * earlier bin), empty slots (-1, -1).  Record per slot: bin, power, Re X,
 * Im X (phase/amplitude reconstruction :559-573 needs Re/Im). */
ORA_EXPORT void ora_topk_bins(const double *re, const double *im, int n, int top_k, double min_period,
                              double max_period, double *rec) {
    double top_pow[64];
    int top_bin[64];
    if (top_k > 64) top_k = 64;
    for (int s = 0; s < top_k; s++) { top_pow[s] = -1.0; top_bin[s] = -1; }
    const int bins = n / 2;
    int min_index = (int)ceil((double)n / max_period);
    int max_index = (int)floor((double)n / min_period);
    if (max_index >= bins) max_index = bins - 1;
    for (int b = min_index; b <= max_index; b++) {
        if (b < 0) continue;
        double p = re[b] * re[b] + im[b] * im[b];
        for (int s = 0; s < top_k; s++) {
            if (p > top_pow[s]) {
                for (int t = top_k - 1; t > s; t--) { top_pow[t] = top_pow[t - 1]; top_bin[t] = top_bin[t - 1]; }
                top_pow[s] = p; top_bin[s] = b;
                break;
            }
        }
    }
    for (int s = 0; s < top_k; s++) {
        rec[4 * s] = top_bin[s];
        rec[4 * s + 1] = top_pow[s];
        rec[4 * s + 2] = top_bin[s] >= 0 ? re[top_bin[s]] : 0.0;
        rec[4 * s + 3] = top_bin[s] >= 0 ? im[top_bin[s]] : 0.0;
    }
}

/* ------------------------------------------------------ inverse real FFT */

/* Complex radix-2 DIT with FourierTransformManual's structure
 * (L/WaveSpecZZ_1.0.2.mq5:938-974) on a complex input: bit reversal, then
 * butterflies with the twiddle recurrence and sign -2*pi/len. */
static void cfft_manual(double *re, double *im, int n) {
    for (int i = 1, j = 0; i < n; i++) {
        int bit = n >> 1;
        for (; (j & bit) != 0; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) {
            double t = re[i]; re[i] = re[j]; re[j] = t;
            t = im[i]; im[i] = im[j]; im[j] = t;
        }
    }
    for (int len = 2; len <= n; len <<= 1) {
        double ang = -2 * M_PI / len;
        double wlen_real = cos(ang), wlen_imag = sin(ang);
        for (int i = 0; i < n; i += len) {
            double w_real = 1.0, w_imag = 0.0;
            for (int j = 0; j < len / 2; j++) {
                int idx1 = i + j, idx2 = i + j + len / 2;
                double t_real = re[idx2] * w_real - im[idx2] * w_imag;
                double t_imag = re[idx2] * w_imag + im[idx2] * w_real;
                re[idx2] = re[idx1] - t_real;
                im[idx2] = im[idx1] - t_imag;
                re[idx1] += t_real;
                im[idx1] += t_imag;
                double w_temp = w_real;
                w_real = w_real * wlen_real - w_imag * wlen_imag;
                w_imag = w_temp * wlen_imag + w_imag * wlen_real;
            }
        }
    }
}

/* gpu_fft_real_inverse (declared L/WaveSpecZZ_1.0.4-core.mq5:65; called at
 * :426 on the output of gpu_fft_real_forward :344 after the spectral stages,
 * result copied back into the time-domain pipeline :432).  DLL-only, no CPU
 * counterpart in the reference, so BUILD-DEFINED as the exact inverse of the
 * packed forward layout: X_k = in[2k] + i in[2k+1] for 0 < k < N/2,
 * X_0 = in[0] (a real signal's Im X_0 is 0: in[1] is ignored), X_{N/2} = 0
 * (the layout has no slot for it), X_{N-k} = conj X_k, and
 * x_n = (1/N) sum_k X_k e^{+2 pi i k n/N} = conj(DFT(conj X))_n / N. */
ORA_EXPORT void ora_fft_real_inverse(const double *in, int n, double *out) {
    if (n < 2) { if (n == 1) out[0] = in[0]; return; }
    double *re = (double *)malloc(sizeof(double) * (size_t)n);
    double *im = (double *)malloc(sizeof(double) * (size_t)n);
    const int h = n / 2;
    for (int k = 0; k < n; k++) { /* conj X_k */
        if (k == 0) { re[k] = in[0]; im[k] = 0.0; }
        else if (k < h) { re[k] = in[2 * k]; im[k] = -in[2 * k + 1]; }
        else if (k == h) { re[k] = 0.0; im[k] = 0.0; }
        else { re[k] = in[2 * (n - k)]; im[k] = in[2 * (n - k) + 1]; }
    }
    cfft_manual(re, im, n);
    for (int i = 0; i < n; i++) out[i] = re[i] / (double)n;
    free(re); free(im);
}

/* -------------------------------------------------- phase / unwrap / delay */

/* CalculateFFTPhase + UnwrapPhase + CalculateGroupDelay,
 * L/WaveSpecZZ_1.0.4-new.mq5:1040-1120 (same as L/WaveSpecZZ_1.0.2.mq5:980-1060),
 * called at :3225-3227 with n = InpFFTWindow over fft_real/fft_imag as the GPU
 * unpack path leaves them (:3183-3196): X_k for k < N/2, zero above.
 * Same expression order as the MQL5 source (sequential unwrap).  Writes the
 * first N/2 entries of each requested array (NULL skips it). */
ORA_EXPORT void ora_phase_unwrap(const double *re, const double *im, int n, double *phase_out,
                                 double *unwrapped_out, double *gd_out) {
    if (n < 2) return;
    double *ph = (double *)malloc(sizeof(double) * (size_t)n);
    double *u = (double *)malloc(sizeof(double) * (size_t)n);
    double *gd = (double *)malloc(sizeof(double) * (size_t)n);
    for (int i = 0; i < n; i++) /* :1046-1049; upper half zero -> atan2(0, 0) = 0 */
        ph[i] = i < n / 2 ? atan2(im[i], re[i]) : atan2(0.0, 0.0);
    u[0] = ph[0]; /* :1063 */
    for (int i = 1; i < n; i++) { /* :1066-1080 */
        double diff = ph[i] - ph[i - 1];
        double correction = 0;
        if (diff > M_PI) correction = -2.0 * M_PI;
        else if (diff < -M_PI) correction = 2.0 * M_PI;
        u[i] = u[i - 1] + diff + correction;
    }
    if (n < 3) { /* :1092-1096 */
        for (int i = 0; i < n; i++) gd[i] = 0.0;
    } else {
        gd[0] = -(u[1] - u[0]); /* :1102 */
        for (int i = 1; i < n - 1; i++) gd[i] = -(u[i + 1] - u[i - 1]) / 2.0; /* :1105-1108 */
        gd[n - 1] = -(u[n - 1] - u[n - 2]); /* :1111 */
        for (int i = 0; i < n; i++) { /* :1115-1119 */
            if (gd[i] > 100.0) gd[i] = 100.0;
            if (gd[i] < -100.0) gd[i] = -100.0;
        }
    }
    for (int k = 0; k < n / 2; k++) {
        if (phase_out) phase_out[k] = ph[k];
        if (unwrapped_out) unwrapped_out[k] = u[k];
        if (gd_out) gd_out[k] = gd[k];
    }
    free(ph); free(u); free(gd);
}

/* ---------------------------------------------------------- full pipeline */

static int is_pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }

/* One window through the legacy CPU path (L/WaveSpecZZ_1.0.2.mq5:3019-3101):
 * detrend -> ApplyWindow -> FourierTransformManual -> |X|^2 (output 0) or the
 * packed gpu_fft_real_forward layout (output 1).  Returns 0 or -1. */
ORA_EXPORT int ora_window_spectrum(const double *x, int n, int detrend, int window, int trend_period,
                                   const double *kalman16, int output, double *out) {
    if (!is_pow2(n) || n < 2) return -1;
    double *d = (double *)malloc(sizeof(double) * (size_t)n);
    double *re = (double *)malloc(sizeof(double) * (size_t)n);
    double *im = (double *)malloc(sizeof(double) * (size_t)n);
    switch (detrend) {
    case ORA_DETREND_MEAN: ora_detrend_mean(x, n, d); break;
    case ORA_DETREND_IIR: ora_detrend_iir(x, n, trend_period, d); break;
    case ORA_DETREND_KALMAN: {
        double def[16];
        if (!kalman16) { ora_kalman_default_params(def); kalman16 = def; }
        ora_detrend_kalman(x, n, kalman16, d);
        break;
    }
    default: memcpy(d, x, sizeof(double) * (size_t)n); break; /* 1.1.0:1239 */
    }
    ora_apply_window(d, n, window);
    ora_fft_manual(d, n, re, im);
    if (output == 1) ora_pack_interleaved(re, im, n, out);
    else ora_power(re, im, n, out);
    free(d); free(re); free(im);
    return 0;
}

/* Top-k records for every window of a series (4*top_k doubles per window). */
ORA_EXPORT int64_t ora_batch_topk(const double *series, int64_t series_len, int n, int64_t hop, int detrend,
                                  int window, int trend_period, const double *kalman16, int top_k, double min_period,
                                  double max_period, double *out) {
    if (!is_pow2(n) || hop <= 0 || series_len < n) return -1;
    int64_t nwin = 1 + (series_len - n) / hop;
#pragma omp parallel for schedule(static)
    for (int64_t w = 0; w < nwin; w++) {
        double *packed = (double *)malloc(sizeof(double) * (size_t)n);
        double *re = (double *)malloc(sizeof(double) * (size_t)n / 2);
        double *im = (double *)malloc(sizeof(double) * (size_t)n / 2);
        ora_window_spectrum(series + w * hop, n, detrend, window, trend_period, kalman16, 1, packed);
        for (int k = 0; k < n / 2; k++) { re[k] = packed[2 * k]; im[k] = packed[2 * k + 1]; }
        ora_topk_bins(re, im, n, top_k, min_period, max_period, out + w * 4 * top_k);
        free(packed); free(re); free(im);
    }
    return nwin;
}

/* Batch over a chronological series: window w = series[w*hop, w*hop+N).
 * nwin = 1 + (len-N)/hop as in 1.1.0:1016.  Output row stride N/2 (power)
 * or N (packed).  `threads` > 1 uses OpenMP over windows when compiled with
 * -fopenmp (the all-core CPU baseline).  Returns number of windows. */
ORA_EXPORT int64_t ora_batch_spectrum(const double *series, int64_t series_len, int n, int64_t hop,
                                      int64_t max_windows, int detrend, int window, int trend_period,
                                      const double *kalman16, int output, double *out) {
    if (!is_pow2(n) || hop <= 0 || series_len < n) return -1;
    int64_t nwin = 1 + (series_len - n) / hop;
    if (max_windows > 0 && max_windows < nwin) nwin = max_windows;
    const int64_t stride = output == 1 ? n : n / 2;
#pragma omp parallel for schedule(static)
    for (int64_t w = 0; w < nwin; w++)
        ora_window_spectrum(series + w * hop, n, detrend, window, trend_period, kalman16, output,
                            out + w * stride);
    return nwin;
}

/* MTB_OUT_PHASE records for every window: [P_k | unwrapped phase_k |
 * group delay_k], k < N/2 (3N/2 doubles per window). */
ORA_EXPORT int64_t ora_batch_phase(const double *series, int64_t series_len, int n, int64_t hop, int detrend,
                                   int window, int trend_period, const double *kalman16, double *out) {
    if (!is_pow2(n) || hop <= 0 || series_len < n) return -1;
    int64_t nwin = 1 + (series_len - n) / hop;
    const int h = n / 2;
#pragma omp parallel for schedule(static)
    for (int64_t w = 0; w < nwin; w++) {
        double *packed = (double *)malloc(sizeof(double) * (size_t)n);
        double *re = (double *)malloc(sizeof(double) * (size_t)h);
        double *im = (double *)malloc(sizeof(double) * (size_t)h);
        double *rec = out + w * 3 * (int64_t)h;
        ora_window_spectrum(series + w * hop, n, detrend, window, trend_period, kalman16, 1, packed);
        for (int k = 0; k < h; k++) { re[k] = packed[2 * k]; im[k] = packed[2 * k + 1]; }
        ora_power(re, im, n, rec);
        ora_phase_unwrap(re, im, n, NULL, rec + h, rec + 2 * h);
        free(packed); free(re); free(im);
    }
    return nwin;
}

/* MTB_OUT_TOPK_PHASE records: the top-k scan (ora_topk_bins) plus the
 * unwrapped phase and group delay of each chosen bin -- the values the ETA
 * estimators read at the dominant bin (L/WaveSpecZZ_1.0.4-new.mq5:1165, :1239)
 * -- 6 doubles per slot [bin, power, Re, Im, phase, delay]; empty slots
 * [-1, -1, 0, 0, 0, 0]. */
ORA_EXPORT int64_t ora_batch_topk_phase(const double *series, int64_t series_len, int n, int64_t hop, int detrend,
                                        int window, int trend_period, const double *kalman16, int top_k,
                                        double min_period, double max_period, double *out) {
    if (!is_pow2(n) || hop <= 0 || series_len < n || top_k < 1 || top_k > 64) return -1;
    int64_t nwin = 1 + (series_len - n) / hop;
    const int h = n / 2;
#pragma omp parallel for schedule(static)
    for (int64_t w = 0; w < nwin; w++) {
        double *packed = (double *)malloc(sizeof(double) * (size_t)n);
        double *re = (double *)malloc(sizeof(double) * (size_t)h);
        double *im = (double *)malloc(sizeof(double) * (size_t)h);
        double *u = (double *)malloc(sizeof(double) * (size_t)h);
        double *gd = (double *)malloc(sizeof(double) * (size_t)h);
        double rec4[4 * 64];
        ora_window_spectrum(series + w * hop, n, detrend, window, trend_period, kalman16, 1, packed);
        for (int k = 0; k < h; k++) { re[k] = packed[2 * k]; im[k] = packed[2 * k + 1]; }
        ora_topk_bins(re, im, n, top_k, min_period, max_period, rec4);
        ora_phase_unwrap(re, im, n, NULL, u, gd);
        double *rec = out + w * 6 * (int64_t)top_k;
        for (int s = 0; s < top_k; s++) {
            const int b = (int)rec4[4 * s];
            for (int j = 0; j < 4; j++) rec[6 * s + j] = rec4[4 * s + j];
            rec[6 * s + 4] = b >= 0 ? u[b] : 0.0;
            rec[6 * s + 5] = b >= 0 ? gd[b] : 0.0;
        }
        free(packed); free(re); free(im); free(u); free(gd);
    }
    return nwin;
}
