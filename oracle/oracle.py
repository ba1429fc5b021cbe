"""ctypes view of the CPU restatement (wavespec_oracle.c) + numpy helpers.

TEST INFRASTRUCTURE ONLY -- the checker for tests/, __graft_entry__.smoke()
and the cpu_baseline leg of bench.py.  Never imported by the product
(fft-wavespec_amd/).  Parity status: "parity unpinned" against the reference
binary (MQL5 + un-vendored mt-bridge.dll, no reference fixtures); pinned by
analytic known-answer tests and numpy.fft in tests/test_oracle.py.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
LIB = ROOT / "build" / "libwavespec_oracle.so"
DETREND = {"none": 0, "mean": 1, "iir": 2, "kalman": 3}
WINDOW = {"none": 0, "hann": 1, "hamming": 2, "blackman": 3, "bartlett": 4}
KALMAN_DEFAULTS = [1.0, 0.01, 0.003, 0.0008, 0.0002, 0.8, 1.0, 16.0, 9.0, 4.0, 1.0, 0.0, 0.0, 0.0, 6.0, 0.0]

_d = C.POINTER(C.c_double)
_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(ROOT)], check=True)
    return LIB


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        h = C.CDLL(str(LIB))
        h.ora_fft_manual.argtypes = [_d, C.c_int, _d, _d]
        h.ora_window_spectrum.argtypes = [_d, C.c_int, C.c_int, C.c_int, C.c_int, _d, C.c_int, _d]
        h.ora_window_spectrum.restype = C.c_int
        h.ora_batch_spectrum.argtypes = [_d, C.c_int64, C.c_int, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int,
                                         _d, C.c_int, _d]
        h.ora_batch_spectrum.restype = C.c_int64
        h.ora_window_value.argtypes = [C.c_int, C.c_int, C.c_int]
        h.ora_window_value.restype = C.c_double
        h.ora_detrend_iir.argtypes = [_d, C.c_int, C.c_int, _d]
        h.ora_detrend_mean.argtypes = [_d, C.c_int, _d]
        h.ora_kalman_trend.argtypes = [_d, C.c_int, _d, _d]
        h.ora_gather_series.argtypes = [_d, C.c_int64, C.c_int, _d]
        h.ora_topk_bins.argtypes = [_d, _d, C.c_int, C.c_int, C.c_double, C.c_double, _d]
        h.ora_batch_topk.argtypes = [_d, C.c_int64, C.c_int, C.c_int64, C.c_int, C.c_int, C.c_int, _d, C.c_int,
                                     C.c_double, C.c_double, _d]
        h.ora_batch_topk.restype = C.c_int64
        h.ora_fft_real_inverse.argtypes = [_d, C.c_int, _d]
        h.ora_phase_unwrap.argtypes = [_d, _d, C.c_int, _d, _d, _d]
        h.ora_batch_phase.argtypes = [_d, C.c_int64, C.c_int, C.c_int64, C.c_int, C.c_int, C.c_int, _d, _d]
        h.ora_batch_phase.restype = C.c_int64
        h.ora_batch_topk_phase.argtypes = [_d, C.c_int64, C.c_int, C.c_int64, C.c_int, C.c_int, C.c_int, _d, C.c_int,
                                           C.c_double, C.c_double, _d]
        h.ora_batch_topk_phase.restype = C.c_int64
        _lib = h
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(_d)


def fft_manual(x: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """FourierTransformManual (L/WaveSpecZZ_1.0.2.mq5:938-974)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    re, im = np.empty_like(x), np.empty_like(x)
    lib().ora_fft_manual(_p(x), x.size, _p(re), _p(im))
    return re, im


def window_spectrum(x, detrend="none", window="hann", trend_period=0, kalman=None, output="power") -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float64)
    n = x.size
    out = np.empty(n if output == "packed" else n // 2)
    kp = None if kalman is None else np.ascontiguousarray(kalman, dtype=np.float64)
    st = lib().ora_window_spectrum(_p(x), n, DETREND[detrend], WINDOW[window], trend_period,
                                   None if kp is None else _p(kp), 1 if output == "packed" else 0, _p(out))
    if st != 0:
        raise ValueError("oracle rejected the window (N must be a power of two)")
    return out


def batch_spectrum(series, n, hop, detrend="none", window="hann", trend_period=0, kalman=None, output="power",
                   max_windows=0) -> np.ndarray:
    """ora_batch_spectrum: window w = series[w*hop : w*hop+n] (OpenMP over windows)."""
    s = np.ascontiguousarray(series, dtype=np.float64)
    nwin = 1 + (s.size - n) // hop
    if max_windows:
        nwin = min(nwin, max_windows)
    rec = n if output == "packed" else n // 2
    out = np.empty((nwin, rec))
    kp = None if kalman is None else np.ascontiguousarray(kalman, dtype=np.float64)
    got = lib().ora_batch_spectrum(_p(s), s.size, n, hop, nwin, DETREND[detrend], WINDOW[window], trend_period,
                                   None if kp is None else _p(kp), 1 if output == "packed" else 0, _p(out))
    assert got == nwin, (got, nwin)
    return out


def batch_topk(series, n, hop, detrend="none", window="hann", trend_period=0, kalman=None, top_k=8,
               min_period=18.0, max_period=200.0) -> np.ndarray:
    """(nwin, top_k, 4) records [bin, power, Re X, Im X] (gpuopt-nodetrend.mq5:536-554)."""
    s = np.ascontiguousarray(series, dtype=np.float64)
    nwin = 1 + (s.size - n) // hop
    out = np.empty((nwin, top_k, 4))
    kp = np.ascontiguousarray(KALMAN_DEFAULTS if kalman is None else kalman, dtype=np.float64)
    got = lib().ora_batch_topk(_p(s), s.size, n, hop, DETREND[detrend], WINDOW[window], trend_period, _p(kp), top_k,
                               min_period, max_period, _p(out))
    assert got == nwin
    return out


def fft_real_inverse(packed) -> np.ndarray:
    """Build-defined inverse of the packed forward layout (wavespec_oracle.c ora_fft_real_inverse)."""
    p = np.ascontiguousarray(packed, dtype=np.float64)
    out = np.empty_like(p)
    lib().ora_fft_real_inverse(_p(p), p.size, _p(out))
    return out


def phase_unwrap(packed) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(wrapped, unwrapped, group delay) for k < len/2 of a packed spectrum (1.0.4-new.mq5:1040-1120)."""
    p = np.ascontiguousarray(packed, dtype=np.float64)
    re, im = np.ascontiguousarray(p[0::2]), np.ascontiguousarray(p[1::2])
    h = p.size // 2
    ph, u, gd = np.empty(h), np.empty(h), np.empty(h)
    lib().ora_phase_unwrap(_p(re), _p(im), p.size, _p(ph), _p(u), _p(gd))
    return ph, u, gd


def batch_phase(series, n, hop, detrend="none", window="hann", trend_period=0, kalman=None) -> np.ndarray:
    """(nwin, 3, N/2): [power, unwrapped phase, group delay] per window (MTB_OUT_PHASE)."""
    s = np.ascontiguousarray(series, dtype=np.float64)
    nwin = 1 + (s.size - n) // hop
    out = np.empty((nwin, 3, n // 2))
    kp = np.ascontiguousarray(KALMAN_DEFAULTS if kalman is None else kalman, dtype=np.float64)
    got = lib().ora_batch_phase(_p(s), s.size, n, hop, DETREND[detrend], WINDOW[window], trend_period, _p(kp), _p(out))
    assert got == nwin
    return out


def batch_topk_phase(series, n, hop, detrend="none", window="hann", trend_period=0, kalman=None, top_k=8,
                     min_period=18.0, max_period=200.0) -> np.ndarray:
    """(nwin, top_k, 6): [bin, power, Re, Im, unwrapped phase, group delay] (MTB_OUT_TOPK_PHASE)."""
    s = np.ascontiguousarray(series, dtype=np.float64)
    nwin = 1 + (s.size - n) // hop
    out = np.empty((nwin, top_k, 6))
    kp = np.ascontiguousarray(KALMAN_DEFAULTS if kalman is None else kalman, dtype=np.float64)
    got = lib().ora_batch_topk_phase(_p(s), s.size, n, hop, DETREND[detrend], WINDOW[window], trend_period, _p(kp),
                                     top_k, min_period, max_period, _p(out))
    assert got == nwin
    return out


# ---------------------------------------------------------------- numpy cross-check
def numpy_kalman_trend(X, params=None, dtype=np.float64) -> np.ndarray:
    """Second, independent transliteration of ResetKalmanState / StepKalman4D
    (L/WaveSpecZZ_1.0.3-pla-kalman-fast.mq5:2015-2029 / :2031-2125), vectorised over windows:
    X is (W, n) or (n,); every window is reset with its first sample and stepped over all of its
    samples (the per-window discipline of wavespec_oracle.c ora_kalman_trend).  Expression order
    follows the MQL5 source statement by statement, including the full 16-entry covariance and
    the P11 prediction of :2052; shares no code with the C oracle.

    dtype=np.float32 runs the same statements in float32 (numpy keeps float32 arrays float32
    against Python-float constants): an emulation of a SEQUENTIAL fp32 filter, used to bound
    what fp32 arithmetic itself costs on a given input (tests of the device's fp32 filter)."""
    kp = KALMAN_DEFAULTS if params is None else list(params)
    (follow, q_pos, q_vel, q_acc, q_jerk, adapt_gain, meas_noise, var_pos, var_vel, var_acc, var_jerk, init_vel,
     init_acc, init_jerk, clip_std, ema_period) = [float(v) for v in kp]
    X = np.asarray(X, dtype=dtype)
    one = X.ndim == 1
    X = np.atleast_2d(X)
    W, n = X.shape
    # ResetKalmanState(first_meas) :2015-2029
    pos, vel = X[:, 0].copy(), np.full(W, init_vel, dtype=dtype)
    acc, jerk = np.full(W, init_acc, dtype=dtype), np.full(W, init_jerk, dtype=dtype)
    P = np.zeros((W, 4, 4), dtype=dtype)
    P[:, 0, 0], P[:, 1, 1] = max(1e-9, var_pos), max(1e-9, var_vel)
    P[:, 2, 2], P[:, 3, 3] = max(1e-9, var_acc), max(1e-9, var_jerk)
    ema_ready, ema_prev = False, np.zeros(W, dtype=dtype)
    q_scale = max(0.05, follow)
    Qp, Qv = max(1e-9, q_pos * q_scale), max(1e-9, q_vel * q_scale)
    Qa, Qj = max(1e-9, q_acc * q_scale), max(1e-9, q_jerk * q_scale)
    R = max(1e-9, meas_noise)
    trend = np.empty((W, n), dtype=dtype)
    g = lambda i, j: P[:, i, j]  # noqa: E731
    for t in range(n):
        z = X[:, t]
        x0p = pos + vel + 0.5 * acc + (1.0 / 6.0) * jerk
        x1p = vel + acc + 0.5 * jerk
        x2p = acc + jerk
        x3p = jerk
        P00p = (g(0, 0) + g(0, 1) + 0.5 * g(0, 2) + (1.0 / 6.0) * g(0, 3)
                + g(1, 0) + g(1, 1) + 0.5 * g(1, 2) + (1.0 / 6.0) * g(1, 3)
                + 0.5 * g(2, 0) + 0.5 * g(2, 1) + 0.25 * g(2, 2) + (1.0 / 12.0) * g(2, 3)
                + (1.0 / 6.0) * g(3, 0) + (1.0 / 6.0) * g(3, 1) + (1.0 / 12.0) * g(3, 2) + (1.0 / 36.0) * g(3, 3)
                + Qp)
        P01p = (g(0, 1) + g(0, 2) + 0.5 * g(0, 3) + g(1, 1) + g(1, 2) + 0.5 * g(1, 3) + 0.5 * g(2, 1) + 0.5 * g(2, 2)
                + 0.25 * g(2, 3) + (1.0 / 6.0) * g(3, 1) + (1.0 / 6.0) * g(3, 2) + (1.0 / 12.0) * g(3, 3))
        P02p = (g(0, 2) + g(0, 3) + g(1, 2) + g(1, 3) + 0.5 * g(2, 2) + 0.5 * g(2, 3) + (1.0 / 6.0) * g(3, 2)
                + (1.0 / 6.0) * g(3, 3))
        P03p = g(0, 3) + g(1, 3) + 0.5 * g(2, 3) + (1.0 / 6.0) * g(3, 3)
        P11p = (g(1, 1) + 2.0 * g(1, 2) + g(1, 3) + g(2, 1) + 2.0 * g(2, 2) + g(2, 3) + 0.5 * g(3, 1) + 0.5 * g(3, 2)
                + 0.25 * g(3, 3) + Qv)
        P12p = g(1, 2) + g(1, 3) + g(2, 2) + g(2, 3) + 0.5 * g(3, 2) + 0.5 * g(3, 3)
        P13p = g(1, 3) + g(2, 3) + 0.5 * g(3, 3)
        P22p = g(2, 2) + 2.0 * g(2, 3) + g(3, 3) + Qa
        P23p = g(2, 3) + g(3, 3)
        P33p = g(3, 3) + Qj
        P10p, P20p, P30p, P21p, P31p, P32p = P01p, P02p, P03p, P12p, P13p, P23p
        y = z - x0p
        S = P00p + R
        if adapt_gain > 0.0:
            sigma = np.sqrt(S)
            k = np.minimum(5.0, np.abs(y) / sigma) * adapt_gain
            boost = 1.0 + k
            P00p = P00p + (boost - 1.0) * Qp
            P11p = P11p + (boost - 1.0) * Qv
            P22p = P22p + (boost - 1.0) * Qa
            P33p = P33p + (boost - 1.0) * Qj
            S = P00p + R
        if clip_std > 0.0:
            lim = clip_std * np.sqrt(S)
            y = np.where(y > lim, lim, y)
            y = np.where(y < -lim, -lim, y)
        K0, K1, K2, K3 = P00p / S, P10p / S, P20p / S, P30p / S
        pos = x0p + K0 * y
        vel = x1p + K1 * y
        acc = x2p + K2 * y
        jerk = x3p + K3 * y
        rows = ((P00p, P01p, P02p, P03p), (P10p, P11p, P12p, P13p), (P20p, P21p, P22p, P23p),
                (P30p, P31p, P32p, P33p))
        Kv = (K0, K1, K2, K3)
        Pn = np.empty_like(P)
        for j in range(4):
            Pn[:, 0, j] = (1.0 - K0) * rows[0][j]
        for i in range(1, 4):
            for j in range(4):
                Pn[:, i, j] = rows[i][j] - Kv[i] * rows[0][j]
        for i in range(4):
            Pn[:, i, i] = np.maximum(1e-12, Pn[:, i, i])
        P = Pn
        out = pos
        if ema_period > 0.0:  # :2117-2123
            alpha = 2.0 / (ema_period + 1.0)
            if not ema_ready:
                ema_prev, ema_ready = out.copy(), True
            ema_prev = alpha * out + (1.0 - alpha) * ema_prev
            out = ema_prev
        trend[:, t] = out
    return trend[0] if one else trend


def numpy_spectrum(x, detrend="none", window="hann", trend_period=0, kalman=None) -> np.ndarray:
    """Independent numpy restatement (no shared code with the C oracle)."""
    x = np.asarray(x, dtype=np.float64)
    n = x.size
    if detrend == "kalman":
        d = x - numpy_kalman_trend(x, kalman)
    elif detrend == "mean":
        d = x - x.mean()
    elif detrend == "iir" and trend_period > 0:
        om = 2 * np.pi / trend_period
        al = (1 - np.sin(om)) / np.cos(om)
        c = (1 - al) / 2
        t = np.empty(n)
        prev_x, prev_t = x[0], 0.0
        for j in range(n):
            prev_t = c * (x[j] + prev_x) + al * prev_t
            prev_x = x[j]
            t[j] = prev_t
        d = x - t
    else:
        d = x.copy()
    i = np.arange(n)
    w = {"none": np.ones(n),
         "hann": 0.5 * (1 - np.cos(2 * np.pi * i / (n - 1))),
         "hamming": 0.54 - 0.46 * np.cos(2 * np.pi * i / (n - 1)),
         "blackman": 0.42 - 0.5 * np.cos(2 * np.pi * i / (n - 1)) + 0.08 * np.cos(4 * np.pi * i / (n - 1)),
         "bartlett": 1 - np.abs((2 * i - n + 1) / (n - 1))}[window]
    X = np.fft.fft(d * w)[: n // 2]
    return X.real ** 2 + X.imag ** 2


def rel_err(p: np.ndarray, ref: np.ndarray) -> float:
    """Per-window max_k |P - P_ref| / max_k P_ref, worst over windows."""
    p = np.atleast_2d(p)
    ref = np.atleast_2d(ref)
    den = np.max(np.abs(ref), axis=1)
    den = np.where(den > 0, den, 1.0)
    return float(np.max(np.max(np.abs(p - ref), axis=1) / den))


def band(n: int, min_period: float = 18.0, max_period: float = 200.0) -> tuple[int, int]:
    """The reference's scan range [ceil(N/MaxPeriod), floor(N/MinPeriod)] clamped to N/2-1
    (L/WaveSpecZZ_1.0.3-pla-kalman-fast-gpuopt-nodetrend.mq5:539-541; InpMinPeriod 18 /
    InpMaxPeriod 200, 1.1.0:22-23): the cycle bins the indicator actually reads."""
    import math
    kmin = max(0, math.ceil(n / max_period))
    kmax = min(n // 2 - 1, math.floor(n / min_period))
    return kmin, kmax


def inband_err(p: np.ndarray, ref: np.ndarray, kmin: int, kmax: int) -> float:
    """Per-window max_{k in [kmin,kmax]} |P - P_ref| / max_{k in [kmin,kmax]} P_ref, worst over
    windows.  rel_err normalises by the whole row's maximum, which with detrend "none" is P_0
    (~1e6 x the cycle bins at prices ~1.1): this metric holds the cycle bins to the same bar."""
    p = np.atleast_2d(p)[:, kmin:kmax + 1]
    ref = np.atleast_2d(ref)[:, kmin:kmax + 1]
    den = np.max(np.abs(ref), axis=1)
    den = np.where(den > 0, den, 1.0)
    return float(np.max(np.max(np.abs(p - ref), axis=1) / den))


def worst_elementwise(p: np.ndarray, ref: np.ndarray, kmin: int = 0, kmax: int | None = None) -> float:
    """max |P_k - P_ref,k| / |P_ref,k| over the bins [kmin, kmax] (SURVEY 8c "also report worst
    element-wise").  Reported, not a bar over the whole row: bins near zero (e.g. the Hann
    window's nulls) carry round-off far above their own size in any fp64 FFT."""
    p = np.atleast_2d(p)[:, kmin:None if kmax is None else kmax + 1]
    ref = np.atleast_2d(ref)[:, kmin:None if kmax is None else kmax + 1]
    ok = np.abs(ref) > 0
    return float(np.max(np.abs(p - ref)[ok] / np.abs(ref)[ok])) if ok.any() else 0.0

