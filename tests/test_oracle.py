"""CPU tests of the oracle (the CPU restatement of the reference hot path).

The reference holds no fixtures or golden vectors and
its code is MQL5, so the oracle is "parity unpinned" against the reference
binary.  It is pinned here against (a) mathematics -- analytic known-answer
tests and a 50-digit mpmath DFT -- and (b) numpy.fft as independent code,
and (c) the committed golden vectors (regression).
"""
from pathlib import Path

import numpy as np
import pytest

import oracle
from wavespec_amd import synth

GOLDEN = sorted((Path(__file__).parent / "golden").glob("*.npz"))


def test_fft_manual_impulse_and_dc():
    n = 256
    x = np.zeros(n)
    x[0] = 1.0
    re, im = oracle.fft_manual(x)
    assert np.array_equal(re, np.ones(n)) and np.array_equal(im, np.zeros(n))
    re, im = oracle.fft_manual(np.full(n, 2.0))
    assert re[0] == 2.0 * n
    assert np.max(np.abs(re[1:])) < 1e-12 and np.max(np.abs(im)) < 1e-12


@pytest.mark.parametrize("n,k0", [(64, 5), (1024, 37), (4096, 200)])
def test_cosine_bin_rect(n, k0):
    """|X_k0|^2 = (A N/2)^2 for A cos(2 pi k0 t/N), rectangular window."""
    a = 0.75
    x = a * np.cos(2 * np.pi * k0 * np.arange(n) / n)
    p = oracle.window_spectrum(x, "none", "none")
    assert abs(p[k0] - (a * n / 2) ** 2) / (a * n / 2) ** 2 < 1e-12
    mask = np.ones(n // 2, bool)
    mask[k0] = False
    assert np.max(p[mask]) < 1e-18 * n * n


@pytest.mark.parametrize("n", [32, 512, 4096])
def test_parseval(n):
    x = np.random.default_rng(n).standard_normal(n)
    re, im = oracle.fft_manual(x)
    assert abs(np.sum(re ** 2 + im ** 2) / n - np.sum(x ** 2)) / np.sum(x ** 2) < 1e-12


def test_fft_manual_vs_mpmath_exact_dft():
    mp = pytest.importorskip("mpmath")
    mp.mp.dps = 50
    n = 64
    x = synth.random_walk(n, seed=3)
    re, im = oracle.fft_manual(x)
    for k in (0, 1, 7, 31, 32, 63):
        s = mp.fsum(mp.mpf(float(x[t])) * mp.expjpi(-2 * mp.mpf(k * t) / n) for t in range(n))
        assert abs(float(s.real) - re[k]) < 1e-13 and abs(float(s.imag) - im[k]) < 1e-13


@pytest.mark.parametrize("n", [32, 256, 2048])
@pytest.mark.parametrize("detrend,period", [("none", 0), ("mean", 0), ("iir", 1024), ("iir", 40)])
@pytest.mark.parametrize("window", ["none", "hann", "hamming", "blackman", "bartlett"])
def test_oracle_vs_numpy(n, detrend, period, window):
    x = synth.random_walk(n, seed=n + period)
    p = oracle.window_spectrum(x, detrend, window, period)
    ref = oracle.numpy_spectrum(x, detrend, window, period)
    assert oracle.rel_err(p, ref) < 1e-10


def test_packed_layout_matches_fft():
    """out[2k]=Re X_k, out[2k+1]=Im X_k (1.1.0:522-528), so out[1] = Im X_0 = 0."""
    x = synth.sine_noise_window(1024)
    out = oracle.window_spectrum(x, "none", "none", output="packed")
    X = np.fft.fft(x)[:512]
    assert np.max(np.abs(out[0::2] - X.real)) < 1e-9 and np.max(np.abs(out[1::2] - X.imag)) < 1e-9
    assert out[1] == 0.0


def test_hann_is_symmetric_n_minus_1():
    """Symmetric Hann, denominator N-1 (L/WaveSpecZZ_1.0.2.mq5:884-889), not scipy's periodic one."""
    n = 16
    w = np.array([oracle.lib().ora_window_value(1, i, n) for i in range(n)])
    assert w[0] == 0.0 and w[-1] < 1e-15 and np.allclose(w, w[::-1])


def test_gather_reverses_series_order():
    close = np.arange(100, dtype=np.float64)[::-1].copy()  # newest first
    out = np.empty(8)
    oracle.lib().ora_gather_series(oracle._p(close), 5, 8, oracle._p(out))
    assert np.array_equal(out, close[5:13][::-1])


def test_iir_trend_period_nonpositive_is_copy():
    x = synth.random_walk(64, 1)
    assert np.array_equal(oracle.window_spectrum(x, "iir", "hann", 0), oracle.window_spectrum(x, "none", "hann"))


def test_kalman_tracks_a_ramp():
    n = 512
    x = 1.1 + 1e-3 * np.arange(n)
    t = np.empty(n)
    kp = np.asarray(oracle.KALMAN_DEFAULTS)
    oracle.lib().ora_kalman_trend(oracle._p(x), n, oracle._p(kp), oracle._p(t))
    assert abs(t[0] - x[0]) < 1e-12
    assert np.max(np.abs(t[100:] - x[100:])) < 1e-3


@pytest.mark.parametrize("kw", [{}, {"ema": 12.0}, {"adapt": 0.0}, {"clip": 0.0}, {"follow": 2.5, "iv": 1e-4, "ia": -1e-6}])
def test_kalman_c_vs_numpy_transliteration(kw):
    """The C oracle's StepKalman4D (wavespec_oracle.c) against the independent numpy transliteration
    (oracle.numpy_kalman_trend, same expression order as kalman-fast.mq5:2031-2125): identical bits
    for the defaults and four other parameter sets, over windows of every shape the tests use."""
    names = ["follow", "qp", "qv", "qa", "qj", "adapt", "r", "vp", "vv", "va", "vj", "iv", "ia", "ij", "clip", "ema"]
    kp = list(oracle.KALMAN_DEFAULTS)
    for k, v in kw.items():
        kp[names.index(k)] = v
    n, w = 1024, 6
    s = synth.random_walk(n * w, seed=77)
    s[2000] += 0.05  # a jump that trips the innovation clip and the adaptive boost
    X = s.reshape(w, n)
    got = oracle.numpy_kalman_trend(X, kp)
    kpa = np.asarray(kp, dtype=np.float64)
    for i in range(w):
        t = np.empty(n)
        x = np.ascontiguousarray(X[i])
        oracle.lib().ora_kalman_trend(oracle._p(x), n, oracle._p(kpa), oracle._p(t))
        assert np.array_equal(t, got[i]), (kw, i)


@pytest.mark.parametrize("n", [64, 1024])
def test_kalman_spectrum_vs_numpy(n):
    x = synth.random_walk(n, seed=n)
    p = oracle.window_spectrum(x, "kalman", "hann", 0, kalman=oracle.KALMAN_DEFAULTS)
    ref = oracle.numpy_spectrum(x, "kalman", "hann", 0, kalman=oracle.KALMAN_DEFAULTS)
    assert oracle.rel_err(p, ref) < 1e-10


def test_batch_matches_single_windows():
    s = synth.random_walk(5000, 9)
    b = oracle.batch_spectrum(s, 512, 300, "iir", "hann", 200)
    for w in (0, 7, b.shape[0] - 1):
        assert np.array_equal(b[w], oracle.window_spectrum(s[w * 300: w * 300 + 512], "iir", "hann", 200))


@pytest.mark.parametrize("path", GOLDEN, ids=[p.stem for p in GOLDEN])
def test_golden_vectors(path):
    g = np.load(path, allow_pickle=False)
    args = (g["series"], int(g["n"]), int(g["hop"]), str(g["detrend"]), str(g["window"]), int(g["trend_period"]))
    p = oracle.batch_spectrum(*args, kalman=g["kalman"])
    assert np.array_equal(p, g["power"])
    q = oracle.batch_spectrum(*args, kalman=g["kalman"], output="packed")
    assert np.array_equal(q, g["packed"])


# ---------------------------------------------------------------- top-k, inverse, phase
def test_topk_bins_vs_numpy_sort():
    """ora_topk_bins' insertion scan == a stable sort by (power desc, bin asc) over the period range."""
    n, k = 1024, 8
    s = synth.random_walk(30 * n, 21)
    got = oracle.batch_topk(s, n, n, "none", "hann", 0, None, k, 18.0, 200.0)
    P = oracle.batch_spectrum(s, n, n, "none", "hann")
    lo, hi = int(np.ceil(n / 200.0)), min(int(np.floor(n / 18.0)), n // 2 - 1)
    for w in range(P.shape[0]):
        bins = np.arange(lo, hi + 1)
        order = bins[np.lexsort((bins, -P[w, lo:hi + 1]))][:k]
        assert np.array_equal(got[w, :, 0].astype(int), order)
        assert np.array_equal(got[w, :, 1], P[w, order])


@pytest.mark.parametrize("n", [32, 64, 512, 4096])
def test_inverse_vs_numpy_irfft(n):
    rng = np.random.default_rng(n)
    packed = rng.standard_normal(n)
    x = oracle.fft_real_inverse(packed)
    X = np.zeros(n // 2 + 1, complex)
    X[: n // 2] = packed[0::2] + 1j * packed[1::2]
    X[0] = packed[0]  # in[1] ignored, Nyquist 0 (build-defined contract, wavespec_oracle.c)
    assert np.max(np.abs(x - np.fft.irfft(X, n))) <= 1e-13 * max(1.0, np.max(np.abs(x))) * np.log2(n)


@pytest.mark.parametrize("n", [32, 1024, 4096])
def test_inverse_round_trip(n):
    """inverse(forward(x)) == x for x without a Nyquist component."""
    x = synth.random_walk(n, n + 5)
    alt = (-1.0) ** np.arange(n)
    x = x - alt * (x @ alt) / n
    back = oracle.fft_real_inverse(oracle.window_spectrum(x, "none", "none", output="packed"))
    assert np.max(np.abs(back - x)) <= 1e-13 * np.max(np.abs(x)) * np.log2(n)


@pytest.mark.parametrize("n", [4, 64, 1024, 4096])
def test_phase_unwrap_vs_numpy(n):
    """CalculateFFTPhase/UnwrapPhase/CalculateGroupDelay == numpy angle/unwrap/gradient on the
    reference's n = N arrays (upper half zero)."""
    x = synth.random_walk(n, n + 1)
    # detrend "none": a mean-removed window's X_0 is rounding noise with an arbitrary phase
    packed = oracle.window_spectrum(x, "none", "hann", output="packed")
    ph, u, gd = oracle.phase_unwrap(packed)
    X = packed[0::2] + 1j * packed[1::2]
    full = np.concatenate([np.angle(X), np.zeros(n - n // 2)])
    uf = np.unwrap(full)
    gf = np.clip(-np.gradient(uf), -100.0, 100.0)
    assert np.max(np.abs(ph - full[: n // 2])) <= 1e-15  # libm atan2 vs numpy's: last-ulp
    assert np.max(np.abs(u - uf[: n // 2])) <= 1e-10
    assert np.max(np.abs(gd - gf[: n // 2])) <= 1e-10


def test_batch_phase_and_topk_phase_consistent():
    n, hop = 512, 100
    s = synth.random_walk(20 * hop + n, 4)
    ph = oracle.batch_phase(s, n, hop, "iir", "hann", 300)
    tk = oracle.batch_topk_phase(s, n, hop, "iir", "hann", 300, None, 5, 9.0, 200.0)
    tk4 = oracle.batch_topk(s, n, hop, "iir", "hann", 300, None, 5, 9.0, 200.0)
    assert np.array_equal(tk[:, :, :4], tk4)
    assert np.array_equal(ph[:, 0], oracle.batch_spectrum(s, n, hop, "iir", "hann", 300))
    for w in range(ph.shape[0]):
        packed = oracle.window_spectrum(s[w * hop: w * hop + n], "iir", "hann", 300, output="packed")
        _, u, gd = oracle.phase_unwrap(packed)
        assert np.array_equal(ph[w, 1], u) and np.array_equal(ph[w, 2], gd)
        b = tk[w, :, 0].astype(int)
        assert np.array_equal(tk[w, :, 4], u[b]) and np.array_equal(tk[w, :, 5], gd[b])
