"""CPU model of the seeded sliding DFT (csrc/sliding_dft.hip) against the oracle.

The kernel computes hop = 1 spectra by sliding three (Hann / Hamming) or five (Blackman) trackers
per bin instead of an FFT per window.  This numpy restatement uses the same
decomposition, the same seeds (complex FFTs of the modulated first window), the same per-step
uniforms and the same closed-form H_k as the host tables in mtbridge.cpp, so the identity, its
signs and indices, and the rounding growth over a 512-window segment are checked on the CPU
against the oracle (the reference's FourierTransformManual path, L/WaveSpecZZ_1.0.2.mq5:884-974).
"""
import numpy as np
import pytest

import oracle
from wavespec_amd import synth

COEF = {"none": (1.0, 0.0, 0.0), "hann": (0.5, -0.5, 0.0), "hamming": (0.54, -0.46, 0.0),
        "blackman": (0.42, -0.5, 0.08)}


def slide_tables(n, window):
    a0, a1, a2 = COEF[window]
    nf = 1 if a1 == 0 and a2 == 0 else (3 if a2 == 0 else 5)
    mf = np.array([0, 1, -1, 2, -2][:nf])
    sc = np.array([a0, a1 / 2, a1 / 2, a2 / 2, a2 / 2][:nf])
    k = np.arange(n // 2)
    f = k[None, :] / n + mf[:, None] / (n - 1)
    omega = np.exp(2j * np.pi * f)
    # H_k by the closed form of the host table
    with np.errstate(divide="ignore", invalid="ignore"):
        num = np.where((k[None, :] + mf[:, None]) % 2 == 1, -1.0, 1.0) * np.sin(np.pi * mf[:, None] / (n - 1))
        g = num / np.sin(np.pi * f) * np.exp(-1j * np.pi * (k[None, :] * (n - 1) / n + mf[:, None]))
    g[0, 0] = n
    h = (sc[:, None] * g).sum(axis=0)
    return nf, sc, omega, h


def slide_model(series, n, window, detrend, seg):
    """Power rows of every hop = 1 window, segment by segment as the kernel runs them."""
    nf, sc, omega, h = slide_tables(n, window)
    m2, nw = n // 2, series.size - n + 1
    th = 2 * np.pi / (n - 1)
    out = np.empty((nw, m2))
    i = np.arange(n)
    for w0 in range(0, nw, seg):
        ln = min(seg, nw - w0)
        lvl = series[w0] if detrend == "mean" else 0.0  # the kernel centres the mean path
        x = series[w0:w0 + n] - lvl
        tr = np.empty((nf, m2), complex)
        tr[0] = sc[0] * np.fft.fft(x)[:m2]
        for m in range(1, (nf - 1) // 2 + 1):
            y = np.fft.fft(x * np.exp(-1j * m * th * i))
            tr[2 * m - 1] = sc[2 * m - 1] * y[:m2]
            tr[2 * m] = sc[2 * m] * np.conj(y[(n - np.arange(m2)) % n])
        s = x.sum()
        for st in range(ln):
            X = tr.sum(axis=0)
            if detrend == "mean":
                X = X - (s / n) * h
            out[w0 + st] = X.real ** 2 + X.imag ** 2
            if st + 1 < ln:
                xw, xn = series[w0 + st] - lvl, series[w0 + st + n] - lvl
                u = np.empty(nf, complex)
                u[0] = sc[0] * (xn - xw)
                for m in range(1, (nf - 1) // 2 + 1):
                    ur = sc[2 * m - 1] * (xn * np.cos(m * th) - xw)
                    ui = -(sc[2 * m - 1] * (xn * np.sin(m * th)))
                    u[2 * m - 1], u[2 * m] = ur + 1j * ui, ur - 1j * ui
                tr = omega * (tr + u[:, None])
                s += xn - xw
    return out


@pytest.mark.parametrize("window", ["none", "hann", "hamming", "blackman"])
@pytest.mark.parametrize("detrend", ["none", "mean"])
def test_slide_model_matches_oracle(window, detrend):
    n, seg = 512, 512
    s = synth.random_walk(2 * seg + 37 + n - 1, seed=21)
    got = slide_model(s, n, window, detrend, seg)
    want = oracle.batch_spectrum(s, n, 1, detrend, window)
    assert got.shape == want.shape
    kmin, kmax = oracle.band(n)
    # the bar is 1e-10; the model sits at <= 3e-12 (centred mean) and <= 1e-14 (no detrend)
    assert oracle.rel_err(got, want) <= 1e-11
    assert oracle.inband_err(got, want, kmin, kmax) <= 1e-11


def test_slide_model_window_dft_closed_form():
    """H_k of the host table = the DFT of the window the oracle applies."""
    for n in (512, 2048, 8192):
        for window in ("hann", "hamming", "blackman", "none"):
            _, _, _, h = slide_tables(n, window)
            ones = np.ones(n)
            # DFT of the window = packed FFT of the windowed constant 1 (detrend none)
            re, im = oracle.fft_manual(np.asarray(_window(n, window)) * ones)
            ref = re[: n // 2] + 1j * im[: n // 2]
            assert np.max(np.abs(h - ref)) <= 1e-9 * max(1.0, np.max(np.abs(ref))), (n, window)


def _window(n, window):
    a0, a1, a2 = COEF[window]
    i = np.arange(n)
    return a0 + a1 * np.cos(2 * np.pi * i / (n - 1)) + a2 * np.cos(4 * np.pi * i / (n - 1))


def test_slide_model_level_shift_stress():
    """Prices far from zero (level 100) with a jump: the seeds and the slide carry the level."""
    n, seg = 1024, 512
    s = 100.0 + synth.random_walk(seg + 300 + n - 1, seed=5) - 1.1
    s[700:] += 0.5
    got = slide_model(s, n, "hann", "none", seg)
    want = oracle.batch_spectrum(s, n, 1, "none", "hann")
    kmin, kmax = oracle.band(n)
    assert oracle.rel_err(got, want) <= 1e-10
    assert oracle.inband_err(got, want, kmin, kmax) <= 1e-10


def _hi(p):
    """The IEEE high word of non-negative doubles, as the kernel compares powers (orders like the value)."""
    return (np.ascontiguousarray(p, dtype=np.float64).view(np.uint64) >> np.uint64(32)).astype(np.int64)


@pytest.mark.parametrize("n,wb,k,pmin,pmax", [(2048, 16, 8, 18.0, 200.0), (1024, 32, 8, 5.0, 200.0),
                                             (4096, 16, 3, 18.0, 200.0), (2048, 16, 8, 2.0, 10.0)])
def test_probe_threshold_candidates_superset(n, wb, k, pmin, pmax):
    """The probe-threshold scan of the hop = 1 top-k kernel (sliding_core.h slide_topk_p_kernel) restated on
    the oracle's band powers: in window w the probes are the k bins that won window w - WB, tau is their
    smallest power in window w (k distinct bins of this window, so tau <= its k-th largest power), and the
    candidates are the bins whose high word is >= hi(tau) - 1.  Every member of the window's top k -- ties at
    the k-th included -- must be a candidate, and the reference's insertion over the candidates alone
    (ascending bins, strict '>') must give the full scan's records.  Also reports how many candidates a window
    has (the kernel's list holds 16; a window with more takes the exact scan)."""
    nwin = 1500
    s = synth.random_walk(nwin + n - 1, seed=n + wb)
    spec = oracle.batch_spectrum(s, n, 1, "none", "hann")
    kmin, kmax = int(np.ceil(n / pmax)), min(int(np.floor(n / pmin)), n // 2 - 1)
    band = spec[:, kmin:kmax + 1]
    counts = []
    for w in range(wb, nwin):
        prev = band[w - wb]
        probes = np.lexsort((np.arange(prev.size), -prev))[:k]  # winners of the slot's previous window
        tau_hi = _hi(band[w, probes]).min()
        cand = np.nonzero(_hi(band[w]) >= tau_hi - 1)[0]
        counts.append(cand.size)
        order = np.lexsort((np.arange(band[w].size), -band[w]))
        kth = band[w, order[k - 1]]
        assert set(np.nonzero(band[w] >= kth)[0]) <= set(cand), w  # ties at the k-th included
        # the insertion over the candidates only (ascending bins, strict '>') = the full scan's top k
        top = []
        for j in cand:
            p = band[w, j]
            pos = next((i for i, (tp, _) in enumerate(top) if p > tp), len(top))
            top.insert(pos, (p, j))
            del top[k:]
        assert [j for _, j in top] == list(order[:k]), w
    counts = np.array(counts)
    assert np.median(counts) <= 16  # the list's capacity holds the typical window (the rest: exact scan)
