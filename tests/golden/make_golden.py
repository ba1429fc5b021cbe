"""Generates tests/golden/*.npz -- small input/expected-output vectors.

Provenance: the reference ships no fixtures and cannot run here (MQL5 +
un-vendored mt-bridge.dll), so expected outputs come from the CPU
restatement oracle/wavespec_oracle.c (FourierTransformManual & co.), and
every vector is cross-checked here against numpy.fft (independent code)
before it is written.  Re-run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "fft-wavespec_amd"))

import oracle  # noqa: E402
from wavespec_amd import synth  # noqa: E402

OUT = Path(__file__).resolve().parent


def cases():
    # C1: single 1024-pt window, sine+noise, Hann, no detrend (BASELINE configs[0])
    x = synth.sine_noise_window(1024, 1234)
    yield "c1_n1024_hann", dict(series=x, n=1024, hop=1024, detrend="none", window="hann", trend_period=0)
    # the 1.1.0 live path: no detrend, no window
    yield "live_n1024_rect", dict(series=x, n=1024, hop=1024, detrend="none", window="none", trend_period=0)
    # small multi-window batches per detrend / window mode
    rw = synth.random_walk(64 * 7 + 256, seed=7)
    for n, hop in ((64, 64), (256, 37), (1024, 512)):
        s = synth.random_walk((6 - 1) * hop + n, seed=100 + n)
        for det, win, per in (("none", "hann", 0), ("mean", "hamming", 0), ("iir", "blackman", 1024),
                              ("iir", "hann", 50), ("none", "bartlett", 0), ("kalman", "hann", 0)):
            yield f"n{n}_hop{hop}_{det}{per or ''}_{win}", dict(series=s, n=n, hop=hop, detrend=det, window=win,
                                                                  trend_period=per)
    yield "n64_hop1_none_hann", dict(series=rw[:64 + 40], n=64, hop=1, detrend="none", window="hann", trend_period=0)


def main():
    for name, c in cases():
        s = c["series"]
        power = oracle.batch_spectrum(s, c["n"], c["hop"], c["detrend"], c["window"], c["trend_period"],
                                      kalman=oracle.KALMAN_DEFAULTS)
        packed = oracle.batch_spectrum(s, c["n"], c["hop"], c["detrend"], c["window"], c["trend_period"],
                                       kalman=oracle.KALMAN_DEFAULTS, output="packed")
        # independent numpy restatement (Kalman: oracle.numpy_kalman_trend, a second transliteration of
        # StepKalman4D) for every case
        nwin = power.shape[0]
        ref = np.stack([oracle.numpy_spectrum(s[w * c["hop"]: w * c["hop"] + c["n"]], c["detrend"], c["window"],
                                              c["trend_period"], kalman=oracle.KALMAN_DEFAULTS) for w in range(nwin)])
        err = oracle.rel_err(power, ref)
        assert err < 1e-10, (name, err)  # the parity bar; observed <= 3e-12
        np.savez_compressed(OUT / f"{name}.npz", series=s, n=c["n"], hop=c["hop"], detrend=c["detrend"],
                            window=c["window"], trend_period=c["trend_period"],
                            kalman=np.asarray(oracle.KALMAN_DEFAULTS), power=power, packed=packed)
        print(f"{name}: windows={power.shape[0]}")


if __name__ == "__main__":
    main()
