"""Precision of a SEQUENTIAL fp32 Kalman filter on the data of
tests/test_gpu_parity.py::test_kalman_f32_segments_fallback: oracle.numpy_kalman_trend run in
float32 (state centred on the window's first sample, as the device filter), spectra against the
fp64 filter.  CPU only; documents why the jump cases are bounded by the fp32 filter's own error.
  python3 scripts/kalman_f32_emulation.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "fft-wavespec_amd")]
import oracle  # noqa: E402
from wavespec_amd import synth  # noqa: E402


def f32_filter_err(s32, n):
    """rel_err / inband_err of the float32-emulated sequential filter's spectra vs the fp64 filter's."""
    X = s32.reshape(-1, n)
    Xc = X - X[:, :1]
    d64 = Xc - oracle.numpy_kalman_trend(Xc)
    x32 = Xc.astype(np.float32)
    d32 = (x32 - oracle.numpy_kalman_trend(x32, dtype=np.float32)).astype(np.float64)
    w = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n) / (n - 1))
    P64 = np.abs(np.fft.fft(d64 * w, axis=1)[:, :n // 2]) ** 2
    P32 = np.abs(np.fft.fft(d32 * w, axis=1)[:, :n // 2]) ** 2
    return oracle.rel_err(P32, P64), oracle.inband_err(P32, P64, *oracle.band(n))


if __name__ == "__main__":
    n, wu = 4096, 256
    S = (n + 3 * wu) // 4 - wu
    for kind, k, at in [("jump", 2, 0), ("jump", 1, 200), ("spike", 2, 0), ("none", 0, 0)]:
        s = synth.random_walk(64 * n, seed=17)
        for w in range(0, 64, 3):
            i = w * n + k * S + at
            if kind == "spike":
                s[i] += 1000.0
            elif kind == "jump":
                s[i:(w + 1) * n] += 0.5
        print(kind, k, at, "emulated sequential fp32: rel_err %.3e inband %.3e" % f32_filter_err(s.astype(np.float32).astype(np.float64), n))
