"""Precision of fp32 Kalman filters on level-jump data (CPU only).

Emulates the device's fp32 filter (two-stage predict, normalised update, kalman_core.h kstep_pk2)
in numpy float32 with two centring policies:
  x0    state centred on the window's first sample (rounds 1-2)
  tile  re-centred on a sample every J = 16 steps (round 3, the device default: kalman_core.h kRecentre)
and prints the spectrum error of each against the fp64 oracle filter (oracle.numpy_kalman_trend).
A 0.5 level jump costs the x0 form 1.7e-5 - 3.8e-5; the tile form stays near 1e-6.
  python3 scripts/kalman_f32_emulation.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "fft-wavespec_amd")]
import oracle  # noqa: E402
from wavespec_amd import synth  # noqa: E402


def device_f32_filter(X32, mode="tile", J=16):
    """Detrended windows d = z - trend of the device-form fp32 filter (reference default flags)."""
    (follow, q_pos, q_vel, q_acc, q_jerk, adapt, R, vp, vv, va, vj, iv, ia, ij, clip, _ema) = oracle.KALMAN_DEFAULTS
    f = np.float32
    W, n = X32.shape
    qs = max(0.05, follow)
    Qp, Qv, Qa, Qj = [f(max(1e-9, q * qs)) for q in (q_pos, q_vel, q_acc, q_jerk)]
    Rr, ad, cl = f(max(1e-9, R)), f(adapt), f(clip)
    gQp, gQv, gQa, gQj = ad * Qp, ad * Qv, ad * Qa, ad * Qj
    base = X32[:, 0].copy()
    pos, vel, acc, jerk = np.zeros(W, f), np.full(W, f(iv)), np.full(W, f(ia)), np.full(W, f(ij))
    p00, p11, p22, p33 = np.full(W, f(vp)), np.full(W, f(vv)), np.full(W, f(va)), np.full(W, f(vj))
    p01 = p02 = p03 = p12 = p13 = p23 = np.zeros(W, f)
    d = np.empty((W, n), f)
    h, s6 = f(0.5), f(1 / 6)
    for t in range(n):
        if mode == "tile" and t % J == 0 and t > 0:
            nb = X32[:, t]
            pos = (pos + (base - nb)).astype(f)
            base = nb.copy()
        z = (X32[:, t] - base).astype(f)
        x0p, x1p, x2p, x3p = pos + vel + h * acc + s6 * jerk, vel + acc + h * jerk, acc + jerk, jerk
        a00, a01 = p00 + p01 + h * p02 + s6 * p03, p01 + p11 + h * p12 + s6 * p13
        a02, a03 = p02 + p12 + h * p22 + s6 * p23, p03 + p13 + h * p23 + s6 * p33
        a11, a12, a13 = p11 + p12 + h * p13, p12 + p22 + h * p23, p13 + p23 + h * p33
        a22, a23 = p22 + p23, p23 + p33
        P00, P01, P02, P03 = a00 + a01 + h * a02 + s6 * a03 + Qp, a01 + a02 + h * a03, a02 + a03, a03
        P11, P12, P13 = a11 + f(2) * a12 + h * (a13 + p13) + Qv, a12 + a13, a13
        P22, P23, P33 = a22 + a23 + Qa, a23, p33 + Qj
        y = z - x0p
        k = np.minimum(f(5), np.abs(y * (f(1) / np.sqrt(P00 + Rr)).astype(f)))
        P00, P11, P22, P33 = P00 + k * gQp, P11 + k * gQv, P22 + k * gQa, P33 + k * gQj
        rs = (f(1) / np.sqrt(P00 + Rr)).astype(f)
        yn = np.clip(y * rs, -cl, cl)
        g0, g1, g2, g3 = P00 * rs, P01 * rs, P02 * rs, P03 * rs
        pos, vel, acc, jerk = x0p + g0 * yn, x1p + g1 * yn, x2p + g2 * yn, x3p + g3 * yn
        p00, p01, p02, p03 = np.maximum(f(1e-12), P00 - g0 * g0), P01 - g1 * g0, P02 - g2 * g0, P03 - g3 * g0
        p11, p12, p13 = np.maximum(f(1e-12), P11 - g1 * g1), P12 - g2 * g1, P13 - g3 * g1
        p22, p23, p33 = np.maximum(f(1e-12), P22 - g2 * g2), P23 - g3 * g2, np.maximum(f(1e-12), P33 - g3 * g3)
        d[:, t] = z - pos
    return d.astype(np.float64)


def f32_filter_err(s32, n, mode="tile"):
    """rel_err / inband_err of the emulated fp32 filter's spectra vs the fp64 oracle filter's."""
    X = s32.reshape(-1, n)
    Xc = X - X[:, :1]
    d64 = Xc - oracle.numpy_kalman_trend(Xc)
    d32 = device_f32_filter(X.astype(np.float32), mode)
    w = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n) / (n - 1))
    P64 = np.abs(np.fft.fft(d64 * w, axis=1)[:, :n // 2]) ** 2
    P32 = np.abs(np.fft.fft(d32 * w, axis=1)[:, :n // 2]) ** 2
    return oracle.rel_err(P32, P64), oracle.inband_err(P32, P64, *oracle.band(n))


if __name__ == "__main__":
    n, wu = 4096, 256
    S = (n + 3 * wu) // 4 - wu
    for kind, k, at in [("jump", 2, 0), ("jump", 1, 200), ("spike", 2, 0), ("none", 0, 0)]:
        s = synth.random_walk(16 * n, seed=17)
        for w in range(0, 16, 3):
            i = w * n + k * S + at
            if kind == "spike":
                s[i] += 1000.0
            elif kind == "jump":
                s[i:(w + 1) * n] += 0.5
        s32 = s.astype(np.float32).astype(np.float64)
        for mode in ("x0", "tile"):
            print("%-5s k=%d at=%3d  %-4s rel_err %.3e inband %.3e" % ((kind, k, at, mode) + f32_filter_err(s32, n, mode)))
