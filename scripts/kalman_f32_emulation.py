"""Precision of the SEQUENTIAL fp32 Kalman filter on the data of
tests/test_gpu_parity.py::test_kalman_f32_two_segments_fallback: oracle.numpy_kalman_trend
re-run in numpy float32 (state centred on the window's first sample, as the device filter),
spectra against the fp64 filter.  CPU only; documents why the jump cases carry a looser bar.
  python3 scripts/kalman_f32_emulation.py
"""
import sys, inspect, numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'fft-wavespec_amd')]
import oracle
from wavespec_amd import synth
src = inspect.getsource(oracle.numpy_kalman_trend)
src = src.replace('X = np.asarray(X, dtype=np.float64)', 'X = np.asarray(X, dtype=DT)')
src = src.replace('np.full(W, init_vel)', 'np.full(W, init_vel, dtype=DT)').replace('np.full(W, init_acc)', 'np.full(W, init_acc, dtype=DT)').replace('np.full(W, init_jerk)', 'np.full(W, init_jerk, dtype=DT)')
src = src.replace('np.zeros((W, 4, 4))', 'np.zeros((W, 4, 4), dtype=DT)').replace('np.zeros(W)', 'np.zeros(W, dtype=DT)').replace('np.empty((W, n))', 'np.empty((W, n), dtype=DT)')
src = src.replace('def numpy_kalman_trend(', 'def kal(DT, ')
ns = {'np': np, 'KALMAN_DEFAULTS': oracle.KALMAN_DEFAULTS}
exec(src, ns)
kal = ns['kal']
n, wu = 4096, 256; l0 = (n + wu)//2
def spec(d):
    i = np.arange(n); w = 0.5 - 0.5*np.cos(2*np.pi*i/(n-1))
    X = np.fft.fft(d*w, axis=1)[:, :n//2]
    return np.abs(X)**2
for kind, at in [('jump',0),('jump',200),('spike',0),('none',0)]:
    s = synth.random_walk(64 * n, seed=17)
    for w in range(0, 64, 3):
        i = w*n + l0 - wu + at
        if kind == 'spike': s[i] += 1000.0
        elif kind == 'jump': s[i:(w+1)*n] += 0.5
    s32 = s.astype(np.float32).astype(np.float64)
    X = s32.reshape(64, n)
    x0 = X[:, :1]
    t64 = kal(np.float64, X - x0)
    t32 = kal(np.float32, (X - x0).astype(np.float32)).astype(np.float64)
    d64 = (X - x0) - t64; d32 = ((X - x0).astype(np.float32) - t32.astype(np.float32)).astype(np.float64)
    P64, P32 = spec(d64), spec(d32)
    print(kind, at, 'emulated seq fp32 rel_err', oracle.rel_err(P32, P64), 'inband', oracle.inband_err(P32, P64, *oracle.band(n)))
