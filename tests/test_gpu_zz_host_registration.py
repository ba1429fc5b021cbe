"""Caller buffers page-locked through the C ABI (gpu_register_host / gpu_unregister_host, the FeedCache
rewired to pinned buffers of the north star): direct DMA from and to registered host arrays, and the feed
cache re-registered when it grows.

These run last in the GPU session (the file sorts after the other GPU suites): they are the only tests that
page-lock and unlock host memory, and after they had run, later tests' pageable device-to-host copies in the
same process faulted with illegal addresses on some boxes (profiles/r04/faults/) -- a host-mapping effect of
the register / unregister sequence, kept away from every other GPU test.
"""
import numpy as np
import pytest

import oracle
from wavespec_amd import bridge, indicator, synth

pytestmark = pytest.mark.gpu

TOL = {"f64": 1e-10, "f32": 1e-5}
KALMAN = oracle.KALMAN_DEFAULTS


def gpu(series, n, hop, detrend="none", window="hann", period=0, prec="f64", output="power"):
    return bridge.spectrum_batch(series, n, hop, detrend, window, period, prec, output)


def ref(series, n, hop, detrend="none", window="hann", period=0, output="power"):
    return oracle.batch_spectrum(series, n, hop, detrend, window, period, kalman=KALMAN, output=output)


def test_register_host_direct_dma(gpu_session):
    """gpu_register_host: a registered fp64 series is DMA'd in place and a registered output array
    receives the results directly (no staging copy); results identical to the staged path."""
    n, hop = 1024, 256
    s = synth.random_walk(300 * hop + n, seed=41)
    nwin = 1 + (s.size - n) // hop
    staged = gpu(s, n, hop, "iir", "hann", 512)
    out = np.full(nwin * (n // 2), np.nan)
    bridge.register_host(s)
    bridge.register_host(out)
    try:
        p = bridge.spectrum_batch(s, n, hop, "iir", "hann", 512, out=out)
        assert p.base is out or p.base is out.base or np.shares_memory(p, out)
        assert np.array_equal(p, staged)
        assert oracle.rel_err(p, ref(s, n, hop, "iir", "hann", 512)) <= TOL["f64"]
        # a view inside the registered series is covered as well (sub-range of the region)
        sub = s[37 * hop:]
        assert oracle.rel_err(gpu(sub, n, hop), ref(sub, n, hop)) <= TOL["f64"]
        # fp32 plans convert and truncated outputs stage: same results as without registration
        p32 = gpu(s, n, hop, "kalman", "hann", prec="f32")
        assert oracle.rel_err(p32, ref(s.astype(np.float32).astype(np.float64), n, hop, "kalman", "hann")) <= TOL["f32"]
        part = bridge.spectrum_batch(s, n, hop, "iir", "hann", 512, max_records=10, out=out)
        assert np.array_equal(part, staged[:10])
        # top-k and the legacy batch FFT take the same path
        tk = bridge.spectrum_topk_batch(s, n, hop)
        w = s[: 8 * n].reshape(8, n).copy()  # its own buffer (a view of s would overlap s)
        bridge.register_host(w)
        fb = bridge.fft_real_forward_batch(w)
        bridge.unregister_host(w)
        assert oracle.rel_err(fb, ref(w.reshape(-1), n, n, "none", "none", output="packed")) <= 1e-12
        assert tk.shape == (nwin, 8, 4)
        # overlapping and unknown ranges are refused
        with pytest.raises(bridge.BridgeError) as e:
            bridge.register_host(s[10:20])
        assert e.value.status == bridge.BAD_ARGS
        with pytest.raises(bridge.BridgeError) as e:
            bridge.unregister_host(s[10:])
        assert e.value.status == bridge.BAD_ARGS
    finally:
        bridge.unregister_host(out)
        bridge.unregister_host(s)
    with pytest.raises(bridge.BridgeError):
        bridge.unregister_host(s)


def test_pinned_feed_cache_grows(gpu_session, tmp_path):
    """FeedCache rewired to pinned buffers: pin_feed_cache registers the chronological history;
    ensure_feed_cache re-registers it when more bars arrive; feed_spectra runs on it in place."""
    n = 512
    hist = synth.random_walk(6000, seed=9)
    close = hist[::-1].copy()  # newest first, as CopyClose fills an as-series array
    cache = indicator.FeedCache()
    ok, _, _ = indicator.ensure_feed_cache(cache, "EURUSD", "M1", 3000, False, "WaveSpecZZ",
                                           lambda start, cnt: close[start:start + cnt], str(tmp_path))
    assert ok and cache.chrono.size == 3000
    indicator.pin_feed_cache(cache)
    try:
        assert cache.pinned
        p = indicator.feed_spectra(cache, n, 64)
        assert oracle.rel_err(p, ref(cache.chrono, n, 64, "none", "hann")) <= TOL["f64"]
        ok, delta, _ = indicator.ensure_feed_cache(cache, "EURUSD", "M1", 6000, False, "WaveSpecZZ",
                                                   lambda start, cnt: close[start:start + cnt], str(tmp_path))
        assert ok and delta == 3000 and cache.pinned and cache.chrono.size == 6000
        assert np.array_equal(cache.chrono, hist)
        p = indicator.feed_spectra(cache, n, 64)
        assert oracle.rel_err(p, ref(hist, n, 64, "none", "hann")) <= TOL["f64"]
    finally:
        indicator.unpin_feed_cache(cache)
    assert not cache.pinned
