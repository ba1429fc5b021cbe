"""Host-side mirror of the WaveSpecZZ indicator surface around the hot path.

Same names, argument meaning and error behaviour as the MQL5 code that calls
``mt-bridge.dll``; the arithmetic happens in libmtbridge.so (HIP, gfx950).

* :class:`FeedCache` / :func:`ensure_feed_cache` -- Include/FeedCache.mqh:20-115
  (file format: int32 count + doubles, newest first); :func:`pin_feed_cache`
  registers the history with the session (gpu_register_host) across growth; the
  batch path stages it through the library's pinned buffers for hipMemcpyAsync
  -- the north star's "FeedCache rewired to pinned buffers".
* :class:`FeedBuilder` -- FeedBuilder::Build / BuildPlaPriceSeries (1.1.0:474-506, 760-771).
* :class:`FftProcessor` -- EnsureGpu + FftProcessor::Run (1.1.0:511-533, 722-757).
* :func:`on_calculate` -- the per-bar OnCalculate loop restricted to the
  spectrum path (1.1.0:1133-1249).
* :func:`batch_spectra` -- the batch-warmup / WaveCyclesBatchFetcher driver
  shape (1.1.0:997-1040, WaveCyclesBatchFetcher.mq5:91-143) on the spectrum
  batch API.
"""
from __future__ import annotations

import os
import struct
import time
from dataclasses import dataclass, field

import numpy as np

from . import bridge

ALGLIB_STATUS_OK = 0        # 1.1.0:15
ALGLIB_STATUS_NOT_READY = -5  # 1.1.0:16


def feed_cache_file_name(prefix: str, symbol: str, tf: str) -> str:
    """FeedCacheFileName, Include/FeedCache.mqh:30-33."""
    return f"{prefix}_cache_{symbol}_{tf}.bin"


@dataclass
class FeedCache:
    """struct FeedCache, Include/FeedCache.mqh:20-27 (close[] newest first, :12, :69).

    ``chrono`` is the same history oldest first in one contiguous float64 buffer: the physical
    memory of the MQL as-series close[] array, which is what the terminal hands the DLL.  Once
    :func:`pin_feed_cache` has registered it, ``pinned`` is True and ensure_feed_cache keeps the
    registration on the current buffer as the history grows."""
    symbol: str = ""
    tf: str = ""
    close: np.ndarray = field(default_factory=lambda: np.empty(0))
    loaded: bool = False
    from_file: bool = False
    chrono: np.ndarray = field(default_factory=lambda: np.empty(0))
    pinned: bool = False
    pinned_session: int = 0  # gpu_session_id of the session holding the registration


def save_feed_cache(path: str, close_newest_first: np.ndarray) -> None:
    """FileWriteInteger(count) + FileWriteArray(close) (FeedCache.mqh:102-111)."""
    a = np.ascontiguousarray(close_newest_first, dtype="<f8")
    with open(path, "wb") as f:
        f.write(struct.pack("<i", a.size))
        f.write(a.tobytes())


def load_feed_cache(path: str) -> np.ndarray | None:
    """FileReadInteger + FileReadArray (FeedCache.mqh:49-67)."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        head = f.read(4)
        if len(head) < 4:
            return None
        cnt = struct.unpack("<i", head)[0]
        if cnt <= 0:
            return None
        return np.frombuffer(f.read(8 * cnt), dtype="<f8", count=cnt).copy()


def ensure_feed_cache(cache: FeedCache, symbol: str, tf: str, needed_bars: int, enable_cache: bool, prefix: str,
                      copy_close, cache_dir: str = ".") -> tuple[bool, int, bool]:
    """EnsureFeedCache (FeedCache.mqh:36-115).

    ``copy_close(start, count)`` plays CopyClose(symbol, tf, start, count): it
    returns up to ``count`` closes newest-first starting ``start`` bars back.
    Returns (ok, delta_added, from_file) like the MQL out-parameters.
    """
    delta_added, from_file = 0, False
    path = os.path.join(cache_dir, feed_cache_file_name(prefix, symbol, tf))
    if enable_cache and not cache.loaded:
        data = load_feed_cache(path)
        if data is not None:
            cache.close, cache.symbol, cache.tf = data, symbol, tf
            cache.loaded = cache.from_file = from_file = True
    if not (cache.symbol == symbol and cache.tf == tf):
        cache.close = np.empty(0)
    cached = cache.close.size
    max_chunk = 100000  # :80
    parts = [cache.close]
    while cached < needed_bars:
        want = min(max_chunk, needed_bars - cached)
        got = np.asarray(copy_close(cached, want), dtype=np.float64)
        if got.size <= 0:
            break
        parts.append(got)
        cached += got.size
        delta_added += got.size
    cache.close = np.concatenate(parts) if len(parts) > 1 else cache.close
    cache.symbol, cache.tf = symbol, tf
    cache.loaded = cached > 0
    if enable_cache and cache.loaded:
        save_feed_cache(path, cache.close)
    if cache.chrono.size != cache.close.size or (cache.close.size and cache.chrono[-1] != cache.close[0]):
        _restage(cache)
    return cached >= needed_bars, delta_added, from_file


def _restage(cache: FeedCache) -> None:
    """Rebuild the chronological buffer after the history changed (ArrayResize in MQL moves the
    array: the old registration is dropped and the new buffer registered)."""
    was = cache.pinned
    if was:
        unpin_feed_cache(cache)
    cache.chrono = np.ascontiguousarray(cache.close[::-1], dtype=np.float64)
    if was:
        try:
            pin_feed_cache(cache)
        except bridge.BridgeError as e:  # the session is gone (last gpu_shutdown): stay unpinned
            if e.status != bridge.BACKEND_UNAVAILABLE:
                raise


def pin_feed_cache(cache: FeedCache) -> None:
    """Register the feed history with the session (gpu_register_host, needs an open session); batch
    calls on ``cache.chrono`` stage it through the library's pinned buffers (include/mtbridge.h,
    "Pinned feed staging"; round 6: caller memory is never page-locked).  The session that holds
    the registration is remembered (gpu_session_id)."""
    if cache.chrono.size != cache.close.size:
        cache.chrono = np.ascontiguousarray(cache.close[::-1], dtype=np.float64)
    if cache.chrono.size and not cache.pinned:
        bridge.register_host(cache.chrono)
        cache.pinned = True
        cache.pinned_session = bridge.session_id()


def unpin_feed_cache(cache: FeedCache) -> None:
    """gpu_unregister_host of the pinned history.  A registration belongs to the session that made it:
    once the last gpu_shutdown has torn that session down (FftProcessor.shutdown in on_calculate may be
    that call) its registrations went with it, so there is nothing to undo -- the session id tells.
    Under the same session every failure is raised."""
    if not cache.pinned:
        return
    if bridge.session_id() != cache.pinned_session:
        cache.pinned = False  # the session that held it is gone: its registrations went with it
        return
    bridge.unregister_host(cache.chrono)
    cache.pinned = False


class FeedBuilder:
    """FEED_PLA / FEED_CLOSE window gather (1.1.0:485-496, 760-771)."""

    def __init__(self, fft_window: int):
        self.fft_window = fft_window
        self.feed_data = np.empty(fft_window)

    def build(self, cache: FeedCache, shift_end_feed: int) -> bool:
        n = self.fft_window
        if shift_end_feed < 0 or cache.close.size < shift_end_feed + n:
            return False
        # feed_data[j] = close[shift_end_feed + (N-1-j)]: chronological window
        self.feed_data[:] = cache.close[shift_end_feed:shift_end_feed + n][::-1]
        return True


class FftProcessor:
    """EnsureGpu (1.1.0:722-757) + FftProcessor::Run (1.1.0:518-531)."""

    def __init__(self, gpu_streams: int = 64):
        self.session = False
        self.streams = max(16, min(512, gpu_streams))  # 1.1.0:729
        self.init_fail_counter = 0
        self.g_fft_interleaved = np.empty(0)
        self.fft_real = np.empty(0)
        self.fft_imag = np.empty(0)
        self.spectrum = np.empty(0)
        self.last_error = ""

    def ensure(self, length: int) -> bool:
        if length <= 0:
            return False
        if self.session and length == self.g_fft_interleaved.size:
            return True
        if not self.session:
            st = bridge.lib().gpu_init(0, self.streams)
            if st != ALGLIB_STATUS_OK:
                self.init_fail_counter += 1
                self.last_error = bridge.last_error()
                return False
            self.init_fail_counter = 0
            self.session = True
        self.g_fft_interleaved = np.empty(length)
        self.fft_real = np.empty(length)
        self.fft_imag = np.empty(length)
        self.spectrum = np.empty(length // 2)
        return True

    def run(self, data: np.ndarray, length: int) -> bool:
        try:
            self.g_fft_interleaved = bridge.fft_real_forward(np.asarray(data[:length], dtype=np.float64))
        except bridge.BridgeError as e:
            self.last_error = e.reason
            return False
        bins = length // 2
        base = 2 * np.arange(bins)
        self.fft_real[:bins] = self.g_fft_interleaved[base]
        self.fft_imag[:bins] = np.where(base + 1 < length, self.g_fft_interleaved[np.minimum(base + 1, length - 1)],
                                        0.0)
        self.spectrum[:] = self.fft_real[:bins] ** 2 + self.fft_imag[:bins] ** 2
        return True

    def shutdown(self) -> None:
        if self.session:
            bridge.shutdown()
            self.session = False


def on_calculate(cache: FeedCache, fft_window: int, bars: int, fft: FftProcessor | None = None) -> np.ndarray:
    """Per-bar loop of OnCalculate limited to the spectrum path (1.1.0:1180-1249).

    Bars are visited oldest first; bar b ends at feed shift ``bars-1-b``.
    Returns the (bars, N/2) spectra.  Bars whose GPU call fails are skipped
    with NaN rows, as the reference skips them with ``continue`` (1.1.0:1246-1249).
    """
    own = fft is None  # a processor made here lives for this call: OnInit .. OnDeinit of one chart
    fft = fft or FftProcessor()
    feed = FeedBuilder(fft_window)
    out = np.full((bars, fft_window // 2), np.nan)
    try:
        for b in range(bars):
            if not feed.build(cache, bars - 1 - b):
                continue
            detrended = feed.feed_data.copy()  # 1.1.0:1239, "windowing: none"
            if not fft.ensure(fft_window):
                continue
            if not fft.run(detrended, fft_window):
                continue
            out[b] = fft.spectrum
    finally:
        if own:
            fft.shutdown()  # OnDeinit (1.1.0:710-716): drops this chart's reference on the session
    return out


def feed_spectra(cache: FeedCache, fft_window: int, hop: int = 1, detrend="none", window="hann",
                 trend_period: int = 0, out: np.ndarray | None = None) -> np.ndarray:
    """Synchronous spectra of every window of the feed history (gpu_spectrum_batch on
    ``cache.chrono``): with the cache pinned and ``out`` registered, the input and the results
    cross PCIe by DMA only (fp64)."""
    return bridge.spectrum_batch(cache.chrono, fft_window, hop, detrend, window, trend_period, "f64", "power",
                                 out=out)


def batch_spectra(prices: np.ndarray, fft_window: int, hop: int = 1, detrend="none", window="hann",
                  trend_period: int = 0, precision="f64", wait_ms: int = 120000, poll_ms: int = 5) -> np.ndarray:
    """Batch warmup driver (1.1.0:1014-1040) on the spectrum batch API.

    ``prices`` is chronological (physical memory of an as-series CopyClose).
    Submits once, polls try_get with Sleep(poll_ms) until ready or
    ``wait_ms`` (InpBatchWaitMs, 1.1.0:69), always frees the job.
    """
    got = prices.size
    if got < fft_window:
        raise ValueError("need at least one window of prices")
    nwin = 1 + (got - fft_window) // hop  # 1.1.0:1016
    jid = bridge.submit_spectrum_batch(prices, fft_window, hop, detrend, window, trend_period, precision)
    out = np.empty((nwin, fft_window // 2))
    start = time.monotonic()
    try:
        while True:
            st, ready, out_len = bridge.try_get_spectrum_batch(jid, out)
            if st == ALGLIB_STATUS_OK and ready == 1:
                break
            if st not in (ALGLIB_STATUS_OK, ALGLIB_STATUS_NOT_READY):
                raise bridge.BridgeError("gpu_try_get_spectrum_batch", st, bridge.last_error())
            if wait_ms > 0 and (time.monotonic() - start) * 1000 >= wait_ms:
                raise TimeoutError("batch spectrum job timed out")
            time.sleep(poll_ms / 1000)
    finally:
        bridge.free_job(jid)
    return out[:out_len]
