"""CPU tests of the host-side indicator logic (wavespec_amd/indicator.py) that need no device:
FeedCache growth (Include/FeedCache.mqh:36-115) and the pin / unpin lifecycle around a session
that was torn down between pin and growth (gpu_register_host registrations end with the session).
The bridge's register / unregister calls are replaced by a model of the library's registry."""
import numpy as np
import pytest

from wavespec_amd import bridge, indicator, synth


class FakeRegistry:
    """The library's HostRegistry semantics: registrations live in the session (gpu_session_id names it)."""

    def __init__(self):
        self.session = True
        self.sid = 1
        self.regions = set()
        self.refuse = False  # the runtime refuses to unregister (MTB_INTERNAL_ERROR, the buffer stays locked)

    def session_id(self):
        return self.sid if self.session else 0

    def reopen(self):  # gpu_init after the last gpu_shutdown: a new session
        self.session = True
        self.sid += 1

    def register(self, a):
        if not self.session:
            raise bridge.BridgeError("gpu_register_host", bridge.BACKEND_UNAVAILABLE, "no session")
        self.regions.add(a.ctypes.data)

    def unregister(self, a):
        if not self.session:
            raise bridge.BridgeError("gpu_unregister_host", bridge.BACKEND_UNAVAILABLE, "no session")
        if a.ctypes.data not in self.regions:
            raise bridge.BridgeError("gpu_unregister_host", bridge.BAD_ARGS, "not registered")
        if self.refuse:
            raise bridge.BridgeError("gpu_unregister_host", bridge.INTERNAL_ERROR, "still page-locked")
        self.regions.discard(a.ctypes.data)

    def teardown(self):  # last gpu_shutdown: ~HostRegistry unregisters everything
        self.session = False
        self.regions.clear()


@pytest.fixture
def reg(monkeypatch):
    r = FakeRegistry()
    monkeypatch.setattr(bridge, "register_host", r.register)
    monkeypatch.setattr(bridge, "unregister_host", r.unregister)
    monkeypatch.setattr(bridge, "session_id", r.session_id)
    return r


def _grow(cache, close, bars, tmp_path):
    return indicator.ensure_feed_cache(cache, "EURUSD", "M1", bars, False, "WaveSpecZZ",
                                       lambda start, cnt: close[start:start + cnt], str(tmp_path))


def test_pin_follows_growth(reg, tmp_path):
    close = synth.random_walk(5000, seed=3)[::-1].copy()
    cache = indicator.FeedCache()
    assert _grow(cache, close, 2000, tmp_path)[0]
    indicator.pin_feed_cache(cache)
    assert cache.pinned and reg.regions == {cache.chrono.ctypes.data}
    assert _grow(cache, close, 5000, tmp_path)[:2] == (True, 3000)
    assert cache.pinned and reg.regions == {cache.chrono.ctypes.data}  # the new buffer, the old one dropped
    assert np.array_equal(cache.chrono, close[::-1])
    indicator.unpin_feed_cache(cache)
    assert not cache.pinned and not reg.regions


def test_growth_after_session_teardown(reg, tmp_path):
    """the session ends between pin and growth; growing the history must neither raise nor
    leave a stale flag, and a new session lets it pin again."""
    close = synth.random_walk(5000, seed=4)[::-1].copy()
    cache = indicator.FeedCache()
    _grow(cache, close, 2000, tmp_path)
    indicator.pin_feed_cache(cache)
    reg.teardown()
    assert _grow(cache, close, 3000, tmp_path)[0]
    assert not cache.pinned and cache.chrono.size == 3000
    indicator.unpin_feed_cache(cache)  # nothing to undo
    reg.reopen()
    indicator.pin_feed_cache(cache)
    assert cache.pinned and cache.pinned_session == reg.sid


def test_unpin_after_new_session_clears_flag(reg, tmp_path):
    """A new session that never saw this buffer (gpu_shutdown + gpu_init between pin and unpin): the
    registration went with the old session, nothing is unregistered."""
    close = synth.random_walk(3000, seed=5)[::-1].copy()
    cache = indicator.FeedCache()
    _grow(cache, close, 3000, tmp_path)
    indicator.pin_feed_cache(cache)
    reg.teardown()
    reg.reopen()
    indicator.unpin_feed_cache(cache)
    assert not cache.pinned


def test_unpin_surfaces_failures(reg, tmp_path):
    """under the session that registered it, a failed unregistration is raised (it was
    swallowed before) and the cache stays marked pinned -- the buffer is still page-locked; an unknown
    buffer under the same session (BAD_ARGS) is raised too."""
    close = synth.random_walk(3000, seed=6)[::-1].copy()
    cache = indicator.FeedCache()
    _grow(cache, close, 3000, tmp_path)
    indicator.pin_feed_cache(cache)
    reg.refuse = True
    with pytest.raises(bridge.BridgeError) as e:
        indicator.unpin_feed_cache(cache)
    assert e.value.status == bridge.INTERNAL_ERROR and cache.pinned
    reg.refuse = False
    indicator.unpin_feed_cache(cache)
    assert not cache.pinned and not reg.regions
    indicator.pin_feed_cache(cache)
    reg.regions.clear()  # the library lost it under the same session: a bug, not a teardown
    with pytest.raises(bridge.BridgeError) as e:
        indicator.unpin_feed_cache(cache)
    assert e.value.status == bridge.BAD_ARGS


def test_feed_cache_file_round_trip(tmp_path):
    """int32 count + doubles, newest first (FeedCache.mqh:102-111 writes, :49-67 reads)."""
    close = synth.random_walk(1234, seed=6)[::-1].copy()
    p = tmp_path / indicator.feed_cache_file_name("WaveSpecZZ", "EURUSD", "M1")
    indicator.save_feed_cache(str(p), close)
    raw = p.read_bytes()
    assert int.from_bytes(raw[:4], "little") == close.size and len(raw) == 4 + 8 * close.size
    assert np.array_equal(indicator.load_feed_cache(str(p)), close)
