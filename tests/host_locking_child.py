"""Child process of test_gpu_parity.py::test_host_locking_opt_in (gpu_set_host_locking(1), the page-locking form
of gpu_register_host): run in its own process so that the runtime state page-locking leaves behind after a buffer
is unregistered and freed ends with the process.  Prints "ok" and exits 0 when every check holds.

    python tests/host_locking_child.py
"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "fft-wavespec_amd"), str(ROOT / "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (the runtime the library and these queries share, as in the test process)

from wavespec_amd import bridge, synth  # noqa: E402


def hip_knows(addr: int) -> bool:
    class Attr(C.Structure):
        _fields_ = [("type", C.c_int), ("device", C.c_int), ("devicePointer", C.c_void_p),
                    ("hostPointer", C.c_void_p), ("isManaged", C.c_int), ("allocationFlags", C.c_uint)]
    hip = C.CDLL("libamdhip64.so.7")
    a = Attr()
    e = hip.hipPointerGetAttributes(C.byref(a), C.c_void_p(addr))
    hip.hipGetLastError()
    return e == 0 and a.type != 0


def batch(s, n, hop, out=None):
    return bridge.spectrum_batch(s, n, hop, "mean", "hann", out=out)


def main() -> int:
    bridge.init(0, 16)
    assert bridge.set_host_locking(1) == 0  # off by default
    page = 4096
    n, hop = 512, 7
    arena = np.zeros((16 << 20) // 8)
    first = ((37 * 8 - arena.ctypes.data % page) % page) // 8 + page // 8  # 37 doubles past a page start
    s = arena[first:first + 40000]
    s[:] = synth.random_walk(s.size, seed=43)
    nwin = 1 + (s.size - n) // hop
    out = arena[first + 40000:first + 40000 + nwin * (n // 2)]  # starts in s's last page
    assert out.ctypes.data // page == (s.ctypes.data + s.nbytes - 1) // page
    staged = batch(s.copy(), n, hop)
    bridge.register_host(s)
    bridge.register_host(out)
    lo = -(-s.ctypes.data // page) * page
    hi = (s.ctypes.data + s.nbytes) // page * page
    try:
        assert hip_knows(lo) and hip_knows(hi - 1), "inner pages locked"
        assert not hip_knows(lo - 1) and not hip_knows(hi), "shared head / tail pages stay pageable"
        p = batch(s, n, hop, out=out)
        assert np.shares_memory(p, out) and np.array_equal(p, staged), "direct DMA results"
        sub = s[1001:-333]
        assert np.array_equal(batch(sub, n, hop), batch(sub.copy(), n, hop)), "mid-page view"
        try:
            bridge.register_host(s[5:9])
            raise AssertionError("overlap accepted")
        except bridge.BridgeError as e:
            assert e.status == bridge.BAD_ARGS
    finally:
        bridge.unregister_host(out)
        bridge.unregister_host(s)
    assert not hip_knows(lo) and not hip_knows(hi - 1), "unlocked after unregistering"
    tiny = arena[first + 3:first + 300]  # no whole page inside: registered, nothing locked
    bridge.register_host(tiny)
    try:
        assert not hip_knows(tiny.ctypes.data)
        assert np.array_equal(bridge.spectrum_batch(tiny, 64, 5), bridge.spectrum_batch(tiny.copy(), 64, 5))
    finally:
        bridge.unregister_host(tiny)
    assert bridge.set_host_locking(0) == 1
    bridge.shutdown()
    print("ok", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
