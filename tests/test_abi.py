"""CPU tests of the C ABI boundary: the library loads, exports every symbol
include/mtbridge.h declares with the reference's status conventions, and
rejects bad arguments before touching a GPU.  No compute calls here."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import GPU, ROOT
from wavespec_amd import bridge

HEADER = ROOT / "include" / "mtbridge.h"


def declared_symbols():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"MTB_API\s+[\w\s\*]+?\b(\w+)\s*\(", text)))


def test_header_declares_reference_surface():
    syms = declared_symbols()
    # Include/imports.mqh:5-19
    for name in ("gpu_init", "gpu_shutdown", "gpu_fft_real_forward", "gpu_extract_cycles",
                 "gpu_submit_extract_cycles", "gpu_try_get_cycles", "gpu_submit_extract_cycles_batch",
                 "gpu_try_get_cycles_batch", "gpu_free_job", "gpu_get_last_error_w"):
        assert name in syms
    assert "gpu_fft_real_forward_batch" in syms  # L/WaveSpecZZ_1.0.3-pla-batch.mq5:29


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", str(bridge.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    # nothing else leaks (hidden visibility)
    assert exported == set(declared_symbols())


def test_python_binding_covers_header():
    assert set(bridge.SIGNATURES) == set(declared_symbols())


def test_version():
    assert bridge.lib().wsp_version().decode().startswith("mtbridge-mi355x")


def test_status_codes_match_header():
    text = HEADER.read_text()
    for name, val in (("MTB_OK", 0), ("MTB_BAD_ARGS", -1), ("MTB_BACKEND_UNAVAILABLE", -2), ("MTB_TIMEOUT", -3),
                      ("MTB_INTERNAL_ERROR", -4), ("MTB_NOT_READY", -5), ("MTB_NO_MEM", -6)):
        assert re.search(rf"#define {name} \(?{val}\)?", text), name


def test_last_error_counts_terminator():
    L = bridge.lib()
    x = np.zeros(100)
    st = L.gpu_fft_real_forward(x.ctypes.data_as(C.POINTER(C.c_double)), 100, x.ctypes.data_as(
        C.POINTER(C.c_double)))
    assert st == bridge.BAD_ARGS  # 100 is not a power of two
    buf = (C.c_uint16 * 256)()
    n = L.gpu_get_last_error_w(buf, 256)
    msg = "".join(chr(buf[i]) for i in range(n - 1))
    assert buf[n - 1] == 0 and "power of two" in msg
    small = (C.c_uint16 * 4)()
    assert L.gpu_get_last_error_w(small, 4) == 4 and small[3] == 0


@pytest.mark.parametrize("n", [0, 16, 100, 8196, 32768])
def test_bad_window_len(n):
    s = np.zeros(10000)
    out = np.zeros(10000)
    got = C.c_int32(7)
    st = bridge.lib().gpu_spectrum_batch(bridge._dptr(s), s.size, n, 1, 0, 1, 0, 0, 0, bridge._dptr(out), out.size,
                                         C.byref(got))
    assert st == bridge.BAD_ARGS and got.value == 0


def test_bad_modes_and_shapes():
    s = np.zeros(4096)
    out = np.zeros(4096)
    L = bridge.lib()
    got = C.c_int32(0)
    for args in ((1024, 1, 9, 1, 0, 0, 0), (1024, 1, 0, 7, 0, 0, 0), (1024, 1, 0, 1, 0, 5, 0),
                 (1024, 0, 0, 1, 0, 0, 0), (8192, 1, 0, 1, 0, 0, 0), (1024, 1, 0, 1, 0, 0, 5),
                 (1024, 1, 0, 1, 0, 1, 3), (1024, 1, 0, 1, 0, 1, 4)):  # bad output; phase outputs are fp64
        n, hop, det, win, per, prec, outk = args
        st = L.gpu_spectrum_batch(bridge._dptr(s), s.size, n, hop, det, win, per, prec, outk, bridge._dptr(out),
                                  out.size, C.byref(got))
        assert st == bridge.BAD_ARGS, args
    # out_cap smaller than one record
    st = L.gpu_spectrum_batch(bridge._dptr(s), s.size, 1024, 1024, 0, 1, 0, 0, 0, bridge._dptr(out), 100,
                              C.byref(got))
    assert st == bridge.BAD_ARGS


def test_cycles_api_reports_backend_unavailable():
    L = bridge.lib()
    jid = C.c_int64(99)
    s = np.zeros(64)
    st = L.gpu_submit_extract_cycles(bridge._dptr(s), 64, 4, 9.0, 200.0, 60.0, 1, 10, C.byref(jid))
    assert st == bridge.BACKEND_UNAVAILABLE and jid.value == 0
    assert "cycle" in bridge.last_error().lower()


def test_unknown_job_and_plan():
    assert bridge.free_job(123456789) == bridge.BAD_ARGS
    assert bridge.lib().wsp_plan_destroy(987654321) == bridge.BAD_ARGS
    assert bridge.lib().wsp_plan_algorithmic_bytes(987654321) == -1


def test_host_locking_mode():
    """gpu_set_host_locking: round 6 withdrew page-locking of caller memory -- 0 (record the range,
    stage through the library's pinned buffers) is the only mode and returns 0, 1 is refused with an explanation,
    anything else is refused (no session needed)."""
    L = bridge.lib()
    assert L.gpu_set_host_locking(2) == bridge.BAD_ARGS
    assert L.gpu_set_host_locking(-1) == bridge.BAD_ARGS
    assert L.gpu_set_host_locking(1) == bridge.BAD_ARGS
    assert "withdrawn" in bridge.last_error()
    assert bridge.set_host_locking(0) == 0
    assert bridge.set_host_locking(0) == 0
    for mode in (1, 7):
        with pytest.raises(bridge.BridgeError) as e:
            bridge.set_host_locking(mode)
        assert e.value.status == bridge.BAD_ARGS


@pytest.mark.skipif(GPU, reason="checks the no-GPU behaviour")
def test_no_gpu_fails_loudly_without_fallback():
    assert bridge.lib().gpu_init(0, 64) == bridge.BACKEND_UNAVAILABLE
    assert "no CPU fallback" in bridge.last_error()
    x = np.ones(1024)
    st = bridge.lib().gpu_fft_real_forward(bridge._dptr(x), 1024, bridge._dptr(x))
    assert st == bridge.BACKEND_UNAVAILABLE
    assert bridge.lib().wsp_plan_create(0, 1024, 1024, 4, 0, 1, 0, 0, 0) == 0
    assert bridge.lib().gpu_register_host(bridge._dptr(x), x.size) == bridge.BACKEND_UNAVAILABLE
    assert bridge.lib().gpu_unregister_host(bridge._dptr(x)) == bridge.BACKEND_UNAVAILABLE


def test_harness_binary_built():
    h = ROOT / "fft-wavespec_amd" / "bin" / "oncalculate_harness"
    assert h.exists()
    r = subprocess.run([str(h)], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr
