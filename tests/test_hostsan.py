"""Sanitizer builds of the host layer (TSAN on the host harness, ASAN builds), CPU only.

tests/hostsan builds csrc/mtbridge.cpp against fake_hip.cpp -- a test double of the HIP runtime with
real asynchronous streams (worker threads) and launch stubs that write a checkable function of each
window -- under -fsanitize=thread and -fsanitize=address,undefined, and drives the C ABI from 30
threads (stress.cpp): 28 charts with staggered gpu_shutdown, a poller racing gpu_free_job, plans
executed while being re-targeted and destroyed, pinned feeds registered / used / unregistered from
several threads and two threads racing to register overlapping ranges.  The round-1 library fails this driver (12 TSAN
reports, profiles/r02/hostsan_stress.txt); the current one must pass it clean.
"""
import shutil
import subprocess

import pytest

from conftest import ROOT

HS = ROOT / "tests" / "hostsan"


@pytest.fixture(scope="module")
def built():
    if not shutil.which("g++"):
        pytest.skip("no host compiler")
    r = subprocess.run(["make", "-s", "-C", str(HS), "-j4", "all"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return HS / "build"


@pytest.mark.parametrize("san", ["tsan", "asan"])
def test_host_layer_under_sanitizer(built, san):
    r = subprocess.run([str(built / f"stress_{san}"), str(built / f"libmtbridge_{san}.so")], capture_output=True,
                       text=True, timeout=600)
    out = r.stdout + r.stderr
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out, out[-4000:]
    assert "runtime error" not in out, out[-4000:]
    assert r.returncode == 0 and "hostsan stress: ok" in out, out[-4000:]


@pytest.mark.parametrize("devices", [2, 8])
@pytest.mark.parametrize("san", ["tsan", "asan"])
def test_multi_device_sharding_under_sanitizer(built, san, devices):
    """gpu_init(-1) over 2 and 8 fake devices (multidev.cpp): every record of sharded batches (halo,
    disjoint output ranges), the per-device window split, per-device streams and buffers, 8 charts
    polling sharded jobs at once -- clean under TSAN and ASAN+UBSAN."""
    r = subprocess.run([str(built / f"multidev_{san}"), str(built / f"libmtbridge_{san}.so"), str(devices)],
                       capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out, out[-4000:]
    assert "runtime error" not in out, out[-4000:]
    assert r.returncode == 0 and f"hostsan multidev {devices}: ok" in out, out[-4000:]
