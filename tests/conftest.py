import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "fft-wavespec_amd", ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: full-size runs")


def _gpu_present() -> bool:
    # counting devices does not initialise the GPU on this image
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


GPU = _gpu_present()


@pytest.fixture(scope="session")
def gpu_session():
    """Session on device 0 through the C ABI; fails (not skips) on a GPU box
    whose library is missing, so a silent fallback can never pass."""
    if not GPU:
        pytest.skip("no GPU visible")
    from wavespec_amd import bridge
    bridge.lib()  # raises if libmtbridge.so is missing
    bridge.init(0, 16)
    yield bridge
    bridge.shutdown()
