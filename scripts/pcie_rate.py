"""PCIe-inclusive rate of the north-star batch through the host-buffer entry
point gpu_spectrum_batch (pinned staging + H2D + kernel + D2H + copy-out),
for DESIGN.md sec. 5 -- never bench.py's `value`."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "fft-wavespec_amd"))
import numpy as np  # noqa: E402

from wavespec_amd import bridge, synth  # noqa: E402

cfg = synth.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "north_star"]
n, hop, w = cfg["n"], cfg["hop"], cfg["windows"]
s = synth.random_walk((w - 1) * hop + n, seed=cfg["seed"])
out = np.empty((w, n // 2))
bridge.init(0, 16)
try:
    bridge.spectrum_batch(s[: 64 * hop + n], n, hop, cfg["detrend"], cfg["window"], 0, cfg["precision"])  # warm
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        p = bridge.spectrum_batch(s, n, hop, cfg["detrend"], cfg["window"], 0, cfg["precision"])
        ts.append(time.perf_counter() - t0)
finally:
    bridge.shutdown()
best = min(ts)
bytes_moved = (s.size + w * (n // 2)) * 8
print(json.dumps({"config": cfg, "seconds": ts, "windows_per_s": w / best,
                  "host_bytes_per_s": bytes_moved / best, "note": "gpu_spectrum_batch from host memory, 1 GPU"}))
