"""PCIe-inclusive rate of the north-star batch through the host-buffer entry
point gpu_spectrum_batch (pinned staging + H2D + kernel + D2H + copy-out),
for DESIGN.md sec. 5 -- never bench.py's `value`.
  python3 scripts/pcie_rate.py [config] [--registered] [--topk]
--registered: the series and the output array are registered first (gpu_register_host, the pinned
FeedCache).  Round 6: registration records the range only; both forms stage the series through pinned
buffers and return the records through the library's pinned output ring (rounds 2-5 DMA'd registered
arrays in place, a mode withdrawn in round 6).
--topk: gpu_spectrum_topk_batch (top-8 records in periods [18, 200]) instead of the N/2 powers:
the D2H the fused scan removes ("the PCIe wall of C4/C5")."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "fft-wavespec_amd"))
import numpy as np  # noqa: E402

from wavespec_amd import bridge, synth  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
registered = "--registered" in sys.argv
topk = "--topk" in sys.argv
cfg = synth.CONFIGS[args[0] if args else "north_star"]
n, hop, w = cfg["n"], cfg["hop"], cfg["windows"]
s = synth.random_walk((w - 1) * hop + n, seed=cfg["seed"])
out = np.empty((w, 8, 4)) if topk else np.empty((w, n // 2))
bridge.init(0, 16)
try:
    if registered:
        t0 = time.perf_counter()
        bridge.register_host(s)
        bridge.register_host(out)
        t_reg = time.perf_counter() - t0
    bridge.spectrum_batch(s[: 64 * hop + n], n, hop, cfg["detrend"], cfg["window"], 0, cfg["precision"])  # warm
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        if topk:
            p = bridge.spectrum_topk_batch(s, n, hop, cfg["detrend"], cfg["window"], 0, cfg["precision"])
        else:
            p = bridge.spectrum_batch(s, n, hop, cfg["detrend"], cfg["window"], 0, cfg["precision"], out=out)
        ts.append(time.perf_counter() - t0)
finally:
    bridge.shutdown()
best = min(ts)
bytes_moved = (s.size + out.size) * 8
print(json.dumps({"config": cfg, "seconds": ts, "windows_per_s": w / best,
                  "host_bytes_per_s": bytes_moved / best, "registered": registered, "output": "topk8" if topk else "power",
                  "register_seconds": t_reg if registered else None,
                  "note": "gpu_spectrum_batch from host memory, 1 GPU, pinned staging + pinned output ring" + (
                      " (series and output registered: recorded only)" if registered else "")}))
