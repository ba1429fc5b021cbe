"""Per-bar latency of the live path (1.1.0:1249 -> :520): the C++ MT5 stand-in calls
gpu_fft_real_forward once per bar, synchronously, through dlopen (host/oncalculate_harness.cpp
live mode), and prints per-call p50/p99 microseconds.  Beside it: the reference's CPU
fallback FourierTransformManual (L/WaveSpecZZ_1.0.2.mq5:938-974, the oracle's C restatement)
on one core for the same window length.  Writes one JSON object to stdout.

    python scripts/latency.py [N] [bars]
"""
import json
import re
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "fft-wavespec_amd"), str(ROOT / "oracle")]
import oracle  # noqa: E402  (checker / CPU baseline only)
from wavespec_amd import bridge, indicator, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
bars = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
hist = synth.random_walk(n + bars - 1, seed=31)
with tempfile.TemporaryDirectory() as d:
    feed, out = Path(d) / "feed.bin", Path(d) / "out.bin"
    indicator.save_feed_cache(str(feed), hist[::-1].copy())
    r = subprocess.run([str(ROOT / "fft-wavespec_amd" / "bin" / "oncalculate_harness"), str(bridge.LIB_PATH), "live",
                        str(feed), str(n), str(bars), str(out)], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        sys.exit(r.stderr)
    spectra = np.fromfile(out, dtype=np.float64).reshape(bars, n // 2)
m = re.search(r"first=([\d.]+) p50=([\d.]+) p90=([\d.]+) p99=([\d.]+) max=([\d.]+) mean=([\d.]+)", r.stdout)
first, p50, p90, p99, mx, mean = map(float, m.groups())
err = oracle.rel_err(spectra[[0, bars // 2, bars - 1]], oracle.batch_spectrum(hist, n, 1, "none", "none")[[0, bars // 2, bars - 1]])
x = hist[:n].copy()
reps, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < 2.0:
    oracle.fft_manual(x)
    reps += 1
cpu_us = (time.perf_counter() - t0) / reps * 1e6
print(json.dumps({"N": n, "bars": bars, "gpu_fft_real_forward_us": {"first": first, "p50": p50, "p90": p90, "p99": p99,
                                                                    "max": mx, "mean": mean},
                  "cpu_FourierTransformManual_us_1core": cpu_us, "parity_rel_err": err,
                  "harness": r.stdout.strip().splitlines()}))
