"""Per-step HIP-event durations of one bench config from a cold start.

Diagnoses the gap between bench.py's wall-clock ms_per_step under short
warm-ups (the driver runs --steps 20 --warmup 5) and the steady-state kernel
time: prints the duration of each of the first STEPS launches (events on the
launch stream, one pair per step) and wall-clock timed_steps() windows of
20 steps after 5 warm-up steps, repeated.

    python scripts/step_trace.py [config] [steps]
"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "fft-wavespec_amd"))

import torch  # noqa: E402

from wavespec_amd import bridge, synth  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "north_star"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 80
cfg = dict(synth.CONFIGS[cfg_name])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
n, hop, w = cfg["n"], cfg["hop"], cfg["windows"]
tdt = torch.float32 if cfg["precision"] == "f32" else torch.float64
t_gen0 = time.perf_counter()
d_series = synth.random_walk_torch((w - 1) * hop + n, cfg["seed"], dev, tdt)
plan = bridge.Plan(0, n, hop, w, cfg["detrend"], cfg["window"], cfg.get("trend_period", 0), cfg["precision"],
                   cfg.get("output", "power"))
d_out = torch.empty(w * plan.record, dtype=tdt, device=dev)
torch.cuda.synchronize()
t_gen = time.perf_counter() - t_gen0
stream = torch.cuda.current_stream(dev)
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
t0 = time.perf_counter()
for e0, e1 in evs:
    e0.record(stream)
    plan.execute(d_series.data_ptr(), d_out.data_ptr(), stream.cuda_stream)
    e1.record(stream)
torch.cuda.synchronize()
wall = time.perf_counter() - t0
per = [e0.elapsed_time(e1) for e0, e1 in evs]
windows = []
for rep in range(5):
    for _ in range(5):
        plan.execute(d_series.data_ptr(), d_out.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(20):
        plan.execute(d_series.data_ptr(), d_out.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    windows.append((time.perf_counter() - a) / 20 * 1e3)
    time.sleep(0.2)  # let the clocks drop between repetitions, like a fresh process
print(json.dumps({"config": cfg_name, "setup_s": t_gen, "first_steps_ms": [round(x, 4) for x in per],
                  "wall_ms_per_step_cold": wall / steps * 1e3,
                  "timed_20_after_5_ms": [round(x, 4) for x in windows]}))
plan.close()
