"""Timeline of the fused large-N kernel (fft-wavespec_amd/csrc/large_fft.hip fused_kernel, the default for fp64
N = 65536; wsp_plan_set_trace): for each workgroup's first window, per column block and row block, the time until
its samples / rows are in registers (the loads), the FFT, the rest of the block (twiddles / R2C, stores, barriers),
and the gaps -- where a window's ~80 us go.

    python scripts/large_timeline.py <out.json> [config=large]

Builds exactly the workload bench.py times (bench.SingleBatch), runs 20 warm executes, then one traced execute
(the traced instantiation is a separate kernel of the same code), and summarises in microseconds.
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "fft-wavespec_amd")]
import bench  # noqa: E402


def pct(a):
    return [round(float(x), 2) for x in np.percentile(a, [0, 10, 50, 90, 100])] if len(a) else []


def main():
    out = sys.argv[1]
    cfg = sys.argv[2] if len(sys.argv) > 2 else "large"
    wl = bench.SingleBatch(cfg, 0, 0, 1, "weak")
    for _ in range(20):
        wl.step()
    torch.cuda.synchronize()
    nwg = 1024
    tr = torch.zeros(32 * nwg, dtype=torch.int64, device="cuda")
    wl.plan.set_trace(tr.data_ptr(), 32 * nwg)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(wl.stream)
    wl.step()
    ev[1].record(wl.stream)
    torch.cuda.synchronize()
    wl.plan.set_trace(0, 0)
    t = tr.view(nwg, 8, 4).cpu().numpy().astype(np.float64)
    t = t[t[:, 0, 0] > 0]
    t0 = t[:, 0, 0].min()
    t = (t - t0) / 100.0  # 100 MHz wall clock -> us
    res = {"config": cfg, "workgroups": int(len(t)), "event_us": round(ev[0].elapsed_time(ev[1]) * 1000.0, 2),
           "first_window_start_us": pct(t[:, 0, 0]), "first_window_us": pct(t[:, 7, 3] - t[:, 0, 0]), "blocks": []}
    for b in range(8):
        res["blocks"].append({"block": ("col" if b < 4 else "row") + str(b % 4), "load_us": pct(t[:, b, 1] - t[:, b, 0]),
                              "fft_us": pct(t[:, b, 2] - t[:, b, 1]), "after_fft_us": pct(t[:, b, 3] - t[:, b, 2]),
                              "gap_before_us": pct(t[:, b, 0] - (t[:, b - 1, 3] if b else t[:, 0, 0]))})
    print(json.dumps(res, indent=1))
    Path(out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
