"""Timeline of the hop = 1 power slide (slide_kernel; wsp_plan_set_trace) on C4 or one of its strong-scaled shards:
per workgroup start, seeds done and end (XCC id beside), so a shard's time splits into launch ramp, seed phase,
slide and drain.

    python scripts/slide_timeline.py <out.json> [R/G[:seg] ...]        (default: 0/1 and 0/8)

For each case it builds exactly the workload bench.py times (bench.SingleBatch on c4), runs 30 warm executes, then
one traced execute, and writes a summary in microseconds from the first workgroup's start: seed durations, the
percentiles of workgroup starts / seed ends / ends, the span, and the HIP-event time of the traced execute.
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


def run(r, g, seg):
    wl = bench.SingleBatch("c4", r, 0, g, "strong" if g > 1 else "weak", "auto", seg)
    for _ in range(30):
        wl.step()
    torch.cuda.synchronize()
    nblk = 1 << 16
    tr = torch.zeros(4 * nblk, dtype=torch.int64, device="cuda")
    wl.plan.set_trace(tr.data_ptr(), 4 * nblk)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(wl.stream)
    wl.step()
    ev[1].record(wl.stream)
    torch.cuda.synchronize()
    wl.plan.set_trace(0, 0)
    t = tr.view(nblk, 4).cpu().numpy()
    t = t[t[:, 1] > 0]
    t0 = t[:, 1].min()
    us = lambda v: (v - t0) / 100.0  # 100 MHz wall clock
    start, seed, end = us(t[:, 1]), us(t[:, 2]), us(t[:, 3])
    return {"case": f"{r}/{g}" + (f":{seg}" if seg else ""), "workgroups": int(len(t)),
            "event_us": round(ev[0].elapsed_time(ev[1]) * 1000.0, 2), "span_us": round(float(end.max()), 2),
            "seed_us": pct(seed - start), "start_us": pct(start), "seed_end_us": pct(seed), "end_us": pct(end),
            "slide_us": pct(end - seed), "xcc_counts": np.bincount((t[:, 0] >> 32) & 15, minlength=8).tolist()}


def main():
    out = sys.argv[1]
    cases = sys.argv[2:] or ["0/1", "0/8"]
    res = []
    for c in cases:
        rg, _, seg = c.partition(":")
        r, g = (int(v) for v in rg.split("/"))
        res.append(run(r, g, int(seg) if seg else 0))
        print(json.dumps(res[-1]), flush=True)
    Path(out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
