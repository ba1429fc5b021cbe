"""Per-task timeline of C5's mixed-length persistent launch (wsp_group_set_trace): where a strong-scaled
shard's time goes -- seeds, slides, idle workgroups, the tail.

    python scripts/c5_timeline.py <out.json> [R/G ...] [--segment S] [--mode MODE]

For each shard R/G (default: the whole batch and 0/8) it builds exactly the workload bench.py times
(bench.C5Batch, strong split), runs 30 warm executes, then one traced execute, and writes per-task
[class, workgroup, xcc, start, seeds done, end] in microseconds from the launch's first task start, plus
a summary: span, seed time per class, busy fraction of the resident workgroups, tail.
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "fft-wavespec_amd")]
import bench  # noqa: E402


def run(shard, segment, mode):
    r, g = shard
    scaling = "strong" if g > 1 else "weak"
    wl = bench.C5Batch(r, 0, g, scaling, "auto", segment, "greedy", 0,
                       "group" if mode == "auto" else f"group-{mode}", "split")
    for _ in range(30):
        wl.step()
    torch.cuda.synchronize()
    tasks = wl.group.last_tasks
    tr = torch.zeros(4 * tasks, dtype=torch.int64, device="cuda")
    wl.group.set_trace(tr.data_ptr(), tasks)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(wl.stream)
    wl.step()
    ev[1].record(wl.stream)
    torch.cuda.synchronize()
    wl.group.set_trace(0, 0)
    t = tr.view(tasks, 4).cpu().numpy()
    # task -> class from the group's layout: tasks are numbered longest windows first
    lens = sorted({n for n in (wl.group.window_lens)}, reverse=True)
    t0 = t[:, 1].min()
    us = (t[:, 1:] - t0) / 100.0  # 100 MHz wall clock -> us
    wg = (t[:, 0] & 0xFFFFFFFF).astype(int)
    xcc = (t[:, 0] >> 32).astype(int)
    span = us[:, 2].max()
    seed = us[:, 1] - us[:, 0]
    slide = us[:, 2] - us[:, 1]
    nwg = wg.max() + 1
    busy = (us[:, 2] - us[:, 0]).sum() / (nwg * span)
    first_end = np.array([us[wg == w, 2].max() for w in np.unique(wg)])
    summ = {"shard": f"{r}/{g}", "tasks": int(tasks), "workgroups": int(nwg), "event_ms": ev[0].elapsed_time(ev[1]),
            "span_us": float(span), "busy_frac": float(busy),
            "seed_us_mean": float(seed.mean()), "seed_us_first_round": float(seed[us[:, 0] < 1.0].mean()),
            "slide_us_mean": float(slide.mean()), "tasks_per_wg_max": int(np.bincount(wg).max()),
            "wg_end_us_p10_p50_p90": [float(x) for x in np.percentile(first_end, [10, 50, 90])],
            "windows": wl.windows, "lens": lens}
    print(json.dumps(summ), flush=True)
    wl.close()
    return {"summary": summ, "tasks": [[int(wg[i]), int(xcc[i]), *[round(float(x), 2) for x in us[i]]]
                                       for i in range(tasks)]}


def main():
    out = sys.argv[1]
    args = sys.argv[2:]
    seg, mode = 0, "auto"
    shards = []
    i = 0
    while i < len(args):
        if args[i] == "--segment":
            seg = int(args[i + 1]); i += 2; continue
        if args[i] == "--mode":
            mode = args[i + 1]; i += 2; continue
        shards.append(tuple(int(v) for v in args[i].split("/"))); i += 1
    shards = shards or [(0, 1), (0, 8)]
    from wavespec_amd import bridge
    bridge.init(0, 16)
    res = {f"{r}/{g}": run((r, g), seg, mode) for r, g in shards}
    Path(out).write_text(json.dumps(res))
    bridge.shutdown()


if __name__ == "__main__":
    main()
