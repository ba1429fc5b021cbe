"""Timeline of the hop = 1 top-k pair (seed kernel, then probe scan; wsp_plan_set_trace) on C4 top-8 or one of
its strong-scaled shards: where the time goes -- FFT seeds, seed chains, scan workgroups, gaps.

    python scripts/topk_timeline.py <out.json> [R/G[:seg[:chain[:variant]]] ...]

For each case (default: 0/8 at the policy's segment, and 0/8:32:4) it builds exactly the workload bench.py times
(bench.SingleBatch on c4_topk, strong shard), runs 30 warm executes, then one traced execute, and writes a
summary (microseconds from the seed launch's first workgroup start): seed phases (percentiles of FFT 0, FFT 1,
chain and end), scan workgroups' start / end percentiles, the gap between the last seed and the first scan.
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


def run(r, g, seg, chain, variant=0):
    wl = bench.SingleBatch("c4_topk", r, 0, g, "strong" if g > 1 else "weak", "auto", seg, variant, 0, chain)
    for _ in range(30):
        wl.step()
    torch.cuda.synchronize()
    cap = 3 << 19  # half for the seed records (6 entries each), half for the scan records (2 each)
    tr = torch.zeros(cap, dtype=torch.int64, device="cuda")
    wl.plan.set_trace(tr.data_ptr(), cap)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(wl.stream)
    wl.step()
    ev[1].record(wl.stream)
    torch.cuda.synchronize()
    wl.plan.set_trace(0, 0)
    t = tr.cpu().numpy()
    seeds = t[: cap // 2 // 6 * 6].reshape(-1, 6)
    seeds = seeds[seeds[:, 1] > 0]
    scans = t[cap // 2:].reshape(-1, 2)
    scans = scans[scans[:, 0] > 0]
    t0 = seeds[:, 1].min()
    su = (seeds[:, 1:] - t0) / 100.0  # 100 MHz wall clock -> us
    cu = (scans - t0) / 100.0
    summ = {"case": f"{r}/{g}:{seg or 'auto'}:{chain or 'auto'}:v{variant}", "event_ms": ev[0].elapsed_time(ev[1]),
            "seed_workgroups": int(len(seeds)), "scan_workgroups": int(len(scans)),
            "seed_start": pct(su[:, 0]), "seed_fft0_us": pct(su[:, 1] - su[:, 0]), "seed_fft1_us": pct(su[:, 2] - su[:, 1]),
            "seed_chain_us": pct(su[:, 3] - su[:, 2]), "seed_end": pct(su[:, 4]),
            "scan_start": pct(cu[:, 0]), "scan_end": pct(cu[:, 1]), "scan_dur_us": pct(cu[:, 1] - cu[:, 0]),
            "gap_last_seed_first_scan_us": round(float(cu[:, 0].min() - su[:, 4].max()), 2) if len(cu) else None}
    print(json.dumps(summ), flush=True)
    return summ


def main():
    out = sys.argv[1]
    cases = []
    for a in sys.argv[2:] or ["0/8", "0/8:32:4"]:
        rg, *rest = a.split(":")
        r, g = (int(v) for v in rg.split("/"))
        seg = int(rest[0]) if rest else 0
        chain = int(rest[1]) if len(rest) > 1 else 0
        variant = int(rest[2]) if len(rest) > 2 else 0
        cases.append((r, g, seg, chain, variant))
    from wavespec_amd import bridge
    bridge.init(0, 16)
    res = [run(*c) for c in cases]
    Path(out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
