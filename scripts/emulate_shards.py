#!/usr/bin/env python3
"""Single-GPU emulation of strong-scaled multi-GPU runs.

    python scripts/emulate_shards.py <out.json> [--configs north_star,c4,c5] [--gpus 2,4,8]
                                     [--c5-shards split,split-time,symbols] [--steps 50] [--warmup 10]

For every configuration and every G it runs `bench.py --emulate-shard R/G` for each rank R (one child
process each, timed exactly like a normal bench step: settle, W warm-up steps, K timed steps), plus the
whole batch on one GPU (G = 1).  A G-GPU run of a shard-without-exchange workload takes as long as its
slowest rank, so the predicted strong-scaling speed-up is T(1) / max_R T(R, G).  Caveat: this is a
single-GPU emulation -- every rank's shard timed alone on the same device, one after another -- not a
scaling curve: it leaves out the cross-rank barrier and any node-level contention (host memory, power).
"""
from __future__ import annotations

import argparse
import json
import re
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def run_bench(args: list[str], timeout: float) -> dict:
    cmd = [sys.executable, str(ROOT / "bench.py"), "--no-cpu-baseline"] + args
    t0 = time.time()
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    if p.returncode != 0:
        raise RuntimeError(f"{' '.join(cmd)} -> rc {p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}")
    line = json.loads(p.stdout.strip().splitlines()[-1])
    line["_wall_s"] = round(time.time() - t0, 2)
    return line


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--configs", default="north_star,c4,c4_topk,c5")
    ap.add_argument("--gpus", default="2,4,8")
    ap.add_argument("--c5-shards", default="split,split-time,symbols")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--extra", default="", help="extra bench.py arguments, comma- or plus-separated")
    ap.add_argument("--repeat", type=int, default=1,
                    help="passes over the ranks (and the whole batch); each rank's time = the median of its passes")
    a = ap.parse_args()
    gs = [int(g) for g in re.split("[,+]", a.gpus)]
    extra = [x for x in re.split("[,+]", a.extra) if x]
    common = ["--steps", str(a.steps), "--warmup", str(a.warmup)] + extra
    res = {"caveat": "single-GPU emulation, not a scaling curve: each rank's strong-scaling shard is timed alone on "
                     "one MI355X (bench.py --emulate-shard R/G); predicted speed-up = T(whole batch on 1 GPU) / "
                     "max over ranks of T(shard)",
           "steps": a.steps, "warmup": a.warmup, "repeat": a.repeat, "configs": {}}
    for cfg in re.split("[,+]", a.configs):
        modes = re.split("[,+]", a.c5_shards) if cfg == "c5" else ["windows"]
        ones = [run_bench(["--config", cfg] + common, 300) for _ in range(a.repeat)]
        one = sorted(ones, key=lambda x: x["ms_per_step"])[len(ones) // 2]
        t1 = one["ms_per_step"]
        print(f"{cfg} G=1: {t1:.4f} ms ({one['value']:.4g} windows/s, frac {one['roofline']['frac']:.3f})", flush=True)
        for mode in modes:
            key = cfg if cfg != "c5" else f"c5[{mode}]"
            entry = {"t1_ms": t1, "t1_frac": one["roofline"]["frac"], "t1_passes": [x["ms_per_step"] for x in ones],
                     "split": mode, "by_g": {}}
            for g in gs:
                runs = {r: [] for r in range(g)}
                for _ in range(a.repeat):  # passes over the ranks: box drift touches every rank alike
                    for r in range(g):
                        args = ["--config", cfg, "--emulate-shard", f"{r}/{g}"] + common
                        if cfg == "c5":
                            args += ["--c5-shard", mode]
                        ln = run_bench(args, 300)
                        runs[r].append(ln)
                        print(f"  {key} {r}/{g}: {ln['ms_per_step']:.4f} ms, {ln['config']['windows_per_gpu']} windows, "
                              f"frac {ln['roofline']['frac']:.3f}", flush=True)
                ranks = []
                for r in range(g):
                    ln = sorted(runs[r], key=lambda x: x["ms_per_step"])[len(runs[r]) // 2]
                    ranks.append({"rank": r, "ms": ln["ms_per_step"], "kernel_ms": ln["roofline"]["kernel_ms"],
                                  "ms_passes": [x["ms_per_step"] for x in runs[r]],
                                  "windows": ln["config"]["windows_per_gpu"],
                                  "alg_bytes": ln["roofline"]["algorithmic_bytes_per_launch"],
                                  "frac": ln["roofline"]["frac"], "workload": ln["config"]["workload"]})
                worst = max(x["ms"] for x in ranks)
                mean = sum(x["ms"] for x in ranks) / g
                entry["by_g"][str(g)] = {"ranks": ranks, "worst_ms": worst, "mean_ms": mean,
                                         "predicted_speedup": t1 / worst, "predicted_efficiency": t1 / worst / g,
                                         "imbalance": worst / mean}
                print(f"  {key} G={g}: worst {worst:.4f} ms -> predicted {t1 / worst:.2f}x "
                      f"({t1 / worst / g:.2f} of linear), imbalance {worst / mean:.3f}", flush=True)
            res["configs"][key] = entry
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
