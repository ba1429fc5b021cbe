#!/usr/bin/env python3
"""bench.py -- windows/s of the MI355X spectrum hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config north_star]

One step = one launch of the hot path over the configuration's whole window
batch, input already resident in HBM (series generated on device).  N > 1 is
launched by torch.distributed.run: every rank owns a full, independent batch
on its own GPU (weak scaling, no data-path collective; a CPU gloo group only
brackets the timed region with barriers and takes the max time over ranks).

Prints ONE JSON line (rank 0) with the driver's contract fields plus
`roofline` (live HIP-event kernel time vs HBM peak) and `cpu_baseline` (the
oracle -- CPU restatement of the reference path -- timed on a bounded sample
on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "fft-wavespec_amd"))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "FFT-windows/sec"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="north_star",
                    choices=["c2", "c3", "north_star", "c4", "c5", "ns_topk", "ns_phase", "ns_topk_phase", "inverse", "large",
                             "large_262144"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the 1-core CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def dist_env():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


class Control:
    """Barrier + max-over-ranks on a CPU gloo group (no GPU collective)."""

    def __init__(self, world: int):
        self.world = world
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def timed_steps(step, sync, ctl: Control, steps: int, warmup: int) -> float:
    """W untimed steps, then K steps bracketed by barrier + device sync; returns max seconds over ranks."""
    for _ in range(warmup):
        step()
    sync()
    ctl.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    ctl.barrier()
    t1 = time.perf_counter()
    return ctl.max(t1 - t0)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def cpu_threads() -> int:
    """Threads for the all-core leg: the job's CPU share (OMP_NUM_THREADS on the GPU box), at most 16."""
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    return max(1, min(16, n or (os.cpu_count() or 1)))


def cpu_baseline(d_series, cfg: dict, budget_s: float, threads: int = 1) -> dict:
    """Oracle (CPU restatement of the reference per-window path, C -O3) on
    `threads` cores (OpenMP over windows; 1 = the single-threaded MQL5
    OnCalculate), on the leading windows of the same device-resident workload
    (copied to the host chunk by chunk, outside the timed CPU work), for
    about budget_s seconds."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    lib = oracle.lib()
    threads = lib.ora_set_threads(threads)
    n, hop = cfg["n"], cfg["hop"]
    out = cfg.get("output", "power")
    args = (n, hop, cfg["detrend"], cfg["window"], cfg.get("trend_period", 0))

    def work(seg):
        if out == "inverse":
            for row in seg.reshape(-1, n):
                oracle.fft_real_inverse(row)
        elif out == "phase":
            oracle.batch_phase(seg, *args, kalman=oracle.KALMAN_DEFAULTS)
        elif out in ("topk", "topk_phase"):
            f = oracle.batch_topk if out == "topk" else oracle.batch_topk_phase
            f(seg, *args, oracle.KALMAN_DEFAULTS, 8, 18.0, 200.0)
        else:
            oracle.batch_spectrum(seg, *args, kalman=oracle.KALMAN_DEFAULTS)

    chunk = 256 * threads
    done, spent = 0, 0.0
    max_w = cfg["windows"]
    while spent < budget_s and done < max_w:
        take = min(chunk, max_w - done)
        seg = d_series[done * hop: (done + take - 1) * hop + n].double().cpu().numpy()
        t0 = time.perf_counter()
        work(seg)
        spent += time.perf_counter() - t0
        done += take
    dt = spent
    lib.ora_set_threads(1)
    return {"value": done / dt, "unit": "windows/s", "cores": threads, "kind": "port",
            "sample": f"first {done} windows of the same {cfg['windows']}x{n} workload (hop={hop}, "
                      f"{cfg['detrend']} detrend, {cfg['window']} window, output {out}), "
                      f"oracle/wavespec_oracle.c -O3, {threads} thread(s) on {cpu_model()}, {dt:.1f} s"}


def load_traffic(config: str):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/), or None."""
    p = ROOT / "profiles" / "traffic.json"
    if not p.exists():
        return None
    try:
        return json.loads(p.read_text()).get(config, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def run_c5(args, rank, local_rank, world, ctl):
    """C5: 28 symbols x 20000 bars, N in {512,1024,2048,4096} (7 symbols each),
    hop = 1, fp64, Hann -- the WaveCyclesBatchFetcher shape
    (WaveCyclesBatchFetcher.mq5:106-133: one batch per symbol).  One step =
    every symbol's batch; each window length runs on its own stream."""
    import torch
    from wavespec_amd import bridge, synth
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    bars, lens = 20000, (512, 1024, 2048, 4096)
    streams = [torch.cuda.Stream(dev) for _ in lens]
    jobs = []  # (plan, series, out, stream)
    for sym in range(28):
        n = lens[sym // 7]
        nw = bars - n + 1
        series = synth.random_walk_torch(bars, 100 + sym + 1000 * rank, dev)
        out = torch.empty(nw * (n // 2), dtype=torch.float64, device=dev)
        jobs.append((bridge.Plan(local_rank, n, 1, nw, "none", "hann"), series, out, streams[sym // 7]))
    total_w = sum(j[0].n_windows for j in jobs)
    alg = sum(j[0].algorithmic_bytes for j in jobs)
    main_stream = torch.cuda.current_stream(dev)

    def step():
        for st in streams:
            st.wait_stream(main_stream)
        for plan, series, out, st in jobs:
            plan.execute(series.data_ptr(), out.data_ptr(), st.cuda_stream)
        for st in streams:
            main_stream.wait_stream(st)

    secs = timed_steps(step, torch.cuda.synchronize, ctl, args.steps, args.warmup)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    ev0.record(main_stream)
    for _ in range(reps):
        step()
    ev1.record(main_stream)
    ev1.synchronize()
    step_s = ev0.elapsed_time(ev1) / 1e3 / reps
    value = ctl.sum(float(total_w * args.steps)) / secs
    baseline = baseline_all = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        plan0, s0, _, _ = jobs[-1]  # a 4096-pt symbol: the costliest per window
        c5cfg = {"n": 4096, "hop": 1, "windows": plan0.n_windows, "detrend": "none", "window": "hann"}
        baseline = cpu_baseline(s0, c5cfg, args.cpu_seconds)
        baseline_all = cpu_baseline(s0, c5cfg, args.cpu_seconds / 2, cpu_threads())
    if rank == 0:
        achieved = alg / step_s / 1e9
        per_launch = load_traffic("c5")  # PMC bytes per spectrum dispatch; one step is len(jobs) dispatches
        c5_traffic = per_launch * len(jobs) if per_launch else None
        print(json.dumps({
            "metric": METRIC, "value": value, "unit": "windows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": secs / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (28 random-walk symbols generated on device)",
            "config": {"workload": f"c5: 28 symbols x {bars} bars, N in {lens} (7 each), hop=1, f64, Hann, |X|^2",
                       "windows_per_gpu": total_w, "window_len": "mixed", "hop": 1,
                       "parallelism": f"symbols' batches on 4 streams, x{world} GPUs"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": c5_traffic,
                         "algorithmic_bytes_per_launch": alg, "kernel_ms": step_s * 1e3,
                         "note": "one step = 28 launches on 4 streams; time per step from HIP events"},
            "cpu_baseline": baseline, "cpu_baseline_all_cores": baseline_all}), flush=True)
    for j in jobs:
        j[0].close()
    ctl.close()


def main():
    args = parse()
    rank, local_rank, world = dist_env()
    import torch
    from wavespec_amd import bridge, synth

    if args.config == "c5":
        return run_c5(args, rank, local_rank, world, Control(world))
    cfg = dict(synth.CONFIGS[args.config])
    cfg.setdefault("trend_period", 0)
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    ctl = Control(world)

    n, hop, w = cfg["n"], cfg["hop"], cfg["windows"]
    f32 = cfg["precision"] == "f32"
    tdt = torch.float32 if f32 else torch.float64
    length = (w - 1) * hop + n
    output = cfg.get("output", "power")
    if output == "inverse":  # rows of packed spectra (random, resident in HBM)
        gen = torch.Generator(device=dev)
        gen.manual_seed(cfg["seed"] + 1000 * rank)
        d_series = torch.randn(w * n, dtype=tdt, device=dev, generator=gen)
        plan = bridge.Plan.inverse(local_rank, n, w)
    else:
        d_series = synth.random_walk_torch(length, cfg["seed"] + 1000 * rank, dev, tdt)  # resident in HBM
        plan = bridge.Plan(local_rank, n, hop, w, cfg["detrend"], cfg["window"], cfg["trend_period"],
                           cfg["precision"], output)
        if output in ("topk", "topk_phase"):
            plan.set_topk(8, 18.0, 200.0)  # the reference's scan (1.1.0:22-23)
    d_out = torch.empty(w * plan.record, dtype=tdt, device=dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    def step():
        plan.execute(d_series.data_ptr(), d_out.data_ptr(), sptr)

    sync = torch.cuda.synchronize
    secs = timed_steps(step, sync, ctl, args.steps, args.warmup)

    # live kernel time with HIP events on the launch stream (roofline)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = max(10, min(args.steps, 50))
    ev0.record(stream)
    for _ in range(reps):
        step()
    ev1.record(stream)
    ev1.synchronize()
    kernel_s = ev0.elapsed_time(ev1) / 1e3 / reps
    alg_bytes = plan.algorithmic_bytes
    achieved = alg_bytes / kernel_s / 1e9

    total_windows = ctl.sum(float(w * args.steps))
    value = total_windows / secs
    baseline = baseline_all = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        baseline = cpu_baseline(d_series, cfg, args.cpu_seconds)
        baseline_all = cpu_baseline(d_series, cfg, args.cpu_seconds / 2, cpu_threads())

    if rank == 0:
        traffic = load_traffic(args.config)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "windows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": secs / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if f32 else "f64",
            "data": "synthetic (random-walk close prices generated on device, seed per rank)",
            "config": {"workload": f"{args.config}: {w} windows x {n}-pt, hop={hop}, {cfg['precision']}, "
                                   f"{cfg['detrend']} detrend, {cfg['window']} window, " + {
                                       "power": "|X|^2 k<N/2", "topk": "top-8 bins in periods [18, 200]",
                                       "phase": "[|X|^2, unwrapped phase, group delay] k<N/2",
                                       "topk_phase": "top-8 bins + phase/delay in periods [18, 200]",
                                       "inverse": "inverse real FFT of packed spectra"}[output],
                       "windows_per_gpu": w, "window_len": n, "hop": hop, "parallelism": f"windows sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes_per_launch": alg_bytes, "kernel_ms": kernel_s * 1e3},
            "cpu_baseline": baseline,
            "cpu_baseline_all_cores": baseline_all,
        }
        print(json.dumps(line), flush=True)
    plan.close()
    ctl.close()


if __name__ == "__main__":
    main()
