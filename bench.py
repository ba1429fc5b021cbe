#!/usr/bin/env python3
"""bench.py -- windows/s of the MI355X spectrum hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config north_star]
                    [--scaling weak|strong]

One step = one launch of the hot path over the configuration's whole window
batch, input already resident in HBM (series generated on device).  One
process per GPU: with --gpus N > 1 and no WORLD_SIZE in the environment the
script starts `torch.distributed.run` with N ranks as a child process (before
any GPU call) and exits with its status; under torchrun WORLD_SIZE must equal
--gpus.  A CPU gloo group only brackets the timed region with barriers and
takes the max time over ranks -- no collective is on the data path (windows
shard with no exchange).

  --scaling weak   every rank owns a full, independent batch (seed per rank)
  --scaling strong the configuration's one batch is split over the ranks:
                   contiguous window ranges with the N - hop halo (north star,
                   C3, C4) or whole symbols balanced by bytes (C5)

Before the W warm-up steps the step is repeated until its HIP-event duration
is steady (the MI355X holds its memory clocks low after idle and needs ~40
launches of this size to ramp; a short timed region otherwise measures the
ramp -- scripts/step_trace.py, profiles/r02/step_trace_*.json).  That settle
phase is untimed and reported in the line ("settle").  The timed region is
exactly K full steps; `roofline.kernel_ms` comes from HIP events recorded on
the launch stream around those same K steps.

Prints ONE JSON line (rank 0) with the driver's contract fields plus
`roofline` and `cpu_baseline` (the oracle -- CPU restatement of the reference
path -- timed on a bounded sample on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "fft-wavespec_amd"))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "FFT-windows/sec"
CONFIGS = ["c2", "c3", "north_star", "c4", "c4_topk", "c5", "ns_topk", "ns_phase", "ns_topk_phase", "inverse", "large",
           "large_131072", "large_262144"]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="north_star", choices=CONFIGS)
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the 1-core CPU baseline sample")
    ap.add_argument("--algo", default="auto", choices=["auto", "fft", "slide"],
                    help="hop = 1 power batches: seeded sliding DFT or FFT per window (wsp_plan_set_algorithm)")
    ap.add_argument("--slide-seg", type=int, default=0, help="windows per sliding-DFT workgroup (0 = library policy)")
    ap.add_argument("--seed-chain", type=int, default=0,
                    help="hop = 1 top-k: segments per seed workgroup (wsp_plan_set_seed_chain; 0 = library policy)")
    ap.add_argument("--variant", type=int, default=0, help="kernel form (wsp_plan_set_variant; ablations)")
    ap.add_argument("--chunk", type=int, default=0, help="windows per chunk of the two-pass large-N path (wsp_plan_set_chunk)")
    ap.add_argument("--grid", type=int, default=0, help="workgroups of the FFT-kernel / inverse launch (wsp_plan_set_grid)")
    ap.add_argument("--c5-layout", default="greedy", choices=["length", "greedy", "nlogn"],
                    help="C5: symbols to streams by window length, or greedy by output bytes / by N log N work")
    ap.add_argument("--c5-streams", type=int, default=0,
                    help="C5: lanes the grouped plan runs its launches on (wsp_group_set_streams; 0 = the library's "
                         "default, one per window length up to 4) / streams the symbol plans use (0 = 3)")
    ap.add_argument("--c5-mode", default="group",
                    choices=["group", "group-per-length", "group-mixed-b4", "group-mixed-tail-half", "group-mixed-uniform",
                             "group-mixed-lds-seeds", "group-mixed-plain-stores", "plans"],
                    help="C5: one grouped device plan (wsp_group_*: one mixed-length persistent launch), the grouped "
                         "plan's per-length launches on lanes (round-3 form), the mixed launch with four bins per thread "
                         "for N <= 1024 / half-length segments for the shortest window length at every size / one segment length (wsp_group_set_mode 2 / 3 / 4, "
                         "ablations), or one plan per symbol spread over --c5-streams streams (round-2 form)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-settle", action="store_true", help="skip the clock-settle phase (diagnostics)")
    ap.add_argument("--c5-shard", default="split", choices=["split", "split-time", "symbols"],
                    help="C5 under --scaling strong: cut the symbols' windows on one cost line into equal parts "
                         "(McNaughton wrap-around; cost per window = output bytes, or split-time: the measured "
                         "time per window of each length) or assign whole symbols greedily by output bytes")
    ap.add_argument("--emulate-shard", default="",
                    help="R/G: run exactly rank R's part of the --scaling strong split over G ranks on this one GPU "
                         "(single-GPU emulation of one rank of a G-GPU run, not a scaling measurement)")
    ap.add_argument("--pmc", default="auto", choices=["auto", "on", "off"],
                    help="roofline.traffic from this run: rocprofv3 FETCH_SIZE / WRITE_SIZE passes over a 3-step run "
                         "of the same command, as child processes after the timed region (scripts/pmc_traffic.py); "
                         "auto = on for a one-GPU line with its CPU baseline (the driver's default line and the "
                         "closing check), off for A/B and shard runs, which keep the committed profiles/traffic.json")
    ap.add_argument("--plan-only", action="store_true",
                    help="print every rank's shard of the batch and exit, without touching a GPU (CPU tests)")
    return ap.parse_args(argv)


def dist_env():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args, argv) -> int:
    """--gpus N > 1 outside torchrun: one process per GPU via torch.distributed.run, started as a
    child (this process has not touched the GPU), returning its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(Path(__file__).resolve())] + argv
    return subprocess.call(cmd)


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

    def _reduce(self, v: float, op) -> float:
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, v: float) -> float:
        return v if self.world == 1 else self._reduce(v, self.dist.ReduceOp.MAX)

    def sum(self, v: float) -> float:
        return v if self.world == 1 else self._reduce(v, self.dist.ReduceOp.SUM)

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def timed_steps(step, sync, ctl: Control, steps: int, warmup: int, events=None) -> float:
    """W untimed steps, then K steps bracketed by barrier + device sync; returns max seconds over
    ranks.  `events` = (start, end, stream): HIP events recorded on the launch stream around the
    same K steps."""
    for _ in range(warmup):
        step()
    sync()
    ctl.barrier()
    sync()
    t0 = time.perf_counter()
    if events:
        events[0].record(events[2])
    for _ in range(steps):
        step()
    if events:
        events[1].record(events[2])
    sync()
    ctl.barrier()
    t1 = time.perf_counter()
    return ctl.max(t1 - t0)


def settle(step, stream, batch=8, min_ms=150.0, max_ms=800.0, tol=0.02) -> dict:
    """Untimed clock settle: the MI355X raises its memory clock only under sustained load, so run
    `step` back to back in batches of `batch` launches (one HIP-event pair and one host sync per batch, no gap
    between the launches of a batch) until at least `min_ms` of GPU time has passed and the last three batches'
    per-launch times agree within `tol` (or `max_ms`).  Returns what it did for the JSON line."""
    import torch
    per = []
    total = 0.0
    n = 0
    t0 = time.perf_counter()
    while True:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(batch):
            step()
        b.record(stream)
        b.synchronize()
        ms = a.elapsed_time(b)
        total += ms
        n += batch
        per.append(ms / batch)
        last = per[-3:]
        if total >= min_ms and len(per) >= 3 and max(last) <= (1 + tol) * min(last):
            break
        if total >= max_ms:
            break
    return {"launches": n, "ms": round(total, 2), "first_ms": round(per[0], 4), "last_ms": round(per[-1], 4),
            "wall_s": round(time.perf_counter() - t0, 3)}


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
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/traffic.json), or None; the pass's
    source directory (prof_<tag>_<key>) is kept beside it for the line's traffic_source."""
    p = ROOT / "profiles" / "traffic.json"
    if not p.exists():
        return None
    try:
        e = json.loads(p.read_text()).get(config, {})
    except Exception:
        return None
    TRAFFIC_SOURCE[config] = e.get("source")
    return e.get("hbm_bytes_per_launch")


TRAFFIC_SOURCE = {}


def load_valu(config: str):
    """VALU-issue roofline of a VALU-bound configuration (profiles/valu.json, scripts/valu_roofline.py), or None."""
    p = ROOT / "profiles" / "valu.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text()).get(config)
    except Exception:
        return None
    if not d:
        return None
    return {"kernel": d["kernel"], "issue_frac": d["issue_frac"], "clock_ghz": d["clock_ghz"],
            "valu_insts_per_wave": d.get("valu_insts_per_wave"), "wave_active_frac": d.get("wave_active_frac"),
            "source": d["source"],
            "definition": "4 x SQ_ACTIVE_INST_VALU / (1024 SIMDs x SQ_BUSY_CYCLES / 32): share of the SIMDs' "
                          "4-cycle wave64 VALU issue slots in use (scripts/valu_roofline.py)"}


class Workload:
    """What one rank runs: step() enqueues one step on `stream`; `windows` / `alg_bytes` are this
    rank's per step."""
    stream = None
    windows = 0
    alg_bytes = 0
    describe = ""
    cpu_cfg = None      # (series tensor, cfg) for the CPU baseline
    traffic = None      # PMC HBM bytes per step, from profiles/traffic.json
    valu = None         # VALU-issue roofline (VALU-bound configurations), from profiles/valu.json

    def step(self):
        raise NotImplementedError

    def close(self):
        pass


C5_BARS, C5_LENS = 20000, (512, 1024, 2048, 4096)
# C5 cost per window of each length for --c5-shard split-time, in units of 10 ps per window: round 5 calibrated them at
# shard scale from the G = 8 emulation of the final tree (profiles/r05/shards.json, ranks holding one or two lengths
# solved for per-window times: 0.48 / 0.96 / 1.94 / 4.14 ns) -- a 4096-point window costs ~7 % more per output byte
# than the shorter ones at one round of tasks (its seed is the longest); round 3's whole-batch kernel trace gave
# {512: 51, 1024: 92, 2048: 187, 4096: 336}
C5_TIME_WEIGHTS = {512: 48, 1024: 96, 2048: 194, 4096: 414}


def c5_symbols():
    """(window length, window count) of C5's 28 symbols: 7 per length, 20000 bars each."""
    return [(C5_LENS[s // 7], C5_BARS - C5_LENS[s // 7] + 1) for s in range(28)]


def shard_plan(name: str, rank: int, world: int, scaling: str, c5_shard: str = "split") -> dict:
    """This rank's part of a configuration: windows [w0, w0+nw) and series samples [a, b) (the
    N - hop halo included) of one batch (strong), or a whole batch of its own (weak); for C5 the
    pieces (symbol, first window, windows) it owns."""
    from wavespec_amd import sharding, synth
    if name == "c5":
        syms = c5_symbols()
        nwins = [nw for _, nw in syms]
        if scaling != "strong":
            pieces = [(s, 0, nw) for s, nw in enumerate(nwins)]
        elif c5_shard == "symbols":
            owned = sharding.shard_symbols([nw * n // 2 for n, nw in syms], world, rank)
            pieces = [(s, 0, nwins[s]) for s in owned]
        else:
            cost = [n // 2 if c5_shard == "split" else C5_TIME_WEIGHTS[n] for n, _ in syms]
            pieces = [tuple(p) for p in sharding.split_symbols(cost, nwins, world, rank)]
        return {"rank": rank, "symbols": sorted({p[0] for p in pieces}), "pieces": [list(p) for p in pieces],
                "windows": sum(p[2] for p in pieces), "split": c5_shard if scaling == "strong" else None,
                "seed_offset": 0 if scaling == "strong" else 1000 * rank}
    cfg = synth.CONFIGS[name]
    w, n, hop = cfg["windows"], cfg["n"], cfg["hop"]
    if scaling == "strong":
        w0, nw = sharding.shard_windows(w, world, rank)
        seed = cfg["seed"]
    else:
        w0, nw, seed = 0, w, cfg["seed"] + 1000 * rank
    a, b = (w0 * n, (w0 + nw) * n) if cfg.get("output") == "inverse" else sharding.shard_series_slice(w0, nw, hop, n)
    return {"rank": rank, "w0": w0, "windows": nw, "series": [a, b], "seed": seed, "of": w}


class SingleBatch(Workload):
    """One plan over one window batch (every config but C5)."""

    def __init__(self, name, rank, local_rank, world, scaling, algo="auto", slide_seg=0, variant=0, chunk=0,
                 seed_chain=0, grid=0):
        import torch
        from wavespec_amd import bridge, synth
        cfg = dict(synth.CONFIGS[name])
        cfg.setdefault("trend_period", 0)
        if os.environ.get("WSP_BENCH_WINDOW"):  # ablation only: another window on the same batch (not a BASELINE config)
            cfg["window"] = os.environ["WSP_BENCH_WINDOW"]
        dev = torch.device("cuda", local_rank)
        n, hop, w = cfg["n"], cfg["hop"], cfg["windows"]
        f32 = cfg["precision"] == "f32"
        tdt = torch.float32 if f32 else torch.float64
        output = cfg.get("output", "power")
        sp = shard_plan(name, rank, world, scaling)  # this rank's window range (+ halo) or its own batch
        w0, nw, seed = sp["w0"], sp["windows"], sp["seed"]
        a, b = sp["series"]
        if nw <= 0:
            raise SystemExit(f"rank {rank}: no windows to own ({w} windows over {world} ranks)")
        if output == "inverse":  # rows of packed spectra (random, resident in HBM)
            gen = torch.Generator(device=dev)
            gen.manual_seed(seed)
            full = torch.randn(w * n, dtype=tdt, device=dev, generator=gen)
            self.series = full[a:b].contiguous() if (a, b) != (0, full.numel()) else full
            self.plan = bridge.Plan.inverse(local_rank, n, nw)
            if variant:
                self.plan.set_variant(variant)
            if grid:
                self.plan.set_grid(grid)
        else:
            full = synth.random_walk_torch((w - 1) * hop + n, seed, dev, tdt)  # resident in HBM
            self.series = full[a:b].contiguous() if (a, b) != (0, full.numel()) else full
            self.plan = bridge.Plan(local_rank, n, hop, nw, cfg["detrend"], cfg["window"], cfg["trend_period"],
                                    cfg["precision"], output)
            if output in ("topk", "topk_phase"):
                self.plan.set_topk(8, 18.0, 200.0)  # the reference's scan (1.1.0:22-23)
            if algo != "auto":
                self.plan.set_algorithm(algo)
            if slide_seg:
                self.plan.set_slide_segment(slide_seg)
            if variant:
                self.plan.set_variant(variant)
            if seed_chain:
                self.plan.set_seed_chain(seed_chain)
            if chunk:
                self.plan.set_chunk(chunk)
            if grid:
                self.plan.set_grid(grid)
        self.algorithm = self.plan.algorithm() if output != "inverse" else "inverse"
        del full
        self.out = torch.empty(nw * self.plan.record, dtype=tdt, device=dev)
        self.stream = torch.cuda.current_stream(dev)
        self._sptr = self.stream.cuda_stream
        self._args = (self.series.data_ptr(), self.out.data_ptr(), self._sptr)
        self.windows = nw
        self.alg_bytes = self.plan.algorithmic_bytes
        self.f32 = f32
        self.cfg = cfg
        self.cpu_cfg = (self.series, cfg)
        self.traffic = load_traffic(name if algo == "auto" else f"{name}_{algo}") if scaling != "strong" else None
        self.valu = load_valu(name) if (algo, variant) == ("auto", 0) else None
        shard = f", windows [{w0}, {w0 + nw}) of {w}" if scaling == "strong" else ""
        self.describe = (f"{name}: {w} windows x {n}-pt, hop={hop}, {cfg['precision']}, {cfg['detrend']} detrend, "
                         f"{cfg['window']} window, " + {
                             "power": "|X|^2 k<N/2", "topk": "top-8 bins in periods [18, 200]",
                             "phase": "[|X|^2, unwrapped phase, group delay] k<N/2",
                             "topk_phase": "top-8 bins + phase/delay in periods [18, 200]",
                             "inverse": "inverse real FFT of packed spectra"}[output] + shard)
        self.n, self.hop = n, hop

    def step(self):
        self.plan.execute(*self._args)

    def close(self):
        self.plan.close()


class C5Batch(Workload):
    """C5: 28 symbols x 20000 bars, N in {512,1024,2048,4096} (7 symbols each), hop = 1, fp64,
    Hann -- the WaveCyclesBatchFetcher shape (WaveCyclesBatchFetcher.mq5:106-133: one batch per
    symbol).  One step = every owned piece's batch (a whole symbol, or under --scaling strong a
    window range of one with its N - 1 halo).  Default (--c5-mode group): one grouped device plan
    (wsp_group_*), the pieces of each window length in one sliding-DFT launch on the launch
    stream.  --c5-mode plans: one plan per piece, spread over --c5-streams streams joined into the
    launch stream (the round-2 form)."""

    def __init__(self, rank, local_rank, world, scaling, algo="auto", slide_seg=0, c5_layout="greedy", c5_streams=3,
                 c5_mode="group", c5_shard="split"):
        import torch
        from wavespec_amd import bridge, synth
        dev = torch.device("cuda", local_rank)
        syms = c5_symbols()
        sp = shard_plan("c5", rank, world, scaling, c5_shard)
        pieces, seed_off = [tuple(p) for p in sp["pieces"]], sp["seed_offset"]
        self.f32 = False
        self.stream = torch.cuda.current_stream(dev)
        self.group = None
        self.describe = (f"c5: 28 symbols x {C5_BARS} bars, N in {C5_LENS} (7 each), hop=1, f64, Hann, |X|^2"
                         + (f", rank {rank}/{world} of a {c5_shard} split: {len(pieces)} pieces of "
                            f"{len(sp['symbols'])} symbols" if scaling == "strong" else ""))
        full = {}

        def piece_series(sym, w0, nw):  # the symbol's bars, then the piece's windows + N - 1 halo (resident in HBM)
            if sym not in full:
                full[sym] = synth.random_walk_torch(C5_BARS, 100 + sym + seed_off, dev)
            x = full[sym]
            n = syms[sym][0]
            return x if (w0, nw) == (0, syms[sym][1]) else x[w0: w0 + nw - 1 + n].contiguous()

        lens = [syms[p[0]][0] for p in pieces]
        if c5_mode.startswith("group") and algo in ("auto", "slide"):
            self.series = [piece_series(*p) for p in pieces]
            self.outs = [torch.empty(p[2] * (n // 2), dtype=torch.float64, device=dev) for p, n in zip(pieces, lens)]
            self.group = bridge.Group(local_rank, lens, [p[2] for p in pieces])
            if c5_mode == "group-per-length":
                self.group.set_mode("per-length")
            elif c5_mode in ("group-mixed-b4", "group-mixed-tail-half", "group-mixed-uniform", "group-mixed-lds-seeds",
                             "group-mixed-plain-stores"):
                self.group.set_mode(c5_mode[len("group-"):])
            if c5_streams:
                self.group.set_streams(c5_streams)
            if slide_seg:
                self.group.set_segment(slide_seg)
            self._ptrs = ([x.data_ptr() for x in self.series], [o.data_ptr() for o in self.outs])
            self.algorithm = "slide-group" + {"group-per-length": "-per-length", "group-mixed-b4": "-mixed-b4", "group-mixed-tail-half": "-mixed-tail-half", "group-mixed-uniform": "-mixed-uniform", "group-mixed-lds-seeds": "-mixed-lds-seeds", "group-mixed-plain-stores": "-mixed-plain-stores"}.get(c5_mode, "")
            self.layout = {"mode": "group", "launches": self.group.launches, "streams": c5_streams or "library default",
                           "segment": slide_seg or "auto", "pieces": len(pieces)}
            self.windows = sum(p[2] for p in pieces)
            self.alg_bytes = self.group.algorithmic_bytes
            self.traffic = load_traffic("c5") if scaling != "strong" else None
            i4 = [i for i, n in enumerate(lens) if n == 4096]
            i = i4[-1] if i4 else len(pieces) - 1
            self.cpu_cfg = (self.series[i], {"n": lens[i], "hop": 1, "windows": pieces[i][2], "detrend": "none",
                                             "window": "hann"})
            full.clear()
            return
        # Three streams, within the box's 4 HIP hardware queues together with the launch stream (with
        # one stream per length two of them shared a hardware queue and ran 14 kernels back to back:
        # the whole step, profiles/r02/c5_kernel_stats.csv).  --c5-layout: "length" puts {4096}, {2048},
        # {1024, 512} on their own streams; "greedy" assigns pieces longest-first to the least-loaded
        # stream by output bytes (what the hop = 1 sliding DFT's time follows: nwin x N/2), "nlogn" the
        # same by windows x N log N (the FFT kernel's work).  --c5-streams 1 runs every piece on one
        # stream (ablation).
        nstreams = c5_streams or 3
        self.streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
        if c5_layout == "nlogn":
            cost = [p[2] * n * int(np.log2(n)) for p, n in zip(pieces, lens)]
        else:
            cost = [p[2] * (n // 2) for p, n in zip(pieces, lens)]
        order = sorted(range(len(pieces)), key=lambda i: -cost[i])
        load, assign = [0] * nstreams, {}
        if c5_layout in ("greedy", "nlogn"):
            for i in order:
                k = load.index(min(load))
                assign[i] = k
                load[k] += cost[i]
        else:  # by window length: {4096}, {2048}, {1024, 512}
            for i in order:
                assign[i] = {4096: 0, 2048: 1, 1024: 2, 512: 2}[lens[i]] % nstreams
        self.layout = {"layout": c5_layout, "streams": nstreams,
                       "stream_load": [sum(cost[i] for i in order if assign[i] == k) for k in range(nstreams)]}
        self.jobs = []  # (plan, series, out, stream), launched longest first
        for i in order:
            n, nw = lens[i], pieces[i][2]
            series = piece_series(*pieces[i])
            out = torch.empty(nw * (n // 2), dtype=torch.float64, device=dev)
            plan = bridge.Plan(local_rank, n, 1, nw, "none", "hann")
            if algo != "auto":
                plan.set_algorithm(algo)
            if slide_seg:
                plan.set_slide_segment(slide_seg)
            self.jobs.append((plan, series, out, self.streams[assign[i]]))
        full.clear()
        self.algorithm = "+".join(sorted({j[0].algorithm() for j in self.jobs}))
        self.windows = sum(j[0].n_windows for j in self.jobs)
        self.alg_bytes = sum(j[0].algorithmic_bytes for j in self.jobs)
        self.traffic = load_traffic("c5_plans" if algo == "auto" else f"c5_{algo}") if scaling != "strong" else None
        big = [j for j in self.jobs if j[0].window_len == 4096] or self.jobs
        p0, s0 = big[-1][0], big[-1][1]
        self.cpu_cfg = (s0, {"n": p0.window_len, "hop": 1, "windows": p0.n_windows, "detrend": "none",
                             "window": "hann"})

    def step(self):
        if self.group is not None:
            self.group.execute(*self._ptrs, self.stream.cuda_stream)
            return
        for st in self.streams:
            st.wait_stream(self.stream)
        for plan, series, out, st in self.jobs:
            plan.execute(series.data_ptr(), out.data_ptr(), st.cuda_stream)
        for st in self.streams:
            self.stream.wait_stream(st)

    def close(self):
        if self.group is not None:
            self.group.close()
            return
        for j in self.jobs:
            j[0].close()


def want_pmc(args) -> bool:
    """--pmc auto: this run's traffic for a one-GPU line that carries its CPU baseline (the driver's default line,
    the closing check's lines), never inside a PMC child or for an emulated shard."""
    if os.environ.get("WSP_BENCH_PMC_CHILD") or args.emulate_shard:
        return False
    return args.pmc == "on" or (args.pmc == "auto" and not args.no_cpu_baseline)


def run_pmc(args, argv):
    """rocprofv3 FETCH_SIZE and WRITE_SIZE passes (each its own child run, scripts/pmc_traffic.py) over 3 steps of
    this same command; the per-step bytes, or None (no rocprofv3, a failed or timed-out pass)."""
    sys.path.insert(0, str(ROOT / "scripts"))
    import pmc_traffic
    drop = {"--steps": 1, "--warmup": 1, "--pmc": 1, "--cpu-seconds": 1, "--no-cpu-baseline": 0, "--no-settle": 0}
    rest, i = [], 0
    while i < len(argv):
        a = argv[i]
        name = a.split("=", 1)[0]
        if name in drop:
            i += 1 + (drop[name] if "=" not in a else 0)
            continue
        rest.append(a)
        i += 1
    cmd = [sys.executable, str(Path(__file__).resolve())] + rest + ["--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                                                                    "--no-settle", "--pmc", "off"]
    key = pmc_traffic.bench_key(args.config, args.algo, args.variant, args.c5_mode)
    return pmc_traffic.collect(cmd, args.config, key)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    rank, local_rank, world = dist_env()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, argv)
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU")
    shard_rank, shard_world, scaling = rank, world, args.scaling
    if args.emulate_shard:
        try:
            shard_rank, shard_world = (int(v) for v in args.emulate_shard.split("/"))
        except ValueError:
            raise SystemExit("--emulate-shard takes R/G, e.g. 3/8")
        if world != 1 or not 0 <= shard_rank < shard_world:
            raise SystemExit("--emulate-shard R/G runs one rank's shard on one GPU: 0 <= R < G, --gpus 1")
        scaling = "strong"
    if args.plan_only:
        ctl = Control(world)
        mine = shard_plan(args.config, shard_rank, shard_world, scaling, args.c5_shard)
        parts = [mine]
        if world > 1:
            parts = [None] * world
            ctl.dist.all_gather_object(parts, mine)
        if rank == 0:
            print(json.dumps({"n_gpus": world, "config": args.config, "scaling": scaling, "shards": parts}),
                  flush=True)
        ctl.close()
        return 0
    import torch

    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    ctl = Control(world)
    if args.config == "c5":
        wl = C5Batch(shard_rank, local_rank, shard_world, scaling, args.algo, args.slide_seg, args.c5_layout,
                     args.c5_streams, args.c5_mode, args.c5_shard)
    else:
        wl = SingleBatch(args.config, shard_rank, local_rank, shard_world, scaling, args.algo, args.slide_seg,
                         args.variant, args.chunk, args.seed_chain, args.grid)
    torch.cuda.synchronize()

    settled = None if args.no_settle else settle(wl.step, wl.stream)
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True), wl.stream)
    secs = timed_steps(wl.step, torch.cuda.synchronize, ctl, args.steps, args.warmup, ev)
    kernel_s = ev[0].elapsed_time(ev[1]) / 1e3 / args.steps  # this rank, same K steps, launch stream
    kernel_s_max = ctl.max(kernel_s)
    achieved = wl.alg_bytes / kernel_s / 1e9

    total_windows = ctl.sum(float(wl.windows * args.steps))
    value = total_windows / secs
    baseline = baseline_all = None
    # The CPU baseline beside every line (north star: "next to the reference CPU path timed on the GPU
    # box's own host cores in the same run"), on rank 0 after the timed region, so it never overlaps the
    # GPU timing; with N > 1 ranks the sample is halved to keep the driver's 1/2/4/8 sweep short.
    if rank == 0 and not args.no_cpu_baseline and wl.cpu_cfg is not None:
        budget = args.cpu_seconds if world == 1 else args.cpu_seconds / 2
        baseline = cpu_baseline(wl.cpu_cfg[0], wl.cpu_cfg[1], budget)
        baseline_all = cpu_baseline(wl.cpu_cfg[0], wl.cpu_cfg[1], budget / 2, cpu_threads())

    pmc = None
    if rank == 0 and world == 1 and want_pmc(args):
        pmc = run_pmc(args, argv)
    if pmc:
        traffic, traffic_source = pmc["hbm_bytes_per_launch"], (
            "this run: " + pmc["method"] + " -- child processes of this bench.py after its timed region, over 3 steps "
            "of the same command (scripts/pmc_traffic.py)")
    else:
        traffic = wl.traffic
        traffic_source = ("profiles/traffic.json (rocprofv3 FETCH_SIZE / WRITE_SIZE passes of a separate run of the same "
                          "command, scripts/parse_prof.py"
                          + (f", {next(v for v in TRAFFIC_SOURCE.values() if v)}" if any(TRAFFIC_SOURCE.values()) else "")
                          + "), not this run") if wl.traffic else None

    if rank == 0:
        valu_bound = bool(wl.valu) and wl.valu["issue_frac"] >= 0.7  # VALU-issue-bound (profiles/valu.json)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "windows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": secs / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32" if wl.f32 else "f64",
            "data": "synthetic (random-walk close prices generated on device, seed per rank)",
            "config": {"workload": wl.describe, "windows_per_gpu": wl.windows, "windows_total": int(total_windows / args.steps),
                       "parallelism": f"windows sharded x{world} ({args.scaling}), no collective",
                       "algorithm": wl.algorithm, **({"c5": wl.layout} if hasattr(wl, "layout") else {})},
            "roofline": {"bound": "valu" if valu_bound else "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_source,
                         **({"traffic_read_bytes": pmc["read_bytes_corrected"], "traffic_write_bytes": pmc["write_bytes"]}
                            if pmc else {}),
                         **({"valu": wl.valu, "note": ("VALU-issue-bound: achieved / frac are the HBM roofline, "
                                                       "valu.issue_frac the bound's") if valu_bound else
                             ("dominant kernel below 0.7 of the VALU issue slots (dependency waits and its own IO): "
                              "reported against HBM, valu beside it")} if wl.valu else {}),
                         "algorithmic_bytes_per_launch": wl.alg_bytes, "kernel_ms": kernel_s * 1e3,
                         "kernel_ms_max_over_ranks": kernel_s_max * 1e3,
                         "timing": "HIP events on the launch stream around the same K timed steps (rank 0)"},
            "settle": settled,
            **({"emulated_shard": {"rank": shard_rank, "of": shard_world, "split": args.c5_shard if args.config == "c5" else "windows",
                                   "caveat": "single-GPU emulation of one rank of a strong-scaled run, not a scaling "
                                             "measurement"}} if args.emulate_shard else {}),
            "cpu_baseline": baseline,
            "cpu_baseline_all_cores": baseline_all,
        }
        print(json.dumps(line), flush=True)
    wl.close()
    ctl.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
