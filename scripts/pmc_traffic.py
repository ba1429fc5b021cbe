"""HBM bytes per bench step from rocprofv3 PMC passes, as MI355X_MICROARCH.md's HBM section prescribes:
FETCH_SIZE and WRITE_SIZE each in a pass of its own (they cannot share one: 3 + 2 TCC counters of 4),
read bytes = FETCH_SIZE (KiB) x 1024 x 2 (gfx950 reports half of a wide coalesced streaming read),
write bytes = WRITE_SIZE (KiB) x 1024.

Used by scripts/parse_prof.py (the committed profiles/traffic.json entries) and by bench.py, which runs
the two passes on its own command as child processes after its timed region (`collect`), so that the
line's roofline.traffic is this run's.  Measurement infrastructure: nothing here is on the product path.
"""
from __future__ import annotations

import csv
import glob
import os
import shutil
import signal
import subprocess
import sys
import tempfile
from pathlib import Path

OURS = ("spectrum_kernel", "slide_kernel", "slide_mixed_kernel", "slide_topk_kernel", "slide_topk_t_kernel",
        "slide_topk_p_kernel", "slide_seed_kernel", "slide_seed_r_kernel", "fused_kernel", "kalman_detrend_kernel",
        "kalman_pk2_kernel", "kalman_pk4_kernel", "inverse_kernel", "inverse_direct_kernel", "col_kernel", "row_kernel",
        "mean_kernel", "iir_kernel")
MAIN = ("spectrum_kernel", "slide_kernel", "slide_mixed_kernel", "slide_topk_kernel", "slide_topk_t_kernel",
        "slide_topk_p_kernel", "inverse_kernel", "inverse_direct_kernel", "row_kernel",
        "fused_kernel")  # one per step; a Kalman pre-pass adds to its step
METHOD = ("rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; all our kernels' dispatches summed per "
          "main (spectrum/inverse) dispatch; read = FETCH_SIZE*1024*2 (gfx950 half-count correction), "
          "write = WRITE_SIZE*1024")


def main_per_step(cfg: str, key: str) -> int:
    """Main-kernel dispatches per bench step: 1, the chunk count of the four-step large-N path
    (one row_kernel per chunk of windows, csrc/large_fft.hip large_chunk: 192 MiB of column results),
    or C5's launches."""
    if cfg == "c5":  # grouped plan: one mixed-length launch (per-length form: one per window length); per-symbol plans: 28
        return 28 if key.endswith(("_plans", "_fft")) else (4 if key.endswith("_per_length") else 1)
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "fft-wavespec_amd"))
    from wavespec_amd import synth
    c = synth.CONFIGS.get(cfg)
    if not c or c["n"] <= 16384:
        return 1
    if c["n"] == 65536 and c["precision"] == "f64" and not key.endswith(("_v1", "_v2", "_v4")):
        return 1  # the fused kernel: one launch over every window (large_fft.hip)
    per = (c["n"] // 2) * (8 if c["precision"] == "f32" else 16)
    chunk = max(1, (192 << 20) // per)
    return -(-c["windows"] // chunk)


def rows(pattern: str) -> list:
    return [r for f in glob.glob(pattern, recursive=True) for r in csv.DictReader(open(f))]


def counter_per_step(rs: list, counter: str, cfg: str, key: str):
    """Counter value per step: every dispatch of our kernels summed, divided by the number of main-kernel
    dispatches, times the main dispatches per step (C3's Kalman pre-pass traffic belongs to the step it
    feeds; a large-N step is several chunks)."""
    rs = [r for r in rs if r.get("Counter_Name") == counter]
    vals = [float(r["Counter_Value"]) for r in rs if any(k in r.get("Kernel_Name", "") for k in OURS)]
    n_main = sum(1 for r in rs if any(k in r.get("Kernel_Name", "") for k in MAIN))
    return sum(vals) / n_main * main_per_step(cfg, key) if n_main else None


def summarize(fetch_rows: list, write_rows: list, cfg: str, key: str) -> dict:
    res = {}
    fetch = counter_per_step(fetch_rows, "FETCH_SIZE", cfg, key)
    write = counter_per_step(write_rows, "WRITE_SIZE", cfg, key)
    if fetch is not None:
        res["fetch_size_kib_raw"] = fetch
        res["read_bytes_corrected"] = fetch * 1024 * 2
    if write is not None:
        res["write_size_kib_raw"] = write
        res["write_bytes"] = write * 1024
    if fetch is not None and write is not None:
        res["hbm_bytes_per_launch"] = res["read_bytes_corrected"] + res["write_bytes"]
        res["method"] = METHOD
    return res


def bench_key(cfg: str, algo: str = "auto", variant: int = 0, c5_mode: str = "group") -> str:
    """The traffic.json key of a bench.py configuration (scripts/gpu_profile.sh's naming)."""
    key = cfg if algo == "auto" else f"{cfg}_{algo}"
    if cfg == "c5" and c5_mode in ("plans", "group-per-length"):
        key += "_plans" if c5_mode == "plans" else "_per_length"
    return key if not variant else f"{key}_v{variant}"


def _pass(counter: str, cmd: list, workdir: str, timeout: float) -> list | None:
    """One `rocprofv3 --pmc <counter> --kernel-trace` pass over cmd (a child process in its own process group,
    killed whole at the time limit); the counter rows, or None."""
    out = os.path.join(workdir, counter.lower())
    full = ["rocprofv3", "--pmc", counter, "--kernel-trace", "--output-format", "csv", "-d", out, "-o", "run", "--"] + cmd
    env = dict(os.environ, WSP_BENCH_PMC_CHILD="1")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "MASTER_ADDR",
              "MASTER_PORT"):  # a torchrun parent's rendezvous is not the child's: it runs as a lone rank
        env.pop(k, None)
    try:
        p = subprocess.Popen(full, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env, start_new_session=True)
    except OSError:
        return None
    try:
        rc = p.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
        p.wait()
        return None
    if rc != 0:
        return None
    r = rows(os.path.join(out, "**", "*counter_collection.csv"))
    return r or None


def collect(cmd: list, cfg: str, key: str, timeout: float = 120.0) -> dict | None:
    """FETCH_SIZE and WRITE_SIZE passes over `cmd` (a short bench.py run of the same configuration), each in
    its own rocprofv3 run; the summarize() dict, or None when rocprofv3 is missing or a pass fails."""
    if shutil.which("rocprofv3") is None:
        return None
    work = tempfile.mkdtemp(prefix="wsp_pmc_")
    try:
        f = _pass("FETCH_SIZE", cmd, work, timeout)
        w = _pass("WRITE_SIZE", cmd, work, timeout) if f else None
        if not f or not w:
            return None
        res = summarize(f, w, cfg, key)
        return res if "hbm_bytes_per_launch" in res else None
    finally:
        shutil.rmtree(work, ignore_errors=True)
