"""Summarises a scripts/gpu_profile.sh output directory.

Prints per-kernel average duration of our kernels (kernel trace) and the HBM
bytes per launch from the PMC passes, corrected as MI355X_MICROARCH.md
sec. HBM prescribes: FETCH_SIZE (KiB) x 1024 x 2 (gfx950 reports half of a
wide coalesced streaming read), WRITE_SIZE (KiB) x 1024.  Merges the result
into profiles/traffic.json under the config name (or the key given as a third argument).
"""
import csv
import glob
import json
import sys
from pathlib import Path

out, cfg = Path(sys.argv[1]), sys.argv[2]
key = sys.argv[3] if len(sys.argv) > 3 else cfg  # e.g. c4_fft: the config under a forced algorithm
OURS = ("spectrum_kernel", "slide_kernel", "slide_mixed_kernel", "slide_topk_kernel", "slide_topk_t_kernel", "slide_topk_p_kernel", "slide_seed_kernel", "slide_seed_r_kernel", "fused_kernel", "kalman_detrend_kernel", "kalman_pk2_kernel", "kalman_pk4_kernel", "inverse_kernel", "inverse_direct_kernel", "col_kernel", "row_kernel", "mean_kernel",
        "iir_kernel")
MAIN = ("spectrum_kernel", "slide_kernel", "slide_mixed_kernel", "slide_topk_kernel", "slide_topk_t_kernel", "slide_topk_p_kernel", "inverse_kernel", "inverse_direct_kernel", "row_kernel",
        "fused_kernel")  # one per step; a Kalman pre-pass adds to its step


def rows(pattern):
    files = glob.glob(str(out / pattern), recursive=True)
    return [r for f in files for r in csv.DictReader(open(f))]


res = {}
for r in rows("trace/**/*kernel_stats.csv"):
    if any(k in r["Name"] for k in OURS):
        res.setdefault("kernels", {})[r["Name"][:120]] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                                          "min_us": float(r["MinNs"]) / 1e3}


def main_per_step(cfg):
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


def pmc(pattern, counter):
    """Counter bytes per step: every dispatch of our kernels summed, divided by the number of
    main-kernel dispatches, times the main dispatches per step (C3's Kalman pre-pass traffic belongs
    to the step it feeds; a large-N step is several chunks)."""
    rs = [r for r in rows(pattern) if r.get("Counter_Name") == counter]
    vals = [float(r["Counter_Value"]) for r in rs if any(k in r.get("Kernel_Name", "") for k in OURS)]
    n_main = sum(1 for r in rs if any(k in r.get("Kernel_Name", "") for k in MAIN))
    return sum(vals) / n_main * main_per_step(cfg) if n_main else None


fetch = pmc("fetch/**/*counter_collection.csv", "FETCH_SIZE")
write = pmc("write/**/*counter_collection.csv", "WRITE_SIZE")
if fetch is not None:
    res["fetch_size_kib_raw"] = fetch
    res["read_bytes_corrected"] = fetch * 1024 * 2
if write is not None:
    res["write_size_kib_raw"] = write
    res["write_bytes"] = write * 1024
if fetch is not None and write is not None:
    res["hbm_bytes_per_launch"] = res["read_bytes_corrected"] + res["write_bytes"]
    res["method"] = ("rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; all our kernels' dispatches "
                     "summed per main (spectrum/inverse) dispatch; read = FETCH_SIZE*1024*2 (gfx950 half-count "
                     "correction), write = WRITE_SIZE*1024")
res["source"] = out.name  # the gpurun_out directory of the passes (gpu_profile.sh: prof_<tag>_<key>)
print(json.dumps(res, indent=1))
tj = Path("profiles/traffic.json")
allres = json.loads(tj.read_text()) if tj.exists() else {}
allres[key] = res
tj.parent.mkdir(exist_ok=True)
tj.write_text(json.dumps(allres, indent=1))
