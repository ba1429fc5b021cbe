"""Summarises a scripts/gpu_profile.sh output directory.

Prints per-kernel average duration of our kernels (kernel trace) and the HBM
bytes per launch from the PMC passes, corrected as MI355X_MICROARCH.md
sec. HBM prescribes: FETCH_SIZE (KiB) x 1024 x 2 (gfx950 reports half of a
wide coalesced streaming read), WRITE_SIZE (KiB) x 1024 (scripts/pmc_traffic.py).
Merges the result into profiles/traffic.json under the config name (or the key given as a third argument).
"""
import csv
import glob
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import pmc_traffic  # noqa: E402

out, cfg = Path(sys.argv[1]), sys.argv[2]
key = sys.argv[3] if len(sys.argv) > 3 else cfg  # e.g. c4_fft: the config under a forced algorithm

res = {}
for f in glob.glob(str(out / "trace/**/*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in pmc_traffic.OURS):
            res.setdefault("kernels", {})[r["Name"][:120]] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                                              "min_us": float(r["MinNs"]) / 1e3}
res.update(pmc_traffic.summarize(pmc_traffic.rows(str(out / "fetch/**/*counter_collection.csv")),
                                 pmc_traffic.rows(str(out / "write/**/*counter_collection.csv")), cfg, key))
res["source"] = out.name  # the gpurun_out directory of the passes (gpu_profile.sh: prof_<tag>_<key>)
print(json.dumps(res, indent=1))
tj = Path("profiles/traffic.json")
allres = json.loads(tj.read_text()) if tj.exists() else {}
allres[key] = res
tj.parent.mkdir(exist_ok=True)
tj.write_text(json.dumps(allres, indent=1))
