"""LDS bank-conflict share per kernel of ours from gpu_run.sh `sq` passes (rocprofv3 --pmc SQ_LDS_BANK_CONFLICT
SQ_LDS_IDX_ACTIVE ...): conflict cycles / all LDS-array cycles (MI355X_MICROARCH.md LDS section), summed over the
dispatches of each kernel.

    python scripts/lds_conflicts.py <gpurun_out/tag> [out.json]
"""
import csv
import glob
import json
import sys
from collections import defaultdict

OURS = ("spectrum_kernel", "slide_kernel", "slide_mixed_kernel", "slide_topk", "slide_seed", "fused_kernel",
        "kalman_", "inverse_", "col_kernel", "row_kernel")


def short(name):
    for k in OURS:
        if k in name:
            i = name.find(k)
            return name[i:i + 90]
    return None


def main():
    d = sys.argv[1]
    res = {}
    for f in sorted(glob.glob(f"{d}/sq_*/**/*counter_collection.csv", recursive=True)):
        cfg = f.split("/sq_")[1].split("/")[0]
        acc = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        for k, c in acc.items():
            conf, act = c.get("SQ_LDS_BANK_CONFLICT", 0.0), c.get("SQ_LDS_IDX_ACTIVE", 0.0)
            res[f"{cfg}: {k}"] = {"bank_conflict_cycles": conf, "lds_active_cycles": act,
                                  "conflict_share": round(conf / act, 4) if act else None}
            print(f"{cfg:14s} {k[:70]:70s} conflict/active = {res[f'{cfg}: {k}']['conflict_share']}")
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
