#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 SQ counter pass (gpu_run.sh sq= / sqv= steps).

    python scripts/sq_summary.py <run_counter_collection.csv> [...]

Per wsp:: kernel, averaged over its dispatches: traced duration, VALU instructions per wave, the share of
the SIMDs' 4-cycle VALU issue slots in use (scripts/valu_roofline.py's issue_frac), and the waits as a
share of the waves' cycles (SQ_WAIT_ANY: any wait; SQ_WAIT_INST_ANY: waiting for an instruction's
dependency)."""
import collections
import csv
import json
import sys

SIMDS, SES = 1024, 32
out = {}
for path in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "wsp::" not in k:
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        acc[k]["_dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    res = {}
    for k, d in acc.items():
        m = {c: sum(x) / len(x) for c, x in d.items()}
        e = {"dur_us": round(m["_dur_us"], 1)}
        if "SQ_BUSY_CYCLES" in m and "SQ_ACTIVE_INST_VALU" in m:
            e["valu_issue_frac"] = round(4 * m["SQ_ACTIVE_INST_VALU"] / (SIMDS * m["SQ_BUSY_CYCLES"] / SES), 3)
        if "SQ_WAVES" in m:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM"):
                if c in m:
                    e[c.lower() + "_per_wave"] = round(m[c] / m["SQ_WAVES"])
        if "SQ_WAVE_CYCLES" in m:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                if c in m:
                    e[c.lower() + "_frac"] = round(m[c] / m["SQ_WAVE_CYCLES"], 3)
        res[k.split("(")[0]] = e
    out[path] = res
print(json.dumps(out, indent=1))
