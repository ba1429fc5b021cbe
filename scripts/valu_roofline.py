#!/usr/bin/env python3
"""VALU-issue roofline of the VALU-bound configurations from rocprofv3 SQ counter passes.

    python scripts/valu_roofline.py [<cfg>=<sq csv> ...]   (default: the committed profiles/r04/sq passes)

Writes profiles/valu.json, which bench.py reads into `roofline.valu` for those configurations (their
`roofline.bound` is then "valu"; the HBM fraction stays beside it).  Per kernel and dispatch:

  kernel cycles    = SQ_BUSY_CYCLES / 32 (the counter sums the chip's 32 shader engines: over the traced
                     dispatch durations this gives 2.0-2.1 GHz, the MI355X engine clock under load)
  issue_frac       = 4 * SQ_ACTIVE_INST_VALU / (1024 SIMDs * kernel cycles)
                     SQ_ACTIVE_INST_VALU counts quad-cycles with a VALU instruction issuing; it is ~1.0 per
                     SQ_INSTS_VALU here, i.e. 4 cycles per wave64 instruction -- the fp64 rate of a SIMD and what
                     one wave alone sustains for any VALU op (MI355X_MICROARCH.md constants table) -- so
                     issue_frac is the share of the SIMDs' 4-cycle VALU issue slots in use
  wave_active_frac = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (per wave: VALU-active share of its lifetime)
"""
from __future__ import annotations

import collections
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
DEFAULT = {"c3": "profiles/r04/sq/c3_sq_counters.csv", "c4_topk": "profiles/r04/sq/c4_topk_sq_counters.csv"}
SIMDS, SES = 1024, 32


def summarize(path: Path) -> dict:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "wsp::" not in k:
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        acc[k]["_dur_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {}
    for k, d in acc.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        if "SQ_ACTIVE_INST_VALU" not in m or "SQ_BUSY_CYCLES" not in m:
            continue
        cyc = m["SQ_BUSY_CYCLES"] / SES
        e = {"dispatches": len(d["SQ_BUSY_CYCLES"]), "dur_us": m["_dur_ns"] / 1e3,
             "clock_ghz": cyc / m["_dur_ns"], "valu_insts": m.get("SQ_INSTS_VALU"),
             "issue_frac": 4 * m["SQ_ACTIVE_INST_VALU"] / (SIMDS * cyc)}
        if "SQ_WAVE_CYCLES" in m:
            e["wave_active_frac"] = m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]
        if "SQ_WAVES" in m and m.get("SQ_INSTS_VALU"):
            e["valu_insts_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
        out[k] = e
    return out


def main(argv) -> int:
    pairs = dict(a.split("=", 1) for a in argv) if argv else DEFAULT
    res = {}
    for cfg, p in pairs.items():
        ks = summarize(ROOT / p)
        # the dominant kernel: the longest
        main_k = max(ks, key=lambda k: ks[k]["dur_us"])
        res[cfg] = {"source": p, "kernel": main_k, **ks[main_k], "kernels": ks}
        print(f"{cfg}: {main_k[:70]} issue_frac {ks[main_k]['issue_frac']:.3f} "
              f"({ks[main_k]['dur_us']:.1f} us, {ks[main_k]['clock_ghz']:.2f} GHz)")
    out = ROOT / "profiles" / "valu.json"
    old = json.loads(out.read_text()) if out.exists() else {}
    old.update(res)
    out.write_text(json.dumps(old, indent=1) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
