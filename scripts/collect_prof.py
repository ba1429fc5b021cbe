"""Copy one gpu_profile.sh output directory into profiles/<round>/ under a key:
<key>_kernel_stats.csv (rocprofv3 --kernel-trace --stats), <key>_pmc_fetch.csv / <key>_pmc_write.csv (the two
--pmc passes) and <key>_summary.json (the profiles/traffic.json entry parse_prof.py wrote for the key).

usage: python scripts/collect_prof.py gpurun_out/prof_r04c_c5 r04 c5 [traffic-key]
"""
import glob
import json
import shutil
import sys
from pathlib import Path

src, rnd, key = Path(sys.argv[1]), sys.argv[2], sys.argv[3]
tkey = sys.argv[4] if len(sys.argv) > 4 else key
dst = Path("profiles") / rnd
dst.mkdir(parents=True, exist_ok=True)


def one(pattern):
    files = sorted(glob.glob(str(src / pattern), recursive=True))
    if not files:
        sys.exit(f"collect_prof: nothing matches {src / pattern}")
    return files[0]


shutil.copy(one("trace/**/*kernel_stats.csv"), dst / f"{key}_kernel_stats.csv")
shutil.copy(one("fetch/**/*counter_collection.csv"), dst / f"{key}_pmc_fetch.csv")
shutil.copy(one("write/**/*counter_collection.csv"), dst / f"{key}_pmc_write.csv")
traffic = json.loads(Path("profiles/traffic.json").read_text())
if tkey not in traffic:
    sys.exit(f"collect_prof: profiles/traffic.json has no entry {tkey!r}: run scripts/parse_prof.py first")
(dst / f"{key}_summary.json").write_text(json.dumps(traffic[tkey], indent=1) + "\n")
print(f"{src} -> {dst}/{key}_*")
