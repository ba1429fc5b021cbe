#!/bin/bash
# Copies one gpu_configs.sh run (tag) from gpurun_out/ into profiles/<round>/ and
# refreshes profiles/traffic.json from its PMC passes.
# Usage: bash scripts/collect_profiles.sh <tag> <round-dir>
set -eu
TAG=$1; DST=profiles/$2
mkdir -p $DST
for f in gpurun_out/bench_${TAG}_*.json; do
  cfg=${f#gpurun_out/bench_${TAG}_}; cfg=${cfg%.json}
  cp $f $DST/bench_$cfg.json
done
for d in gpurun_out/prof_${TAG}_*/; do
  cfg=${d#gpurun_out/prof_${TAG}_}; cfg=${cfg%/}
  cp $d/trace/run_kernel_stats.csv $DST/${cfg}_kernel_stats.csv
  for c in fetch write; do
    [ -f $d/$c/run_counter_collection.csv ] && cp $d/$c/run_counter_collection.csv $DST/${cfg}_pmc_$c.csv
  done
  python3 scripts/parse_prof.py $d $cfg > $DST/${cfg}_summary.json
done
