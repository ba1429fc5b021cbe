#!/bin/bash
# bench.py per config (one JSON line each), then rocprofv3 passes per profiled config.
# Usage: bash scripts/gpu_configs.sh <tag> "<bench configs>" "<profiled configs>"
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
BENCH=${2:-"c2 c3 c4 c5 north_star"}
PROF=${3:-"c2 c3 c4"}
for CFG in $BENCH; do
  timeout -k 10 400 python bench.py --config $CFG --cpu-seconds 5 > gpurun_out/bench_${TAG}_$CFG.json 2> gpurun_out/bench_${TAG}_$CFG.err
  rc=$?; echo "$CFG rc=$rc"; cat gpurun_out/bench_${TAG}_$CFG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${TAG}_$CFG.err; exit $rc; }
done
for CFG in $PROF; do
  bash scripts/gpu_profile.sh $TAG $CFG > gpurun_out/prof_${TAG}_$CFG.summary 2>&1 || exit $?
done
