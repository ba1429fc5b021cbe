#!/bin/bash
# One GPU round: parity tests -> kernel ablation bench -> bench.py.
# Stops at the first step that faults / aborts / times out.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r1}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -x fft-wavespec_amd/bin/kbench ] && [ "${KBENCH:-0}" = 1 ]; then
  timeout -k 10 300 fft-wavespec_amd/bin/kbench 65536 20 2 > gpurun_out/kbench_$TAG.log 2>&1
  rc=$?; echo "kbench rc=$rc"; cat gpurun_out/kbench_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --cpu-seconds 10 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
exit $rc
