#!/bin/bash
# Round-2 GPU pass: full GPU suite (parity metrics logged), latency, bench lines.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02
export WSP_PARITY_LOG=gpurun_out/r02/parity_metrics.json
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r02/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r02/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r02/pytest_gpu.log
timeout -k 10 120 python3 scripts/latency.py 4096 3000 > gpurun_out/r02/live_latency_4096.json || exit 1
timeout -k 10 120 python3 scripts/latency.py 1024 3000 > gpurun_out/r02/live_latency_1024.json || exit 1
timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02/bench_ns_20_5.json || exit 1
timeout -k 10 180 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r02/bench_ns_100_20.json || exit 1
cat gpurun_out/r02/bench_ns_20_5.json
