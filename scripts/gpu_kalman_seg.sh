#!/bin/bash
# Two-segment Kalman: correctness probe, timing ablation, parity tests, C3 bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02
O=gpurun_out/r02
timeout -k 10 60 fft-wavespec_amd/bin/kalman_bench check 256 > $O/kalman_check_256.log 2>&1 || { cat $O/kalman_check_256.log; exit 1; }
timeout -k 10 60 fft-wavespec_amd/bin/kalman_bench check 4096 > $O/kalman_check_4096.log 2>&1 || { cat $O/kalman_check_4096.log; exit 1; }
timeout -k 10 120 fft-wavespec_amd/bin/kalman_bench time 10 > $O/kalman_time_seg.log 2>&1 || { cat $O/kalman_time_seg.log; exit 1; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "kalman or c3" > $O/pytest_kalman.log 2>&1 || { tail -30 $O/pytest_kalman.log; exit 1; }
timeout -k 10 180 python3 bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_c3_seg.json || exit 1
cat $O/kalman_check_4096.log $O/kalman_time_seg.log; tail -2 $O/pytest_kalman.log; cat $O/bench_c3_seg.json
