#!/bin/bash
# Session 2b: packed two-segment Kalman (check, parity, timing, C3 bench) + top-k/phase split exchange.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 120 fft-wavespec_amd/bin/kalman_bench check 4096 > $O/kalman_check_4096.log 2>&1 && timeout -k 10 120 fft-wavespec_amd/bin/kalman_bench check 1024 > $O/kalman_check_1024.log 2>&1 || { cat $O/kalman_check_*.log; exit 1; }
cat $O/kalman_check_1024.log | grep packed
cat $O/kalman_check_4096.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "kalman or topk or phase or c3" > $O/pytest_s2b.log 2>&1 || { tail -40 $O/pytest_s2b.log; exit 1; }
tail -2 $O/pytest_s2b.log
timeout -k 10 300 fft-wavespec_amd/bin/kalman_bench time 10 > $O/kalman_time.log 2>&1 || { cat $O/kalman_time.log; exit 1; }
cat $O/kalman_time.log
for c in c3; do
timeout -k 10 180 python3 bench.py --config $c --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_$c.json || exit 1
python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
