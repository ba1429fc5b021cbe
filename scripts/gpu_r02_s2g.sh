#!/bin/bash
# Session 2g: rotated tile loop of the packed Kalman (vmcnt only for the loads): check, parity, timing, C3.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02c; mkdir -p $O
timeout -k 10 120 fft-wavespec_amd/bin/kalman_bench check 4096 > $O/kalman_check_4096.log 2>&1 && timeout -k 10 120 fft-wavespec_amd/bin/kalman_bench check 1024 > $O/kalman_check_1024.log 2>&1 || { cat $O/kalman_check_*.log; exit 1; }
grep packed $O/kalman_check_4096.log $O/kalman_check_1024.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "kalman or c3 or register or pinned" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 fft-wavespec_amd/bin/kalman_bench time 10 > $O/kalman_time.log 2>&1 || { cat $O/kalman_time.log; exit 1; }
grep -E "round|packed|4-wave WG \+ 1 WG/CU, static, packed" $O/kalman_time.log
timeout -k 10 180 python3 bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_c3.json || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));print('c3', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
