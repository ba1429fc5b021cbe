#!/bin/bash
# Session 2d: Kalman occupancy probe (pk2 vs pk4 by batch size), parity, C3 bench.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 200 fft-wavespec_amd/bin/kalman_bench occ 10 > $O/kalman_occ.log 2>&1 || { cat $O/kalman_occ.log; exit 1; }
cat $O/kalman_occ.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "kalman or c3" > $O/pytest_s2d.log 2>&1 || { tail -40 $O/pytest_s2d.log; exit 1; }
tail -2 $O/pytest_s2d.log
timeout -k 10 180 python3 bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_c3.json || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));print('c3', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
