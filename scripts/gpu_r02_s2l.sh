#!/bin/bash
# Session 2l: fp32 spectrum at 4 waves/SIMD: f32 parity, C3 step + kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02g; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "f32 or c3 or sizes_hann or kalman" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 180 python3 bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_c3.json || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));print('c3', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o run -- python3 bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline > $O/trace_c3.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('$O/trace_c3/run_kernel_stats.csv')):
    if 'spectrum' in r['Name'] or 'kalman' in r['Name']: print(r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3)"
