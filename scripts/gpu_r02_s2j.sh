#!/bin/bash
# Session 2j: C5 stream layouts interleaved on one box.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02e; mkdir -p $O
for rep in 1 2; do for lay in length greedy; do
C5_LAYOUT=$lay timeout -k 10 180 python3 bench.py --config c5 --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_c5_$lay.json || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c5_$lay.json'));print('c5 $lay', d['ms_per_step'], d['roofline']['frac'])"
done; done
