#!/bin/bash
# Session 3h: north star -- compile-time vs run-time nt loads (kbench store mode) + bench.py on the same box.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3h; mkdir -p $O
timeout -k 10 120 fft-wavespec_amd/bin/kbench store 20 4 > $O/kbench_store.log 2>&1 || { cat $O/kbench_store.log; exit 1; }
cat $O/kbench_store.log
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_ns.json 2> $O/bench_ns.err || { tail -5 $O/bench_ns.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_ns.json').read().strip().splitlines()[-1])
print('ns', '%.4f ms'%d['ms_per_step'], 'kernel %.4f'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'])"
