#!/bin/bash
# Session 3i: compile-time NT loads for non-overlapping power / top-k launches: full -m gpu suite + benches.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3i; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest_gpu.log | head -80; exit $rc; }
for cfg in north_star ns_topk c2 north_star; do
timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -5 $O/bench_$cfg.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_$cfg.json').read().strip().splitlines()[-1])
print('$cfg', '%.4f ms'%d['ms_per_step'], 'kernel %.4f'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'])"
done
timeout -k 10 120 fft-wavespec_amd/bin/kbench store 20 3 > $O/kbench_store.log 2>&1; tail -2 $O/kbench_store.log
